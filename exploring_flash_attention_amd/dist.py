"""Split-KV forward sharded over the GPUs of one node (one process per GPU, RCCL over xGMI).

The reference has no multi-GPU code; its only sequence-scaling mechanism is the
single-GPU split-KV pair partial_attention_kernel + reduction_kernel
(flash_attention_v2/CUDA/flash_attention_v2.h:243, :356).  Here the KV splits become GPU
shards and the one real exchange of the algorithm -- every query row needs the partial
results of every key shard -- is an all-to-all:

  rank r holds the full Q [B, H, L, d] and its key shard K_r, V_r [B, H, L/W, d]
  1. partial kernel over its keys, writing (O_r normalised, lse_r) in the all-to-all
     SEND layout [W][B*H][L/W][d]: chunk j = the query rows rank j will own;
  2. all_to_all_single of O (bf16 by default) and lse (fp32): each rank sends W-1 of its
     W chunks straight to their owners, so all 7 xGMI links of a rank carry traffic at
     once (a ring reduce-scatter would serialise on one link per step).  By default steps
     1-2 are pipelined instead: one partial kernel per destination chunk, each chunk sent
     (pairwise send/recv, a shifted exchange) while the next one computes;
  3. combine kernel on the received [W][B*H][L/W][d] = the W partials of rank r's query
     rows -> O rows [r*L/W, (r+1)*L/W) of every head;
  4. optionally all_gather to a replicated O.

The per-rank compute and exchange functions are module attributes so the exchange logic
can be exercised on CPU with the gloo backend in tests (the kernels need the GPU).
"""
import torch
import torch.distributed as dist

from . import ops


def _partial_fn(q, k, v, chunk_rows, partial_dtype):
    return ops.attention_partial(q, k, v, chunk_rows=chunk_rows, partial_dtype=partial_dtype)


def _combine_fn(o_part, lse, B, H, dtype):
    return ops.combine(o_part, lse, B, H, dtype)


def _partial_chunk_fn(q_rows, k, v, o_out, lse_out, partial_dtype):
    """Partials of one chunk of query rows: q_rows a [B, H, Lc, d] row range of q (a view,
    addressed in place), results into o_out [B*H, Lc, d] and lse_out [B*H, Lc] ([B*H, Lc, 2]
    for scaled partials)."""
    ops.attention_partial(q_rows, k, v, partial_dtype=partial_dtype, o_part=o_out[None], lse=lse_out[None])


def shard_bounds(L, world, rank):
    """Key range [lo, hi) of rank's shard (equal shards; L % world == 0)."""
    if L % world:
        raise ValueError(f"L={L} must be divisible by world size {world}")
    n = L // world
    return rank * n, (rank + 1) * n


def _peer(group, r):
    return dist.get_global_rank(group, r) if group is not None else r


def _chunk_ops(o_send, lse_send, o_recv, lse_recv, group, rank, world, s):
    """Step s of the shifted exchange: send chunk rank+s to rank+s, receive chunk rank from
    rank-s (every step a perfect matching: all ranks' links busy at once)."""
    dst, src = (rank + s) % world, (rank - s) % world
    return [dist.P2POp(dist.isend, o_send[dst], _peer(group, dst), group),
            dist.P2POp(dist.irecv, o_recv[src], _peer(group, src), group),
            dist.P2POp(dist.isend, lse_send[dst], _peer(group, dst), group),
            dist.P2POp(dist.irecv, lse_recv[src], _peer(group, src), group)]


def exchange_partials(o_send, lse_send, o_recv, lse_recv, group=None):
    """The exchange step alone, on partials already computed in the send layout
    ([W][B*H][L/W][d] and their lse): chunk j goes to rank j over W-1 shifted send/recv steps
    posted together; the own chunk is copied locally (it never crosses a link).  Returns the
    RCCL works (wait() them, or let the stream order the next kernel).  bench.py times it to
    report the xGMI exchange separately from the kernels."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ops_ = []
    for s in range(1, world):
        ops_ += _chunk_ops(o_send, lse_send, o_recv, lse_recv, group, rank, world, s)
    o_recv[rank].copy_(o_send[rank])
    lse_recv[rank].copy_(lse_send[rank])
    return dist.batch_isend_irecv(ops_) if ops_ else []


def _exchange_overlapped(q, k_shard, v_shard, group, partial_dtype, world, Lc):
    """Steps 1-2 pipelined: the partials are computed one destination chunk at a time, and
    chunk j is handed to RCCL (send to rank j, matched receive from the rank sending to us)
    as soon as its kernel is queued, so its transfer overlaps the next chunk's kernel.  Step s
    pairs rank r -> r+s with r-s -> r (a shifted exchange: every step a perfect matching, all
    ranks' links busy at once); the own chunk is computed last, straight into the receive
    buffer.  RCCL waits on the compute stream at each send; the compute stream never waits
    for RCCL until the combine."""
    B, H, _, d = q.shape
    rank = dist.get_rank(group)
    lse_dtype = torch.float64 if q.dtype == torch.float64 else torch.float32
    scaled = partial_dtype == ops.PARTIAL_FP16_SCALED  # fp16 rows, {lse, exponent} per row
    o_send = torch.empty((world, B * H, Lc, d), dtype=torch.float16 if scaled else partial_dtype,
                         device=q.device)
    lse_send = torch.empty((world, B * H, Lc) + ((2,) if scaled else ()), dtype=lse_dtype, device=q.device)
    o_recv, lse_recv = torch.empty_like(o_send), torch.empty_like(lse_send)

    works = []
    for s in range(1, world):
        dst = (rank + s) % world
        _partial_chunk_fn(q[:, :, dst * Lc:(dst + 1) * Lc], k_shard, v_shard, o_send[dst], lse_send[dst],
                          partial_dtype)
        works += dist.batch_isend_irecv(_chunk_ops(o_send, lse_send, o_recv, lse_recv, group, rank, world, s))
    _partial_chunk_fn(q[:, :, rank * Lc:(rank + 1) * Lc], k_shard, v_shard, o_recv[rank], lse_recv[rank],
                      partial_dtype)
    for w in works:
        w.wait()
    return o_recv, lse_recv


def _uses_rccl(group):
    """True when the group moves device tensors over RCCL: its backend is "nccl", or a
    mixed-backend group ("cpu:gloo,cuda:nccl") whose device half is."""
    b = str(dist.get_backend(group))
    return b == "nccl" or "cuda:nccl" in b


def splitkv_attention(q, k_shard, v_shard, group=None, partial_dtype=None,
                      gather=False, overlap=True):
    """Sharded split-KV forward.

    q: [B, H, L, d] (identical on every rank); k_shard / v_shard: this rank's keys
    [B, H, L/W, d].  Returns this rank's query rows [B, H, L/W, d] of O, or the full
    [B, H, L, d] O when ``gather``.  ``overlap`` (W > 1): per-destination partial kernels
    pipelined with pairwise send/recv (_exchange_overlapped); otherwise one partial kernel
    over all rows, then all_to_all_single.  ``partial_dtype`` (the format sent over xGMI):
    default per-row scaled fp16 (ops.PARTIAL_FP16_SCALED) -- the bytes of bf16 partials with
    3 more significant bits; fp64 for fp64 inputs.
    """
    if partial_dtype is None:
        partial_dtype = torch.float64 if q.dtype == torch.float64 else ops.PARTIAL_FP16_SCALED
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    B, H, L, d = q.shape
    if L % world:
        raise ValueError(f"L={L} must be divisible by world size {world}")
    Lc = L // world
    if world > 1 and overlap and q.is_cuda and not _uses_rccl(group):
        # gloo's send/recv take host memory only (its all_to_all / all_gather stage device
        # tensors): device tensors on a non-RCCL group take the all-to-all path
        overlap = False
    if world > 1 and overlap:
        o_recv, lse_recv = _exchange_overlapped(q, k_shard, v_shard, group, partial_dtype, world, Lc)
        o_local = _combine_fn(o_recv, lse_recv, B, H, q.dtype)
        if not gather:
            return o_local
        parts = [torch.empty_like(o_local) for _ in range(world)]
        dist.all_gather(parts, o_local.contiguous(), group=group)
        return torch.cat(parts, dim=2)
    o_part, lse = _partial_fn(q, k_shard, v_shard, Lc, partial_dtype)  # [W, BH, Lc, d], [W, BH, Lc]
    if world > 1:
        o_recv = torch.empty_like(o_part)
        lse_recv = torch.empty_like(lse)
        dist.all_to_all_single(o_recv, o_part, group=group)
        dist.all_to_all_single(lse_recv, lse, group=group)
    else:
        o_recv, lse_recv = o_part, lse
    o_local = _combine_fn(o_recv, lse_recv, B, H, q.dtype)  # [B, H, Lc, d]
    if not gather:
        return o_local
    if world == 1:
        return o_local
    parts = [torch.empty_like(o_local) for _ in range(world)]
    dist.all_gather(parts, o_local.contiguous(), group=group)
    return torch.cat(parts, dim=2)


# ----------------------------------------------------------------------------------------
# the same forward through the native C ABI (include/fa_mi355x_dist.h): one RCCL
# communicator owned by libfa_mi355x_dist.so, the whole sequence issued from C++
# ----------------------------------------------------------------------------------------

_dist_lib = None


def dist_lib():
    """ctypes handle of libfa_mi355x_dist.so (loaded on first use; raises if not built)."""
    global _dist_lib
    if _dist_lib is None:
        import ctypes
        import os

        from . import _lib
        path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libfa_mi355x_dist.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: build it with `python __graft_entry__.py`")
        _lib.lib()  # the core library first (the dist library links it)
        h = ctypes.CDLL(path)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        for name, res, args in (
                ("fa_dist_last_error", ctypes.c_char_p, []),
                ("fa_dist_get_unique_id", I, [P]),
                ("fa_dist_comm_init", I, [ctypes.POINTER(P), I, I, P]),
                ("fa_dist_comm_destroy", I, [P]),
                ("fa_fwd_v2_dist_workspace_size", I, [I64, I64, I64, I64, I, I, I,
                                                      ctypes.POINTER(ctypes.c_size_t)]),
                ("fa_fwd_v2_dist", I, [P, P, P, P, I64, I64, I64, I64, P, I, P, ctypes.c_size_t,
                                       I, I, P])):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
        _dist_lib = h
    return _dist_lib


def _dcheck(st):
    if st:
        from ._lib import FaError
        raise FaError(st, dist_lib().fa_dist_last_error().decode())


class RcclComm:
    """An RCCL communicator of libfa_mi355x_dist.so over the ranks of ``group``.

    The 128-byte RCCL id is created on rank 0 and broadcast with torch.distributed (any
    backend); with no process group initialised the communicator has one rank.
    """

    def __init__(self, group=None):
        import ctypes
        lib = dist_lib()
        if dist.is_available() and dist.is_initialized():
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self.world, self.rank = 1, 0
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            _dcheck(lib.fa_dist_get_unique_id(uid))
        if self.world > 1:
            box = [bytes(uid.raw)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group else 0, group=group)
            uid = ctypes.create_string_buffer(box[0], 128)
        self._comm = ctypes.c_void_p()
        _dcheck(lib.fa_dist_comm_init(ctypes.byref(self._comm), self.world, self.rank, uid))

    @property
    def handle(self):
        return self._comm

    def close(self):
        if self._comm:
            _dcheck(dist_lib().fa_dist_comm_destroy(self._comm))
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def splitkv_attention_native(q, k_shard, v_shard, comm, gather=False, partial_dtype=None,
                             workspace=None):
    """``splitkv_attention`` through the C ABI (fa_fwd_v2_dist): partial kernel, one grouped
    RCCL send/recv round, combine kernel (and all-gather), all on the current stream."""
    import ctypes
    ops._check_qkv(q, k_shard, v_shard, same_len=False)
    B, H, L, d = q.shape
    W = comm.world
    if L % W or k_shard.shape[2] * W != L:
        raise ValueError(f"L={L} must be divisible by world {W} and k_shard must hold L/W keys")
    # per-row scaled fp16 partials by default, as splitkv_attention (fp64 for fp64 inputs)
    if partial_dtype is None:
        partial_dtype = torch.float64 if q.dtype == torch.float64 else ops.PARTIAL_FP16_SCALED
    pd = partial_dtype
    nbytes = ctypes.c_size_t()
    _dcheck(dist_lib().fa_fwd_v2_dist_workspace_size(B, H, L, d, W, ops._DTYPES[q.dtype],
                                                     ops._PDTYPES[pd], ctypes.byref(nbytes)))
    if workspace is None:
        workspace = torch.empty(nbytes.value, dtype=torch.uint8, device=q.device)
    out = torch.empty((B, H, L if gather else L // W, d), dtype=q.dtype, device=q.device)
    _dcheck(dist_lib().fa_fwd_v2_dist(ops._ptr(q), ops._ptr(k_shard), ops._ptr(v_shard), ops._ptr(out),
                                      B, H, L, d, comm.handle, int(bool(gather)), ops._ptr(workspace),
                                      workspace.numel(), ops._DTYPES[q.dtype], ops._PDTYPES[pd],
                                      ops._stream(q)))
    return out
