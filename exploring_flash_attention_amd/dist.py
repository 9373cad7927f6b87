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
     once (a ring reduce-scatter would serialise on one link per step);
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


def shard_bounds(L, world, rank):
    """Key range [lo, hi) of rank's shard (equal shards; L % world == 0)."""
    if L % world:
        raise ValueError(f"L={L} must be divisible by world size {world}")
    n = L // world
    return rank * n, (rank + 1) * n


def splitkv_attention(q, k_shard, v_shard, group=None, partial_dtype=torch.bfloat16,
                      gather=False):
    """Sharded split-KV forward.

    q: [B, H, L, d] (identical on every rank); k_shard / v_shard: this rank's keys
    [B, H, L/W, d].  Returns this rank's query rows [B, H, L/W, d] of O, or the full
    [B, H, L, d] O when ``gather``.
    """
    world = dist.get_world_size(group)
    B, H, L, d = q.shape
    if L % world:
        raise ValueError(f"L={L} must be divisible by world size {world}")
    Lc = L // world
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
