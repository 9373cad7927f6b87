"""Full-size parity at the BASELINE configs -- the shapes bench.py times.

The reference drivers compare the GPU output against the CPU oracle at the benchmarked size
on every run (flash_attention_v1/CUDA/driver.cu:140-143 and PASS at :275,
flash_attention_v1_tiled_d/CUDA/driver.cu:120-125 and :250, flash_attention_v2/CUDA/
driver.cu:87-90 and :204).  Here:

* C2 / C3 (B32 H8 L1024, d = 32 / 128) and C4 (B32 H8 L4096 d128, KV_TILES_PER_BLOCK = 4:
  as scheduled, and with 16 / 4 partials per query tile through the in-kernel combine with
  scaled fp16 partials, and the automatic split) on N(0,1) bf16 inputs, against the fp64 oracle on 16 sampled heads -- the first
  and last (b, h) included, every query tile of each, so the 2048-workgroup XCD remap, all
  8 (32 at C4) query tiles of a head and the 16-split combine are all covered;
* the drivers' own inputs (srand(42) U[-1,1] fp16, oracle_driver_random) at B32 H8 L1024
  against the C restatement of standard_attention_cpu over ALL 256 heads, with the drivers'
  PASS thresholds: v1 max_abs < 1e-3, tiled-d max_abs < 1e-2, v2 max_abs and max_rel
  (|ref| > 1e-3) < 0.1;
* PyTorch SDPA (the reference's flash_attention_v1/pytorch_imp.py:12) beside the kernel at
  C3, both against the fp64 oracle.
"""
import numpy as np
import pytest
import torch

from oracle.batched import attention_fp64
from test_gpu import _gate

pytestmark = pytest.mark.gpu

B, H = 32, 8


def _sample(n=16):
    idx = sorted({round(i * (B * H - 1) / (n - 1)) for i in range(n)})
    return [(i // H, i % H) for i in idx]


def _device_inputs(L, d, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3)]


def _check_sampled(out, q, k, v, label=None):
    """The gates of test_gpu on the sampled heads (fp64 oracle on the same bf16 inputs); with a
    label, the elements over the waived bf16 max_rel gate are recorded (test_gpu.MAXREL_WAIVER)."""
    assert bool(torch.isfinite(out).all())
    heads = _sample()
    pick = lambda t: torch.stack([t[b, h] for b, h in heads])[None].cpu()  # [1, 16, L, d]
    qs, ks, vs, os_ = (pick(t) for t in (q, k, v, out))
    ref = attention_fp64(qs.double().numpy(), ks.double().numpy(), vs.double().numpy())
    return _gate(os_, ref, torch.bfloat16, label=label)


@pytest.mark.parametrize("d", [32, 128], ids=["C2", "C3"])
def test_fullsize_v1_and_tiled_d(gpu, d):
    from exploring_flash_attention_amd import ops
    q, k, v = _device_inputs(1024, d, seed=d)
    name = {32: "C2", 128: "C3"}[d]
    _check_sampled(ops.attention_v1(q, k, v), q, k, v, label=f"fullsize {name} v1 (16 heads)")
    _check_sampled(ops.attention_tiled_d(q, k, v, 32, 32), q, k, v, label=f"fullsize {name} tiled-d (16 heads)")


@pytest.mark.parametrize("kvt,group", [(4, None), (4, 1), (4, 4), ("auto", None)],
                         ids=["kvtpb4", "kvtpb4-one-wg-per-block", "kvtpb4-4-per-wg", "auto"])
def test_fullsize_c4_splitkv(gpu, kvt, group):
    """C4 as scheduled (the 16 key blocks of a query tile on one workgroup), and with
    blocks_per_workgroup fixing 1 or 4 blocks per workgroup: 16 / 4 partials per query tile
    through the workspace and the in-kernel combine (8192 query tiles)."""
    from exploring_flash_attention_amd import ops
    q, k, v = _device_inputs(4096, 128, seed=4)
    nbytes, ns = ops.v2_workspace_bytes(B, H, 4096, 128, kvt, blocks_per_workgroup=group)
    blocks, per_wg, partials = ops.v2_split_plan(B, H, 4096, 128, kvt, blocks_per_workgroup=group)
    if kvt == 4:
        assert ns == blocks == 16 and partials == 16 // int(group or 16)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    o1 = ops.attention_v2(q, k, v, kvt, workspace=ws, blocks_per_workgroup=group)
    o2 = ops.attention_v2(q, k, v, kvt, workspace=ws, blocks_per_workgroup=group)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)  # the combine order is fixed: bitwise repeatable
    _check_sampled(o1, q, k, v, label=f"fullsize C4 kvtpb={kvt} group={group} (16 heads)")


def _driver_inputs(oracle_lib, L, d):
    """initialize_random of the CUDA drivers after srand(42): Q, K, V in that order, fp16."""
    n = B * H * L * d
    buf = np.empty(3 * n, np.float32)
    oracle_lib.oracle_driver_random(buf.ctypes.data, 3 * n, 42, 1)
    x = buf.astype(np.float16)
    return [x[i * n:(i + 1) * n].reshape(B, H, L, d) for i in range(3)]


def _c_reference(oracle_lib, Q, K, V):
    """standard_attention_cpu (C restatement, OpenMP over heads, fp32 math, fp16 output)."""
    Q, K, V = (np.ascontiguousarray(x) for x in (Q, K, V))
    O = np.empty_like(Q)
    b, h, L, d = Q.shape
    oracle_lib.oracle_standard_attention(Q.ctypes.data, K.ctypes.data, V.ctypes.data, O.ctypes.data,
                                         b, h, L, d, 0)
    return O.astype(np.float32)


def _driver_metrics(out, ref):
    """compare_arrays of flash_attention_v2/CUDA/driver.cu:46-80 (eps = 1e-3 for fp16)."""
    diff = np.abs(out - ref)
    big = np.abs(ref) > 1e-3
    return float(diff.max()), float((diff[big] / np.abs(ref[big])).max())


@pytest.mark.parametrize("group", [None, 1, 2], ids=["as-scheduled", "one-wg-per-block", "2-per-wg"])
@pytest.mark.parametrize("d", [32, 128])
def test_driver_compare_full_size(gpu, oracle_lib, d, group):
    """The drivers' own inputs and PASS thresholds at B32 H8 L1024 over all 256 heads.  The
    library schedules L = 1024 with KV_TILES_PER_BLOCK = 4 on the FA-v1 kernel (4 key blocks,
    one workgroup per query tile); blocks_per_workgroup = 1 / 2 forces the split-KV partials
    (4 / 2 per query tile) through the workspace and the in-kernel combine, so the v2
    driver's thresholds cover the combine too."""
    from exploring_flash_attention_amd import ops
    Q, K, V = _driver_inputs(oracle_lib, 1024, d)
    ref = _c_reference(oracle_lib, Q, K, V)
    q, k, v = (torch.from_numpy(x).to(gpu) for x in (Q, K, V))
    if group is None:
        o1 = ops.attention_v1(q, k, v).float().cpu().numpy()
        ot = ops.attention_tiled_d(q, k, v, 32, 32).float().cpu().numpy()
        ma1, _ = _driver_metrics(o1, ref)
        mat, _ = _driver_metrics(ot, ref)
        assert ma1 < 1e-3, ma1             # flash_attention_v1/CUDA/driver.cu:275
        assert mat < 1e-2, mat             # flash_attention_v1_tiled_d/CUDA/driver.cu:250
    _, _, partials = ops.v2_split_plan(B, H, 1024, d, 4, q.dtype, blocks_per_workgroup=group)
    assert partials == {None: 1, 1: 4, 2: 2}[group]
    o2 = ops.attention_v2(q, k, v, 4, blocks_per_workgroup=group).float().cpu().numpy()
    ma2, mr2 = _driver_metrics(o2, ref)
    assert ma2 < 0.1 and mr2 < 0.1, (ma2, mr2)  # flash_attention_v2/CUDA/driver.cu:204
    assert ma2 < 1e-3, ma2             # and the stricter v1 bound, which the split path also meets


@pytest.mark.parametrize("group", [None, 1], ids=["as-scheduled", "16-partials"])
def test_driver_inputs_c4_sampled(gpu, oracle_lib, group):
    """C4's shape (L = 4096, KV_TILES_PER_BLOCK = 4: 16 key blocks) on the drivers' generator,
    against the C oracle on the 16 sampled heads (the whole batch would take the C oracle
    ~30 s): as scheduled (one workgroup per query tile) and with one workgroup per key block
    (16 partials per query tile through the in-kernel combine)."""
    from exploring_flash_attention_amd import ops
    Q, K, V = _driver_inputs(oracle_lib, 4096, 128)
    q, k, v = (torch.from_numpy(x).to(gpu) for x in (Q, K, V))
    _, _, partials = ops.v2_split_plan(B, H, 4096, 128, 4, q.dtype, blocks_per_workgroup=group)
    assert partials == (16 if group == 1 else 1)
    out = ops.attention_v2(q, k, v, 4, blocks_per_workgroup=group).float().cpu().numpy()
    heads = _sample()
    pick = lambda x: np.stack([x[b, h] for b, h in heads])[None]
    ref = _c_reference(oracle_lib, pick(Q), pick(K), pick(V))
    ma, mr = _driver_metrics(pick(out), ref)
    assert ma < 1e-3 and mr < 0.1, (ma, mr)


def test_sdpa_crosscheck_c3(gpu):
    """torch SDPA (the reference's pytorch_imp.py path) and the kernel at C3 on the same bf16
    inputs: both within the bf16 gates of the fp64 oracle, and within two gates of each other."""
    import torch.nn.functional as F
    from exploring_flash_attention_amd import ops
    q, k, v = _device_inputs(1024, 128, seed=3)
    ours = ops.attention_v1(q, k, v)
    sdpa = F.scaled_dot_product_attention(q, k, v)
    m_ours = _check_sampled(ours, q, k, v)
    m_sdpa = _check_sampled(sdpa, q, k, v)
    assert float((ours.float() - sdpa.float()).abs().max()) <= 2 * 6e-3
    # no worse than the library reference beyond a bf16 rounding step
    assert m_ours["max_abs"] <= max(6e-3, 1.5 * m_sdpa["max_abs"]), (m_ours, m_sdpa)


def test_fullsize_c5_splitkv_emulated_w8(gpu):
    """C5 -- B32 H8 L16384 d128, the keys sharded over W = 8 ranks -- at its full per-rank
    size on ONE GPU, every rank's kernels run in turn:

    * rank p (key shard p) computes its scaled-fp16 partials one destination chunk at a time
      from row-range views of q, exactly as the overlapped exchange does
      (dist._exchange_overlapped -> dist._partial_chunk_fn), and the chunks are placed where
      the exchange delivers them: rank j's receive buffer [W][B*H][L/W][d], slot p;
    * each shard's chunks are bitwise equal to the all-to-all form's one-launch partial in the
      send layout (dist._partial_fn, overlap=False), so both exchanges hand the combine the
      same bytes;
    * rank j's combine (dist._combine_fn, the reduction of
      flash_attention_v2/CUDA/flash_attention_v2.h:356-435 over the 8 shards) gives its query
      rows; sampled heads (first and last included) x 32 sampled rows of EVERY rank's chunk
      (first and last rows included) against the fp64 oracle.
    The RCCL transfer itself is covered by test_gpu_multirank.py (one GPU per rank)."""
    from exploring_flash_attention_amd import dist as fdist
    from exploring_flash_attention_amd import ops
    W, L, d = 8, 16384, 128
    Lc = L // W
    q, k, v = _device_inputs(L, d, seed=5)
    fp16s = ops.PARTIAL_FP16_SCALED
    o_recv = torch.empty((W, W, B * H, Lc, d), dtype=torch.float16, device=gpu)  # [rank j][from p]
    lse_recv = torch.empty((W, W, B * H, Lc, 2), dtype=torch.float32, device=gpu)
    for p in range(W):
        ks = k[:, :, p * Lc:(p + 1) * Lc].contiguous()
        vs = v[:, :, p * Lc:(p + 1) * Lc].contiguous()
        for j in range(W):
            fdist._partial_chunk_fn(q[:, :, j * Lc:(j + 1) * Lc], ks, vs, o_recv[j, p], lse_recv[j, p], fp16s)
        o_a2a, lse_a2a = fdist._partial_fn(q, ks, vs, Lc, fp16s)  # [W][B*H][Lc][d] send layout
        torch.cuda.synchronize()
        assert torch.equal(o_a2a, o_recv[:, p]) and torch.equal(lse_a2a, lse_recv[:, p]), p
        del ks, vs, o_a2a, lse_a2a
    rows = sorted({j * Lc + round(i * (Lc - 1) / 31) for j in range(W) for i in range(32)})
    picked = []
    for j in range(W):
        oj = fdist._combine_fn(o_recv[j], lse_recv[j], B, H, q.dtype)  # [B, H, Lc, d]
        assert oj.shape == (B, H, Lc, d) and oj.dtype == q.dtype
        picked.append(oj[:, :, [r - j * Lc for r in rows if j * Lc <= r < (j + 1) * Lc]])
    torch.cuda.synchronize()
    del o_recv, lse_recv
    out_rows = torch.cat(picked, dim=2)  # [B, H, len(rows), d]
    assert bool(torch.isfinite(out_rows).all())
    heads = _sample()
    pick = lambda t: torch.stack([t[b, h] for b, h in heads])[None].cpu()
    qs = pick(q[:, :, rows])
    ks, vs, os_ = pick(k), pick(v), pick(out_rows)
    ref = attention_fp64(qs.double().numpy(), ks.double().numpy(), vs.double().numpy())
    _gate(os_, ref, torch.bfloat16, label="fullsize C5 W=8 emulated (16 heads x 256 rows)")


@pytest.mark.parametrize("B,H,L", [(4, 16, 1024), (5, 13, 1024), (64, 8, 256), (2, 17, 2048), (8, 33, 512)],
                         ids=["512-items", "520-items-uneven", "ntiles4", "l2048-uneven", "l512-uneven"])
def test_chain_kernel_shapes(gpu, B, H, L):
    """The chained persistent d = 128 kernel (fa_fwd16_chain.hpp: at least as many query tiles as
    a 2-per-CU grid, Lk a multiple of 128 and >= 256) on shapes around its launch conditions:
    exactly one workgroup per query tile, uneven item lists, the shortest chain (4 tiles), a
    partial item count per XCD group -- sampled heads (first and last included, every query tile
    of each) against the fp64 oracle, and bitwise repeatable."""
    from exploring_flash_attention_amd import ops
    d = 128
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + H * 10 + L)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o1 = ops.attention_v1(q, k, v)
    o2 = ops.attention_v1(q, k, v)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    n = min(12, B * H)
    idx = sorted({round(i * (B * H - 1) / (n - 1)) for i in range(n)})
    pick = lambda t: t.reshape(B * H, L, d)[idx][None].cpu()
    ref = attention_fp64(pick(q).double().numpy(), pick(k).double().numpy(), pick(v).double().numpy())
    _gate(pick(o1), ref, torch.bfloat16)


@pytest.mark.parametrize("shape,kvt,group,partials", [
    ((1, 1, 16384), 4, None, 4),        # one-shot grid, 4 blocks of 4096 keys: arrival-first hand-off
    ((1, 2, 4096), 4, None, 4),         # one-shot grid, store-first hand-off, one-batch combine
    ((2, 2, 16384), 4, 4, 16),          # the chained walk (512 tiles), 16 partials: two-pass combine
    ((1, 8, 16384), 4, 16, 4),          # the walk at 4 partials of 4096 keys: one-batch combine
    ((1, 3, 16384), 4, None, 2),        # one-shot, arrival first, 768 workgroups: some queued
], ids=["b1h1-l16k", "b1h2-l4k", "b2h2-l16k-walk16", "b1h8-l16k-walk4", "b1h3-l16k-queued"])
def test_long_sequence_split_paths(gpu, shape, kvt, group, partials):
    """The split-KV schedules of the low-parallelism shapes (the bench extras and the chained
    walk) against the fp64 oracle on 512 sampled query rows of every head -- first and last
    rows, every query tile -- with the full key range; bitwise repeatable across two launches
    on a reused workspace (the counters left at zero)."""
    from exploring_flash_attention_amd import ops
    b, h, L = shape
    g = torch.Generator(device="cuda").manual_seed(L + h)
    q, k, v = (torch.randn(b, h, L, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    _, _, parts = ops.v2_split_plan(b, h, L, 128, kvt, q.dtype, blocks_per_workgroup=group)
    assert parts == partials, parts
    nbytes, _ = ops.v2_workspace_bytes(b, h, L, 128, kvt, blocks_per_workgroup=group)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    o1 = ops.attention_v2(q, k, v, kvt, workspace=ws, blocks_per_workgroup=group)
    o2 = ops.attention_v2(q, k, v, kvt, workspace=ws, blocks_per_workgroup=group)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    rows = torch.tensor(sorted({round(i * (L - 1) / 511) for i in range(512)}), device=gpu)
    qs = q[:, :, rows].cpu().double().numpy()
    ref = attention_fp64(qs, k.cpu().double().numpy(), v.cpu().double().numpy())
    _gate(o1[:, :, rows].cpu(), ref, torch.bfloat16, label=f"long split B{b} H{h} L{L} ({partials} partials)")


def test_launched_kernels_reported(gpu):
    """fa_last_kernels (ops.launched_kernels): each operator reports the kernel and grid the
    library's launcher picked -- the chained persistent grid of exactly 2 workgroups per CU at
    C3-like shapes, the one-shot grid below it, the 32x32x16 kernel for d = 32 and key tails,
    the fused split-KV kernel, the d-tiled kernel, and partial + combine."""
    from exploring_flash_attention_amd import ops
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    grid = 2 * cus // 8 * 8

    def run(fn, *shape, dtype=torch.bfloat16):
        B, H, L, d = shape
        q, k, v = (torch.randn(B, H, L, d, device=gpu, dtype=dtype) for _ in range(3))
        with ops.launched_kernels() as kl:
            fn(q, k, v)
        torch.cuda.synchronize()
        return kl

    tiles = grid  # a C3-like shape with exactly one query tile per workgroup of the grid
    assert run(ops.attention_v1, 1, tiles // 8, 1024, 128) == [f"fa_fwd16_chain_kernel<final> [grid {grid}]"]
    assert run(ops.attention_v1, 1, 2, 1024, 128) == ["fa_fwd16_kernel<final> [grid 16]"]
    assert run(ops.attention_v1, 2, 2, 1024, 32) == ["fa_fwd_kernel<final> [grid 32]"]
    assert run(ops.attention_v1, 1, 2, 1000, 128) == ["fa_fwd_kernel<final> [grid 16]"]
    assert run(lambda q, k, v: ops.attention_tiled_d(q, k, v, 64, 64), 1, 2, 256, 384) == ["fa_fwd_dt_kernel [grid 8]"]
    assert run(lambda q, k, v: ops.attention_tiled_d(q, k, v, 64, 64), 1, 2, 256, 512) == ["fa_fwd_dt_kernel<paired> [grid 8]"]
    kl = run(lambda q, k, v: ops.attention_v2(q, k, v, 4), 1, 2, 4096, 128)
    assert len(kl) == 1 and kl[0].startswith("fa_fwd16_kernel<fused split, in-kernel combine> [grid ")
    with ops.launched_kernels() as kl:
        q, k, v = (torch.randn(1, 2, 512, 128, device=gpu, dtype=torch.bfloat16) for _ in range(3))
        o_part, lse = ops.attention_partial(q, k, v)
        ops.combine(o_part, lse, 1, 2, torch.bfloat16)
    torch.cuda.synchronize()
    assert kl[0] == "fa_fwd16_kernel<partial> [grid 8]" and kl[1].startswith("fa_combine_kernel [grid ")


@pytest.mark.parametrize("shape,kvt", [((1, 2, 4096), 4), ((1, 1, 16384), 4)], ids=["store-first", "arrive-first"])
def test_v2_zeroed_workspace_skips_reset(gpu, shape, kvt):
    """attention_v2(workspace_zeroed=True) (fa_fwd_v2_ex2, FA_V2_COUNTERS_ZERO): no counter
    reset between calls on a workspace zeroed once -- every launch leaves its counters zero, so
    repeated calls stay bitwise equal to the resetting path, for the store-first and the
    arrival-first hand-offs; the launch list holds the kernel only."""
    from exploring_flash_attention_amd import ops
    b, h, L = shape
    g = torch.Generator(device="cuda").manual_seed(L + 7)
    q, k, v = (torch.randn(b, h, L, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    nbytes, _ = ops.v2_workspace_bytes(b, h, L, 128, kvt)
    ws0 = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    ref = ops.attention_v2(q, k, v, kvt, workspace=ws0)
    ws = torch.zeros(nbytes, dtype=torch.uint8, device=gpu)
    outs = []
    for _ in range(3):
        with ops.launched_kernels() as kl:
            outs.append(ops.attention_v2(q, k, v, kvt, workspace=ws, workspace_zeroed=True))
        assert len(kl) == 1 and "in-kernel combine" in kl[0], kl
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
    cnt = ws[-256:].view(torch.int32)  # the counters sit at the end of the workspace
    assert int(cnt.abs().sum()) == 0
