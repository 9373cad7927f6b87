"""Benchmark of the flash-attention forward on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)
    (`python bench.py --gpus N` with N > 1 and no launcher starts the N ranks itself, before
    any GPU work; fewer than N GPUs on the node, or a WORLD_SIZE that disagrees with --gpus,
    is an error with a non-zero exit status, never a one-GPU line)
    python bench.py --mode splitkv-dist ...   (C5: one sequence's keys sharded over ranks)

Default workload (N=1): config C3 of BASELINE.json -- FA-v1 fused forward, B=32 H=8 L=1024
d=128, bf16 storage / fp32 accumulate, synthetic N(0,1) inputs resident in HBM.  A step
is one forward over the whole batch.  With N>1 every rank runs its own C3 batch (heads
are independent units: weak scaling, no collective in the data path).

Prints ONE JSON line on rank 0 with the metric, the MFMA roofline of the forward kernel
(achieved = 4*B*H*L^2*d FLOPs per launch / average launch time from HIP events on the
launch stream), a check of the headline output against fp64 attention on sampled heads, and
the CPU baseline: the oracle's restatement of the reference's
flash_attention_v1/numpy_gpu_like_opt2.py (fp64, Bq=Bk=8) timed on k heads per usable host
core, one head per process, extrapolated to the whole batch (and, beside it, the C/OpenMP
restatement of the drivers' standard_attention_cpu over the whole batch on the same cores).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16/fp16 MFMA (MI355X_MICROARCH.md)
C5_TIMEOUT_S = 240  # watchdog of the C5 split-KV extra (seconds)
CONFIGS = {
    "c2": dict(B=32, H=8, L=1024, d=32, variant="v1"),
    "c3": dict(B=32, H=8, L=1024, d=128, variant="v1"),
    "c4": dict(B=32, H=8, L=4096, d=128, variant="v2", kvtpb=4),
    "c5": dict(B=32, H=8, L=16384, d=128, variant="dist"),
}


def flops(B, H, L, d, Lk=None):
    return 4.0 * B * H * L * (L if Lk is None else Lk) * d


PROBE_LIB = os.path.join(ROOT, "exploring_flash_attention_amd", "_lib", "libfa_probe.so")


def measured_ceiling(d):
    """The MFMA rate this box sustains on random operands, on the shape the headline kernel
    issues (d = 128: v_mfma_f32_16x16x32_bf16; other head dims: 32x32x16), measured live with
    csrc/fa_probe.hip (4 accumulation chains per wave, 2 waves per SIMD, nothing else in the
    loop; ~0.7 s).  The operand values set the MFMA array's power and so the clock the chip
    holds, which puts this ceiling far below the 2.5 PF datasheet figure;
    roofline.frac stays against the datasheet, frac_of_measured is against this."""
    import ctypes
    shape = 1 if d == 128 else 0
    names = {0: "v_mfma_f32_32x32x16_bf16", 1: "v_mfma_f32_16x16x32_bf16"}
    try:
        lib = ctypes.CDLL(PROBE_LIB)
    except OSError as exc:
        return {"error": f"libfa_probe.so not loadable: {exc}"[:200]}
    lib.fa_probe_mfma_ceiling.argtypes = [ctypes.c_int] * 6 + [ctypes.POINTER(ctypes.c_double)]
    res = {"shape": names[shape], "waves_per_simd": 2}
    out = (ctypes.c_double * 3)()
    iters = 2000 if shape == 1 else 1000  # ~50 ms per launch
    # pattern 2: A repeated in pairs (the kernel's order: one K fragment / V^T operand feeds the
    # wave's two query blocks); pattern 1: a new (A, B) pair every MFMA
    for pat, key in ((2, "random_a_pairs"), (1, "random")):
        rc = lib.fa_probe_mfma_ceiling(shape, pat, 2, iters, 5, 10, out)
        if rc != 0:
            return {"error": f"fa_probe_mfma_ceiling returned {rc}"}
        res[key] = {"tflops": round(out[0], 1), "held_clock_mhz": round(out[1])}
    res["tflops"] = res["random_a_pairs"]["tflops"]
    return res


# ------------------------------------------------------------------------------------
# CPU baseline (oracle restatement of numpy_gpu_like_opt2.py), run BEFORE any GPU init
# ------------------------------------------------------------------------------------

def _cpu_head(args):
    L, d, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import numpy as np
    from oracle.fa_v1 import flash_attention_tiled_flat
    rng = np.random.default_rng(seed)
    Q, K, V = (rng.standard_normal(L * d) for _ in range(3))
    O = np.zeros(L * d)
    t0 = time.perf_counter()
    flash_attention_tiled_flat(Q, K, V, O, L, d, Bq=8, Bk=8)
    return time.perf_counter() - t0


def host_cores():
    """(cores this process may use, os.cpu_count()): the CPU affinity set, capped by the
    cgroup CPU quota (cpu.max) where one is set -- on a GPU box os.cpu_count() reports the
    whole machine, of which a job gets a share."""
    n = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return usable, n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(L, d, ncores, k=1, total_heads=256):
    """the oracle's restatement of numpy_gpu_like_opt2.py (fp64, Bq=Bk=8)
    over k heads per core, one head per process on multiprocessing.Pool(ncores); the per-head
    cost is shape-determined, so the whole batch's time is extrapolated linearly."""
    import multiprocessing as mp
    for var in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[var] = "1"
    heads = min(total_heads, k * ncores)
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(ncores) as pool:
        per_head = pool.map(_cpu_head, [(L, d, s) for s in range(heads)])
    wall = time.perf_counter() - t0
    head_s = sum(per_head) / heads
    extrap = wall * total_heads / heads
    _, all_cpus = host_cores()
    return {
        "value": round(heads * flops(1, 1, L, d) / wall / 1e9, 4),
        "unit": "GFLOP/s",
        "cores": ncores,
        "kind": "port",
        "cpu_model": cpu_model(),
        "host_cpus": all_cpus,
        "heads_per_core": k,
        "per_head_s": round(head_s, 2),
        "extrapolated_s": round(extrap, 1),
        "sample": (f"{heads} of the {total_heads} heads of L={L} d={d} (fp64, Bq=Bk=8), k={k} per core, one "
                   f"head per process on Pool({ncores}) ({ncores} usable of {all_cpus} host CPUs, "
                   f"{cpu_model()}); wall {wall:.1f} s, {head_s:.1f} s per head, all {total_heads} heads "
                   f"extrapolated to {extrap:.0f} s; restatement of "
                   f"flash_attention_v1/numpy_gpu_like_opt2.py (oracle/fa_v1.py)"),
    }


_OMP_SNIPPET = r"""
import ctypes, json, sys, time
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
P, I = ctypes.c_void_p, ctypes.c_int
lib.oracle_standard_attention.argtypes = [P, P, P, P, I, I, I, I, I]
H, L, d = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rng = np.random.default_rng(0)
q, k, v = (rng.uniform(-1, 1, (1, H, L, d)).astype(np.float32) for _ in range(3))
o = np.empty_like(q)
t0 = time.perf_counter()
lib.oracle_standard_attention(q.ctypes.data, k.ctypes.data, v.ctypes.data, o.ctypes.data, 1, H, L, d, 2)
print(json.dumps({"wall": time.perf_counter() - t0}))
"""


def cpu_baseline_openmp(L, d, threads, total_heads=256):
    """The C/OpenMP restatement of the reference's standard_attention_cpu
    (common/standard.h:28-102; oracle/standard_attention.c) over the whole batch of the same
    shape (256 heads at C3), fp32, in a child process with OMP_NUM_THREADS = threads
    (SURVEY.md 8(d))."""
    import subprocess
    lib = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib):
        return None
    heads = total_heads
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    try:
        out = subprocess.run([sys.executable, "-c", _OMP_SNIPPET, lib, str(heads), str(L), str(d)],
                             env=env, capture_output=True, text=True, timeout=120, check=True)
        wall = json.loads(out.stdout.strip().splitlines()[-1])["wall"]
    except (subprocess.SubprocessError, ValueError, IndexError, KeyError):
        return None
    return {"value": round(heads * flops(1, 1, L, d) / wall / 1e9, 3), "unit": "GFLOP/s", "cores": threads,
            "kind": "port", "wall_s": round(wall, 2),
            "sample": (f"all {heads} heads of L={L} d={d} (fp32), naive attention with OpenMP over heads at "
                       f"OMP_NUM_THREADS={threads}; wall {wall:.2f} s; restatement of common/standard.h "
                       f"standard_attention_cpu (oracle/standard_attention.c)")}


# ------------------------------------------------------------------------------------
# GPU timing
# ------------------------------------------------------------------------------------

def _make_inputs(torch, dev, B, H, L, d, seed, Lk=None):
    g = torch.Generator(device=dev).manual_seed(seed)
    Lk = L if Lk is None else Lk
    q = torch.randn(B, H, L, d, device=dev, dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, H, Lk, d, device=dev, dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, H, Lk, d, device=dev, dtype=torch.bfloat16, generator=g)
    return q, k, v


def time_step(torch, step, steps, warmup, barrier):
    """Warm up, then time exactly `steps` calls.  Returns (wall_s, event_ms_total)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_time(ev1)


def launched(ops, step):
    """Run `step` once and return the kernels (with their grids) the library reports having
    launched for it (fa_last_kernels via ops.launched_kernels) -- what ran, as the launcher
    chose it, not a restatement of its rules."""
    with ops.launched_kernels() as kl:
        step()
    return " + ".join(dict.fromkeys(kl)) if kl else None


def clock_settle(torch, step, seconds):
    """Run `step` untimed, back to back, for about `seconds` (the MI355X clock ramps over the
    first ~50 ms of sustained work); returns the seconds spent."""
    if seconds <= 0:
        return 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def c5_step(torch, fdist, dev, world, rank, impl="torch"):
    """One C5 split-KV step closure: the keys of B=32 H=8 L=16384 d=128 sharded over the
    ranks, partial kernel -> all-to-all -> combine (dist.splitkv_attention)."""
    cc = CONFIGS["c5"]
    B, H, L, d = cc["B"], cc["H"], cc["L"], cc["d"]
    lo, hi = fdist.shard_bounds(L, world, rank)
    q, _, _ = _make_inputs(torch, dev, B, H, L, d, seed=99)  # same Q on every rank
    _, k, v = _make_inputs(torch, dev, B, H, 1, d, seed=1000 + rank, Lk=hi - lo)
    if impl == "native":
        comm = fdist.RcclComm()

        def step():
            fdist.splitkv_attention_native(q, k, v, comm)
        kernel = ("fa_fwd_partial_ex per destination chunk + RCCL send/recv on the exchange stream + "
                  "fa_combine (C ABI fa_fwd_v2_dist; its launches are internal to libfa_mi355x_dist.so)")
    else:
        def step():
            fdist.splitkv_attention(q, k, v)
        from exploring_flash_attention_amd import ops
        kernel = launched(ops, step)
        if world > 1:
            kernel = f"{kernel} (pipelined RCCL send/recv between the partial chunks and the combine)"
    return step, kernel, flops(B, H, L, d, Lk=hi - lo)


def c5_breakdown(torch, ops, fdist, dev, world, rank, barrier):
    """C5 on this rank, each stage timed alone: the partial kernel over all L query rows (one
    launch, the all-to-all send layout), the exchange of those partials between the ranks
    (N > 1: W-1 shifted RCCL send/recv steps posted together, dist.exchange_partials -- the
    xGMI traffic alone, no kernel beside it), and the combine of the W received partials for the
    rank's L/W rows.  Bytes per rank that cross xGMI, and the rate the exchange moved them at."""
    cc = CONFIGS["c5"]
    B, H, L, d = cc["B"], cc["H"], cc["L"], cc["d"]
    lo, hi = fdist.shard_bounds(L, world, rank)
    Lc = L // world
    q, _, _ = _make_inputs(torch, dev, B, H, L, d, seed=99)
    _, k, v = _make_inputs(torch, dev, B, H, 1, d, seed=1000 + rank, Lk=hi - lo)
    pd = ops.PARTIAL_FP16_SCALED
    o_part, lse = ops.attention_partial(q, k, v, chunk_rows=Lc, partial_dtype=pd)
    n = 5
    _, p_ms = time_step(torch, lambda: ops.attention_partial(q, k, v, chunk_rows=Lc, partial_dtype=pd,
                                                             o_part=o_part, lse=lse), n, 2, barrier)
    del q, k, v
    out = torch.empty(B, H, Lc, d, dtype=torch.bfloat16, device=dev)
    _, c_ms = time_step(torch, lambda: ops.combine(o_part, lse, B, H, torch.bfloat16, out=out), n, 2, barrier)
    p_ms, c_ms = p_ms / n, c_ms / n
    c_bytes = o_part.numel() * 2 + lse.numel() * 4 + out.numel() * 2
    x_bytes = (world - 1) * (o_part[0].numel() * 2 + lse[0].numel() * 4)
    rec = {"partial_ms": round(p_ms, 3), "combine_ms": round(c_ms, 4),
           "combine_gbps": round(c_bytes / (c_ms * 1e-3) / 1e9, 1),
           "exchange_bytes_per_rank": int(x_bytes), "partial_format": "fp16 scaled per row"}
    if world > 1:
        o_recv, lse_recv = torch.empty_like(o_part), torch.empty_like(lse)

        def xchg():
            for w in fdist.exchange_partials(o_part, lse, o_recv, lse_recv):
                w.wait()
        _, x_ms = time_step(torch, xchg, n, 2, barrier)
        x_ms /= n
        rec.update(exchange_ms=round(x_ms, 3), exchange_gbps=round(x_bytes / (x_ms * 1e-3) / 1e9, 1),
                   exchange="W-1 shifted send/recv steps posted together (each rank sends and receives "
                            "exchange_bytes_per_rank; gbps = those bytes / exchange_ms, per rank)")
    return rec


# Split-KV shapes: C4 itself (KV_TILES_PER_BLOCK = 4) under the library's grouping, with the
# grouping forced (4 and 1 key blocks per workgroup: 4 / 16 partials per query tile) and the
# automatic split; and two low-parallelism shapes -- the regime the reference's split-KV exists
# for (flash_attention_v2/README.md:7-21): fewer query tiles than CUs, so the library itself
# splits (4 partials per query tile each) -- each against the same shape forced onto one
# workgroup per query tile (blocks_per_workgroup = all blocks).
EXTRA_SHAPES = (
    # name, B, H, L, d, variant, kv_tiles_per_block, blocks_per_workgroup
    ("c2_fused", 32, 8, 1024, 32, "v1", None, None),
    # head dims past one tile: the d-tiled kernel (K / V column chunks of d_tile = 128 columns)
    ("d384_tiled_d", 32, 8, 1024, 384, "tiled_d", None, None),
    ("d512_tiled_d", 32, 8, 1024, 512, "tiled_d", None, None),
    ("c4_splitkv", 32, 8, 4096, 128, "v2", 4, None),
    ("c4_splitkv_4_blocks_per_wg", 32, 8, 4096, 128, "v2", 4, 4),
    ("c4_splitkv_1_block_per_wg", 32, 8, 4096, 128, "v2", 4, 1),
    ("c4_splitkv_auto", 32, 8, 4096, 128, "v2", "auto", None),
    ("b1h1_l16k_splitkv", 1, 1, 16384, 128, "v2", 4, None),
    ("b1h1_l16k_unsplit", 1, 1, 16384, 128, "v2", 4, "all"),
    ("b1h2_l4k_splitkv", 1, 2, 4096, 128, "v2", 4, None),
    ("b1h2_l4k_unsplit", 1, 2, 4096, 128, "v2", 4, "all"),
)
SPLIT_PAIRS = ("b1h1_l16k", "b1h2_l4k")
# each extra's entry in profiles/hbm_traffic.json (rocprofv3 PMC passes of scripts/run_kernel.py
# at the same shape and plan; kernel-labelled there): L2 egress per launch beside the timing
EXTRA_TRAFFIC = {"c2_fused": "c2", "d384_tiled_d": "d384", "d512_tiled_d": "d512", "c4_splitkv": "c4",
                 "c4_splitkv_4_blocks_per_wg": "c4g4", "c4_splitkv_1_block_per_wg": "c4g1",
                 "c4_splitkv_auto": "c4", "b1h1_l16k_splitkv": "b1h1l16k",
                 "b1h1_l16k_unsplit": "b1h1l16k_unsplit", "b1h2_l4k_splitkv": "b1h2l4k",
                 "b1h2_l4k_unsplit": "b1h2l4k_unsplit"}
EXTRA_SETTLE_S = 0.1  # untimed back-to-back launches of each extra shape before its window


def single_gpu_extras(torch, ops, dev, barrier, names=None):
    """bench extras at N = 1: ms, TFLOP/s and the split plan of each EXTRA_SHAPES entry."""
    out = {}
    for name, B, H, L, d, fn, kvt, grp in EXTRA_SHAPES:
        if names is not None and name not in names:
            continue
        qq, kk, vv = _make_inputs(torch, dev, B, H, L, d, seed=7)
        rec = {"B": B, "H": H, "L": L, "d": d}
        if fn == "v1":
            def st():
                ops.attention_v1(qq, kk, vv)
        elif fn == "tiled_d":
            def st():
                ops.attention_tiled_d(qq, kk, vv, 128, 128)
            rec.update(d_tile_qk=128, d_tile_v=128)
        else:
            if grp == "all":  # every key block of a query tile on one workgroup: no split
                grp = ops.v2_split_plan(B, H, L, d, kvt, qq.dtype)[0]
            nb, _ = ops.v2_workspace_bytes(B, H, L, d, kvt, qq.dtype, blocks_per_workgroup=grp)
            plan = ops.v2_split_plan(B, H, L, d, kvt, qq.dtype, blocks_per_workgroup=grp)
            # zeroed once; every launch leaves its counters zero (ops.attention_v2 workspace_zeroed)
            wsx = torch.zeros(nb, dtype=torch.uint8, device=dev)
            oo = torch.empty_like(qq)

            def st():
                ops.attention_v2(qq, kk, vv, kvt, out=oo, workspace=wsx, blocks_per_workgroup=grp,
                                 workspace_zeroed=True)
            rec.update(kv_tiles_per_block=kvt, key_blocks=plan[0], blocks_per_workgroup=plan[1],
                       partials_per_tile=plan[2], workspace_bytes=nb)
        f = flops(B, H, L, d)
        n = max(10, min(50, int(2e13 / f)))  # >= ~20 TFLOP of work per timing window
        # each shape's own clock settle: the chip's clock after the previous shape (a
        # low-power one boosts it, a hot one holds it down) otherwise carries into this window
        # (C4 read 1.84 ms after the d = 512 shape and 1.74 ms for the same kernel and grid as
        # c4_splitkv_auto; profiles/r04/bench_driver_cmd_g.json)
        rec["kernel"] = launched(ops, st)
        clock_settle(torch, st, EXTRA_SETTLE_S)
        _, ems = time_step(torch, st, n, max(3, n // 3), barrier)
        ms = ems / n
        rec.update(ms=round(ms, 4), tflops=round(f / (ms * 1e-3) / 1e12, 1),
                   frac=round(f / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4))
        tr = extra_traffic(name, B, H, L, d)
        if tr is not None:
            rec["traffic"] = tr
        out[name] = rec
        del qq, kk, vv
    for base in SPLIT_PAIRS:  # split against unsplit, same shape
        if f"{base}_splitkv" in out and f"{base}_unsplit" in out:
            out[f"{base}_splitkv"]["speedup_vs_unsplit"] = round(
                out[f"{base}_unsplit"]["ms"] / out[f"{base}_splitkv"]["ms"], 3)
    return out


def load_traffic(config, full=False):
    """bytes per launch of profiles/hbm_traffic.json[config] (the whole record with full=True),
    None when the table has no such entry."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(config)
        return rec if full or rec is None else rec.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def extra_traffic(name, B, H, L, d):
    """the L2-egress record of an extra (measured in a PMC pass, not in this run) against its
    algorithmic bytes (Q, K, V read once, O written once)."""
    key = EXTRA_TRAFFIC.get(name)
    rec = load_traffic(key, full=True) if key else None
    if rec is None:
        return None
    alg = 4 * B * H * L * d * 2
    return {"bytes_per_launch": int(rec["bytes_per_launch"]), "algorithmic_bytes": alg,
            "ratio": round(rec["bytes_per_launch"] / alg, 2), "kernel": rec.get("kernel"),
            "source": f"profiles/hbm_traffic.json[{key}] ({rec.get('source', 'PMC')})"}


def sample_heads(B, H, n=16):
    """n (b, h) pairs spread over the batch, first and last included."""
    BH = B * H
    idx = sorted({round(i * (BH - 1) / (n - 1)) for i in range(n)})
    return [(i // H, i % H) for i in idx]


def output_check(torch, q, k, v, out, n=16):
    """max_abs / mean_rel of the kernel's output against fp64 attention computed by torch on
    the device, over n sampled heads (every query tile of each), outside the timed region.
    (A torch fp64 reference of the same op: the CPU oracle stays out of the product bench.)"""
    B, H, L, d = q.shape
    worst, rel_sum, rel_n = 0.0, 0.0, 0
    for b, h in sample_heads(B, H, n):
        qq, kk, vv = (t[b, h].double() for t in (q, k, v))
        p = torch.softmax((qq @ kk.T) / d ** 0.5, dim=-1)
        ref = p @ vv
        err = (out[b, h].double() - ref).abs()
        worst = max(worst, float(err.max()))
        big = ref.abs() > 1e-3
        rel_sum += float((err[big] / ref.abs()[big]).sum())
        rel_n += int(big.sum())
    return {"max_abs": round(worst, 6), "mean_rel": round(rel_sum / max(rel_n, 1), 6), "heads": n,
            "reference": "torch fp64 softmax(q k^T / sqrt(d)) v on the device, sampled heads incl. first/last"}


def splitkv_scaling_field(c5, world):
    """The north_star's multi-GPU row (C5: one L=16384 batch's keys sharded over the ranks,
    partials exchanged over RCCL, combined per rank) lifted to the top of the line, so that the
    driver's 1/2/4/8-GPU runs record the split-KV curve beside the heads-parallel headline."""
    rec = {"config": "C5: B=32 H=8 L=16384 d=128 bf16, keys sharded over the ranks", "ranks": world,
           "unit": "GFLOP/s (whole job)"}
    if "error" in c5:
        rec["error"] = c5["error"]
        return rec
    bd = c5.get("breakdown_max_over_ranks", {})
    rec.update(ms=c5["ms"], value=round(c5["tflops"] * 1e3, 1), frac=c5["frac"], exchange=c5.get("exchange"))
    for key in ("partial_ms", "combine_ms", "exchange_ms", "exchange_gbps", "exchange_bytes_per_rank"):
        if key in bd:
            rec[key] = bd[key]
    return rec


WATCHDOG_EXIT = 3


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n, script, script_args, env=None):
    """Run `script` as n ranks of one node (torch.distributed.run, rendezvous on 127.0.0.1)
    as a CHILD process -- never an exec -- and return its exit status: non-zero when any rank
    fails (torch.distributed.run reports a failed rank and exits non-zero)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *script_args]
    return subprocess.call(cmd, env=dict(os.environ if env is None else env))


def self_launch(gpus, argv):
    """`bench.py --gpus N` (N > 1) without a launcher: start N ranks before any GPU work.  A
    box with fewer than N GPUs is an error, never a silent one-GPU line.  (Counting devices
    does not initialise the GPU on this image.)"""
    import torch
    have = torch.cuda.device_count()
    if have < gpus:
        print(f"bench: --gpus {gpus} requested but this node has {have} GPU(s); refusing to report a "
              f"{have}-GPU number as a {gpus}-GPU one", file=sys.stderr, flush=True)
        return 2
    print(f"bench: launching {gpus} ranks (torch.distributed.run, one process per GPU)", file=sys.stderr,
          flush=True)
    return spawn_ranks(gpus, os.path.abspath(__file__), argv)


def start_watchdog(seconds, rank, partial_line):
    """After `seconds`: print partial_line() (rank 0's JSON line with the error recorded, or
    None) and leave the process with status WATCHDOG_EXIT -- a hung exchange is a failed run
    for the driver, never a green one.  Returns the timer (cancel() it when done)."""
    def fire():
        rec = partial_line()
        if rec is not None:
            print(json.dumps(rec), flush=True)
        print(f"bench: watchdog fired after {seconds} s on rank {rank}", file=sys.stderr, flush=True)
        os._exit(WATCHDOG_EXIT)
    dog = threading.Timer(seconds, fire)
    dog.daemon = True
    dog.start()
    return dog


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # The MI355X clock ramps up over the first ~50 ms of back-to-back launches (measured:
    # 183 / 161 / 149 us per C3 step after 20 / 100 / 400 steps), so the defaults time the
    # steady state: 300 untimed steps, then 500 timed (~0.1 s in all).
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
    ap.add_argument("--mode", default="heads", choices=["heads", "splitkv-dist"])
    ap.add_argument("--dist-impl", default="torch", choices=["torch", "native"],
                    help="splitkv-dist exchange: torch.distributed all_to_all, or the C ABI "
                         "fa_fwd_v2_dist (own RCCL communicator, grouped send/recv)")
    ap.add_argument("--cpu-cores", type=int, default=0, help="CPU baseline pool size (0 = the usable host cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the per-variant extra timings")
    ap.add_argument("--clock-warmup", type=float, default=0.25,
                    help="seconds of untimed headline steps right before --warmup (clock settle; 0 = off)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the request disagree",
              file=sys.stderr, flush=True)
        sys.exit(2)

    cfg = CONFIGS["c5"] if args.mode == "splitkv-dist" else CONFIGS[args.config]
    B, H, L, d = cfg["B"], cfg["H"], cfg["L"], cfg["d"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.mode == "heads":
        ncores = args.cpu_cores or host_cores()[0]
        cpu = cpu_baseline(L, d, ncores)  # before any GPU initialisation (fork-safe)
        omp = cpu_baseline_openmp(L, d, ncores)
        if omp is not None:
            cpu["openmp_standard_attention"] = omp

    import torch
    import torch.distributed as dist

    from exploring_flash_attention_amd import dist as fdist
    from exploring_flash_attention_amd import ops

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra and args.mode == "heads":
        # the extras get a settled clock too (C3 forwards, untimed), then each its own warm-up
        cw = CONFIGS["c3"]
        qw, kw, vw = _make_inputs(torch, dev, cw["B"], cw["H"], cw["L"], cw["d"], seed=3)
        clock_settle(torch, lambda: ops.attention_v1(qw, kw, vw), 0.1)
        del qw, kw, vw
        # per-variant timings at N=1 (informational; not the headline value).  They run
        # before the headline, so the headline's window also finds the clock settled.
        # (C3's tiled-d form is the same launch as the headline: fa_fwd_v1_tiled_d validates
        # the d tiles and runs the fused kernel)
        extra.update(single_gpu_extras(torch, ops, dev, barrier))
        torch.cuda.empty_cache()

    check = None
    ceiling = None
    t_warm = 0.0
    if args.mode == "heads":
        q, k, v = _make_inputs(torch, dev, B, H, L, d, seed=1234 + rank)
        out = torch.empty_like(q)
        if cfg["variant"] == "v1":
            def step():
                ops.attention_v1(q, k, v, out=out)
        else:
            nbytes, _ = ops.v2_workspace_bytes(B, H, L, d, cfg["kvtpb"], q.dtype)
            ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)

            def step():
                ops.attention_v2(q, k, v, cfg["kvtpb"], out=out, workspace=ws, workspace_zeroed=True)
        kernel = launched(ops, step)
        # Clock settle, immediately before the headline's --warmup (after the extras, whose
        # last shapes are small): the chip needs ~50 ms of back-to-back work before its clock
        # holds, so the headline's own step runs untimed for
        # --clock-warmup seconds (reported as clock_warmup_s); then exactly --warmup more
        # untimed steps and exactly --steps timed ones.
        t_warm = clock_settle(torch, step, args.clock_warmup)
        wall, ev_ms = time_step(torch, step, args.steps, args.warmup, barrier)
        ceiling = measured_ceiling(d) if rank == 0 else None  # after the timed window
        work = flops(B, H, L, d)
        workload = ("FA-v1 fused / tiled-d forward (one kernel)" if cfg["variant"] == "v1"
                    else "FA-v2 split-KV forward")
        parallel = f"heads{world}" if world > 1 else "single"
        if rank == 0:
            check = output_check(torch, q, k, v, out)
    else:
        # C5: keys of one L=16384 sequence sharded over the ranks; all-to-all combine.
        step, kernel, work = c5_step(torch, fdist, dev, world, rank, args.dist_impl)  # work: this rank's share
        t_warm = clock_settle(torch, step, min(args.clock_warmup, 0.1))
        wall, ev_ms = time_step(torch, step, args.steps, args.warmup, barrier)
        workload = "FA-v2 split-KV forward, keys sharded over ranks"
        parallel = f"kv{world}"

    # max over ranks
    t = torch.tensor([wall, ev_ms], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, ev_ms = float(t[0]), float(t[1])
    ms_per_step = wall / args.steps * 1e3
    total_work = work * world
    value = total_work / (wall / args.steps) / 1e9

    if rank == 0:
        avg_ms = ev_ms / args.steps
        achieved = work / (avg_ms * 1e-3) / 1e12
        tcfg = args.config if args.mode == "heads" else "c5"
        traffic = load_traffic(tcfg)
        line = {
            "metric": "flash-attn fwd GFLOP/s (B=32,H=8,L=1024,d=128; % MFMA roofline)"
            if args.mode == "heads" and args.config == "c3" else f"flash-attn fwd GFLOP/s ({tcfg})",
            "value": round(value, 1),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic N(0,1)",
            "config": {"workload": workload, "B": B, "H": H, "L": L, "d": d,
                       "global_batch": B * H * world, "seq_len": L, "parallelism": parallel,
                       "tiles": {"bq": 128, "bk": 64, "threads": 256}},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                         "traffic": traffic,
                         "traffic_source": (f"profiles/hbm_traffic.json[{tcfg}] (rocprofv3 PMC passes, "
                                            "per launch; not measured in this run)") if traffic else None,
                         "kernel": kernel, "kernel_ms": round(avg_ms, 5)},
            "cpu_baseline": cpu,
        }
        if ceiling is not None:
            rf = line["roofline"]
            rf["ceiling_measured"] = ceiling.get("tflops")
            rf["frac_of_measured"] = (round(achieved / ceiling["tflops"], 4) if ceiling.get("tflops") else None)
            rf["ceiling_source"] = ceiling
        if check is not None:
            line["check"] = check
        line["clock_warmup_s"] = round(t_warm, 3)
    printed, dog = False, None
    if not args.no_extra and args.mode == "heads":
        # C5 split-KV over all ranks (north_star: 1/2/4/8-GPU split-KV throughput and achieved
        # fraction); every rank takes part in the exchange, time = max over ranks.  A watchdog
        # keeps an exchange that never completes from costing the headline line: after
        # C5_TIMEOUT_S rank 0 prints what was measured, and every rank exits with status 3
        # (a hang is a failure, never a green run).
        def _partial_line():
            if rank == 0 and not printed:
                extra["c5_splitkv_dist"] = {"error": f"no result within {C5_TIMEOUT_S} s", "ranks": world}
                line["extra"] = extra
                return line
            return None
        dog = start_watchdog(C5_TIMEOUT_S, rank, _partial_line)
        try:
            st5, _, w5 = c5_step(torch, fdist, dev, world, rank)
            n5 = 10
            wall5, ems5 = time_step(torch, st5, n5, 3, barrier)
            t5 = torch.tensor([wall5, ems5], device=dev, dtype=torch.float64)
            if world > 1:
                dist.all_reduce(t5, op=dist.ReduceOp.MAX)
            ms5 = float(t5[0]) / n5 * 1e3
            tf5 = w5 * world / (ms5 * 1e-3) / 1e12
            extra["c5_splitkv_dist"] = {"ms": round(ms5, 3), "tflops": round(tf5, 1),
                                        "frac": round(tf5 / (PEAK_BF16_TFLOPS * world), 4), "ranks": world,
                                        "exchange": ("per-chunk partials pipelined with pairwise RCCL "
                                                     "send/recv" if world > 1 else "none")}
            del st5
            torch.cuda.empty_cache()
            bd = c5_breakdown(torch, ops, fdist, dev, world, rank, barrier)
            keys = [k_ for k_ in ("partial_ms", "combine_ms", "exchange_ms") if k_ in bd]
            tb = torch.tensor([bd[k_] for k_ in keys], device=dev, dtype=torch.float64)
            if world > 1:
                dist.all_reduce(tb, op=dist.ReduceOp.MAX)
            for i, k_ in enumerate(keys):
                bd[k_] = round(float(tb[i]), 4)
            if "exchange_ms" in bd:
                bd["exchange_gbps"] = round(bd["exchange_bytes_per_rank"] / (bd["exchange_ms"] * 1e-3) / 1e9, 1)
            extra["c5_splitkv_dist"]["breakdown_max_over_ranks"] = bd
        except Exception as exc:  # noqa: BLE001 -- reported, the headline stands
            extra["c5_splitkv_dist"] = {"error": f"{type(exc).__name__}: {exc}"[:300], "ranks": world}
        torch.cuda.empty_cache()

    if rank == 0:
        if extra:
            line["extra"] = extra
        if "c5_splitkv_dist" in extra:
            line["splitkv_scaling"] = splitkv_scaling_field(extra["c5_splitkv_dist"], world)
        print(json.dumps(line), flush=True)
        printed = True
    if dog is not None:
        dog.cancel()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
