"""Phase anatomy of the forward kernel from an FA_STAMPS=1 diagnostic build.

    bash scripts/build_variants.sh stamps "-DFA_STAMPS=1"
    python scripts/stamps.py [--config c3] exploring_flash_attention_amd/_lib/ab/stamps.so

Runs the config back to back (clock warm-up), then one stamped launch, and reports per
workgroup (wave 0's view, s_memtime shader cycles): prologue wait (entry -> Q/K0/V0/K1
landed), first QK^T (-> loop start), KV loop, epilogue issue and store retirement, plus the
per-CU seam: time a CU runs fewer than its two resident workgroups.  Diagnostic only: the
stamps cost a few percent and the numbers are cycles of the stamped build.
"""
import argparse
import collections
import ctypes
import statistics

import numpy as np
import torch

CFG = {"c2": (32, 8, 1024, 32), "c3": (32, 8, 1024, 128), "c4": (32, 8, 4096, 128),
       "l2048": (32, 8, 2048, 128), "d64": (32, 8, 1024, 64), "d256": (32, 8, 1024, 256)}


def pct(xs, p):
    return float(np.percentile(np.asarray(xs, dtype=np.float64), p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warmup", type=int, default=400)
    args = ap.parse_args()
    B, H, L, d = CFG[args.config]
    lib = ctypes.CDLL(args.lib)
    lib.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
    lib.fa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        assert lib.fa_fwd_v1(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, 1, stream) == 0

    for _ in range(args.warmup):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    wall_us = e0.elapsed_time(e1) * 1e3
    bq = 128
    nwg = B * H * ((L + bq - 1) // bq)
    buf = np.zeros(nwg * 16, dtype=np.uint64)
    assert lib.fa_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(nwg, 16).astype(np.int64)
    xcc = s[:, 7] & 0xF
    # s_memtime counters are per XCD (not synchronised across XCDs): spans are per XCD
    spans = [s[xcc == x, 5].max() - s[xcc == x, 0].min() for x in np.unique(xcc)]
    clk = max(spans) / wall_us  # cycles per us
    print(f"config {args.config}: {nwg} workgroups, launch {wall_us:.1f} us (HIP events), longest XCD span "
          f"{max(spans)} cycles (shortest {min(spans)}) -> {clk / 1e3:.2f} GHz effective")
    names = ["prologue wait", "first QK^T", "KV loop", "epilogue issue", "store retire"]
    for i, nm in enumerate(names):
        dt = s[:, i + 1] - s[:, i]
        print(f"  {nm:15s} median {np.median(dt):8.0f}  p10 {pct(dt, 10):8.0f}  p90 {pct(dt, 90):8.0f}  cycles"
              f"  ({np.median(dt) / clk:6.2f} us)")
    life = s[:, 5] - s[:, 0]
    ntiles = (L + 63) // 64
    loop = s[:, 3] - s[:, 2]
    print(f"  lifetime        median {np.median(life):8.0f} cycles; KV loop per step {np.median(loop) / ntiles:.0f} cycles"
          f" over {ntiles} tiles; non-loop share of lifetime {1 - np.median(loop) / np.median(life):.1%}")
    # per-CU timelines on the global 100 MHz clock (slots 8, 9): wave 0's hw_id bits [15:8] + xcc
    rt0 = s[:, 8].min()
    ent, end = (s[:, 8] - rt0) * 0.01, (s[:, 9] - rt0) * 0.01  # us
    print(f"  realtime: first entry -> last end {end.max():.1f} us; entries of the first 512 workgroups "
          f"within {np.sort(ent)[511]:.2f} us")
    cu = collections.defaultdict(list)
    for w in range(nwg):
        cu[(int(s[w, 7]) & 0xF, (int(s[w, 6]) >> 8) & 0xFF)].append((ent[w], end[w]))
    counts = collections.Counter(len(x) for x in cu.values())
    print(f"  distinct CUs seen: {len(cu)}; workgroups per CU histogram {dict(sorted(counts.items()))}")
    last_end = np.array([max(b for _, b in x) for x in cu.values()])
    two_end = np.array([sorted(b for _, b in x)[-2] for x in cu.values()])
    print(f"  per-CU last end: min {last_end.min():.1f} median {np.median(last_end):.1f} max {last_end.max():.1f} us;"
          f" CU idle (one slot) after its second-to-last end: median {np.median(last_end - two_end):.1f} us")
    under, gaps = [], []
    for wgs in cu.values():
        ev = sorted([(a_, 1) for a_, _ in wgs] + [(b_, -1) for _, b_ in wgs])
        occ, last, below = 0, None, 0.0
        for t, dlt in ev:
            if last is not None and occ < 2:
                below += t - last
            occ += dlt
            last = t
        under.append(below)
        ends = sorted(b_ for _, b_ in wgs)
        for a_, _ in sorted(wgs)[2:]:
            prev = [b_ for b_ in ends if b_ <= a_]
            if prev:
                gaps.append(a_ - prev[-1])
    # how the CU's resident workgroups' KV loops overlap: each workgroup's loop interval mapped
    # onto the realtime clock (its own memtime -> realtime line), then per CU the time with 0, 1
    # and 2 workgroups inside their loops, from the CU's first entry to its last end
    scale = (end - ent) / np.maximum(s[:, 5] - s[:, 0], 1)
    lo_a = ent + (s[:, 2] - s[:, 0]) * scale
    lo_b = ent + (s[:, 3] - s[:, 0]) * scale
    cu_loops = collections.defaultdict(list)
    for w in range(nwg):
        cu_loops[(int(s[w, 7]) & 0xF, (int(s[w, 6]) >> 8) & 0xFF)].append((lo_a[w], lo_b[w], ent[w], end[w]))
    in_loop = np.zeros(3)
    for wgs in cu_loops.values():
        ev = sorted([(a_, 1) for a_, _, _, _ in wgs] + [(b_, -1) for _, b_, _, _ in wgs])
        t0, t1 = min(x[2] for x in wgs), max(x[3] for x in wgs)
        occ, last = 0, t0
        for t, dlt in ev:
            in_loop[min(occ, 2)] += t - last
            occ += dlt
            last = t
        in_loop[0] += t1 - last
    in_loop /= in_loop.sum()
    print(f"  CU time with 0 / 1 / 2 workgroups inside their KV loops: "
          f"{in_loop[0]:.1%} / {in_loop[1]:.1%} / {in_loop[2]:.1%}")
    # per XCD: last end, and the clock its workgroups ran at (memtime cycles over realtime)
    wclk = (s[:, 5] - s[:, 0]) / np.maximum(end - ent, 1e-3)  # cycles per us
    step_cyc = (s[:, 3] - s[:, 2]) / ntiles
    parts = []
    for x in np.unique(xcc):
        m_ = xcc == x
        parts.append(f"x{int(x)}: end {end[m_].max():.1f} us, {np.median(wclk[m_]) / 1e3:.2f} GHz, "
                     f"{np.median(step_cyc[m_]):.0f} cyc/step")
    print("  per XCD: " + "; ".join(parts))
    total = end.max()
    print(f"  slot-time lost with < 2 resident workgroups (until the kernel's last end): "
          f"{np.mean([u + (total - le) for u, le in zip(under, last_end)]) / total:.1%} of 2 x span per CU"
          f"; refill gap median {np.median(gaps):.2f} us p90 {pct(gaps, 90):.2f} us")


if __name__ == "__main__":
    main()
