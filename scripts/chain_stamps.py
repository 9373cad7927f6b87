"""Per-step anatomy of the chained d = 128 kernel (fa_fwd16_chain.hpp) from an FA_STAMPS=1
lite build: the start time of each of a workgroup's first 64 steps (s_memtime, one VGPR lane
per step, written out after the loop), so that the cost of each step position within an item
-- the seam -- can be read off.

    bash scripts/build_lite.sh 128 stamps "-DFA_STAMPS=1"
    python scripts/chain_stamps.py exploring_flash_attention_amd/_lib/ab/stamps.so [--config c3]

Diagnostic only (the stamps cost a few VALU per step).
"""
import argparse
import ctypes
import statistics

import numpy as np
import torch

CFG = {"c3": (32, 8, 1024, 128), "l2048": (32, 8, 2048, 128), "c4": (32, 8, 4096, 128)}


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
    run = lambda: lib.fa_fwd_v1(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, 1, stream)
    for _ in range(args.warmup):
        assert run() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert run() == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    nwg = 512
    buf = np.zeros(nwg * 80, np.uint64)
    assert lib.fa_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(nwg, 80)
    t = st[:, :64].astype(np.uint32).astype(np.int64)
    end = st[:, 64].astype(np.uint32).astype(np.int64)
    steps_per_item = L // 64
    n_items = (B * H * (L // 128)) // nwg
    nsteps = min(64, steps_per_item * n_items)
    if nsteps == steps_per_item * n_items:  # every step stamped: the last one ends at the loop end
        d_all = np.diff(np.concatenate([t[:, :nsteps], end[:, None]], axis=1), axis=1)
    else:  # the first 64 of more steps: whole items only
        nsteps = (nsteps // steps_per_item) * steps_per_item
        d_all = np.diff(t[:, :nsteps + 1] if nsteps < 64 else t[:, :64], axis=1)
        d_all = d_all[:, :(d_all.shape[1] // steps_per_item) * steps_per_item] if d_all.shape[1] >= steps_per_item else d_all
    d_all = (d_all + (1 << 32)) % (1 << 32)
    rt0, rt1 = st[:, 65].astype(np.int64), st[:, 66].astype(np.int64)
    mhz = float(np.median((end - t[:, 0]) % (1 << 32) / ((rt1 - rt0) / 100.0)))  # cycles per us
    print(f"{args.config}: launch {ms * 1e3:.1f} us (HIP events), {n_items} items x {steps_per_item} steps per "
          f"workgroup, clock {mhz:.0f} MHz (s_memtime over s_memrealtime)")
    print("cycles per step by position within the item (median over workgroups and items; p90):")
    pos = np.arange(d_all.shape[1]) % steps_per_item
    for p in range(steps_per_item):
        x = d_all[:, pos == p].ravel()
        print(f"  step {p:2d}: {np.median(x):7.0f}  p90 {np.percentile(x, 90):7.0f}")
    per_item = [d_all[:, i * steps_per_item:(i + 1) * steps_per_item].sum(axis=1)
                for i in range(d_all.shape[1] // steps_per_item)]
    for i, x in enumerate(per_item):
        print(f"  item {i}: median {np.median(x):.0f} cycles = {np.median(x) / mhz:.2f} us")
    # launch skew: first-step start and loop end over workgroups, in real time
    start_us = (rt0 - rt0.min()) / 100.0
    end_us = (rt1 - rt0.min()) / 100.0
    print(f"  entry spread {start_us.max():.2f} us, loop end min {end_us.min():.2f} median "
          f"{np.median(end_us):.2f} max {end_us.max():.2f} us")
    # the two workgroups of a CU (HW_ID bits 8..15: CU, SH, SE; plus the XCC): end-time gap
    hw = st[:, 67].astype(np.int64)
    cu_key = (st[:, 68].astype(np.int64) & 0xF) * 256 + ((hw >> 8) & 0xFF)
    gaps, first_faster = [], 0
    for key in set(cu_key.tolist()):
        idx = np.nonzero(cu_key == key)[0]
        if len(idx) == 2:
            a, b = sorted(idx, key=lambda i: rt0[i])
            gaps.append(abs(end_us[a] - end_us[b]))
            first_faster += end_us[a] < end_us[b]
    if gaps:
        print(f"  CU pairs {len(gaps)}: end gap median {np.median(gaps):.2f} p90 {np.percentile(gaps, 90):.2f} us; "
              f"the earlier-started one ends first in {first_faster} of {len(gaps)}")
    xcc = st[:, 68].astype(np.int64) & 0xF
    for x in sorted(set(xcc.tolist())):
        sel = xcc == x
        print(f"  xcc {x}: loop end median {np.median(end_us[sel]):.2f} max {end_us[sel].max():.2f} us")


if __name__ == "__main__":
    main()
