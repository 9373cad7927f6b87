"""Phase anatomy of the persistent forward (fa_fwd_persist.hip) from an FA_STAMPS=1 build.

    bash scripts/build_variants.sh pqst "-DFA_PERSIST=1 -DFA_STAMPS=1"
    python scripts/stamps_persist.py [--config c3] exploring_flash_attention_amd/_lib/ab/pqst.so
"""
import argparse
import ctypes

import numpy as np
import torch

CFG = {"c2": (32, 8, 1024, 32), "c3": (32, 8, 1024, 128), "c4": (32, 8, 4096, 128),
       "l2048": (32, 8, 2048, 128), "d64": (32, 8, 1024, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warmup", type=int, default=400)
    args = ap.parse_args()
    B, H, L, d = CFG[args.config]
    lib = ctypes.CDLL(args.lib)
    lib.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
    lib.fa_debug_pq_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
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
    buf = np.zeros(4096 * 16, dtype=np.uint64)
    assert lib.fa_debug_pq_stamps(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(4096, 16).astype(np.int64)
    s = s[s[:, 5] > 0]
    life = s[:, 1] - s[:, 0]
    rt0 = s[:, 8].min()
    ent, end = (s[:, 8] - rt0) * 0.01, (s[:, 9] - rt0) * 0.01
    ntiles = (L + 63) // 64
    print(f"config {args.config}: {len(s)} workgroups x {np.median(s[:, 5]):.0f} items, launch {wall_us:.1f} us;"
          f" entries within {ent.max():.2f} us, ends {end.min():.1f} .. {end.max():.1f} us (median {np.median(end):.1f})")
    clk = np.median(life) / np.median(end - ent)
    print(f"  lifetime median {np.median(life):.0f} cycles ({clk / 1e3:.2f} GHz from realtime)")
    for nm, col in (("KV loops", 2), ("item prologues", 3), ("epilogues", 4)):
        print(f"  {nm:15s} {np.median(s[:, col]) / np.median(life):6.1%} of lifetime,"
              f" per item {np.median(s[:, col] / s[:, 5]):8.0f} cycles")
    print(f"  KV loop per step {np.median(s[:, 2] / s[:, 5]) / ntiles:.0f} cycles")
    xcc = s[:, 7] & 0xF
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcd {x}: ends {end[m].min():.1f} .. {end[m].max():.1f} us, loop/step median "
              f"{np.median(s[m, 2] / s[m, 5]) / ntiles:.0f} cycles")


if __name__ == "__main__":
    main()
