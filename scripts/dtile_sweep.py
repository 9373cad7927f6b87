"""Time the d-tiled forward at B32 H8 L1024 for d = 384 / 512 over its tile choices
(ops.attention_tiled_d; every choice gives the same bits), interleaved rounds, medians.

    python scripts/dtile_sweep.py [--rounds 8]
"""
import argparse
import statistics

import torch

from exploring_flash_attention_amd import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    B, H, L = 32, 8, 1024
    for d in (384, 512):
        g = torch.Generator(device="cuda").manual_seed(d)
        q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
        tiles = [(None, None), (32, 32), (64, 64), (128, 128), (64, 128), (128, 64)]
        outs = {}
        for t in tiles:
            outs[t] = ops.attention_tiled_d(q, k, v, *t)
        for _ in range(30):
            ops.attention_tiled_d(q, k, v, 128, 128)
        times = {t: [] for t in tiles}
        for _ in range(args.rounds):
            for t in tiles:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    ops.attention_tiled_d(q, k, v, *t)
                e1.record()
                torch.cuda.synchronize()
                times[t].append(e0.elapsed_time(e1) / args.iters)
        fl = 4.0 * B * H * L * L * d
        for t in tiles:
            med = statistics.median(times[t])
            same = torch.equal(outs[t], outs[(128, 128)])
            print(f"d={d} tiles={t}: {med:.4f} ms  {fl / med / 1e9:.1f} TFLOP/s  frac {fl / med / 1e9 / 2500:.3f}"
                  f"  bitwise_equal_128={same}", flush=True)


if __name__ == "__main__":
    main()
