"""Split-KV partials-per-tile sweep on small-batch shapes (one process, product library).

    python scripts/split_sweep.py

For each shape, times ops.attention_v2 with blocks_per_workgroup fixing 1, 2, 4, 8, 16
partials per query tile (KV_TILES_PER_BLOCK = 1: 64-key blocks), interleaved over rounds, and
prints the median ms of each and the library's own choice (blocks_per_workgroup = None).
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from exploring_flash_attention_amd import ops  # noqa: E402

SHAPES = [(1, 1, 16384), (1, 2, 16384), (1, 1, 8192), (1, 2, 4096), (1, 4, 4096), (2, 2, 16384), (1, 8, 2048)]


def main():
    dev = torch.device("cuda", 0)
    for B, H, L in SHAPES:
        d = 128
        g = torch.Generator(device=dev).manual_seed(0)
        q, k, v = (torch.randn(B, H, L, d, device=dev, dtype=torch.bfloat16, generator=g) for _ in range(3))
        blocks = L // 64
        variants = {"lib": None}
        for p in (1, 2, 4, 8, 16):
            if blocks % p == 0:
                variants[f"p{p}"] = blocks // p
        runs = {}
        for name, bpw in variants.items():
            nb, _ = ops.v2_workspace_bytes(B, H, L, d, 1, q.dtype, blocks_per_workgroup=bpw)
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            o = torch.empty_like(q)
            plan = ops.v2_split_plan(B, H, L, d, 1, q.dtype, blocks_per_workgroup=bpw)
            runs[name] = (bpw, ws, o, plan)
        times = {n: [] for n in runs}
        for _ in range(200):  # clock ramp
            ops.attention_v2(q, k, v, 1, out=runs["lib"][2], workspace=runs["lib"][1])
        for _ in range(8):
            for n, (bpw, ws, o, plan) in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ops.attention_v2(q, k, v, 1, out=o, workspace=ws, blocks_per_workgroup=bpw)
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / 20)
        flops = 4.0 * B * H * L * L * d
        ref = runs["lib"][2]
        parts = []
        for n, ts in times.items():
            ms = statistics.median(ts)
            same = torch.allclose(runs[n][2].float(), ref.float(), atol=2e-2, rtol=0)
            parts.append(f"{n}(ppt={runs[n][3][2]}) {ms * 1e3:.1f}us {flops / ms / 1e9:.0f}TF{'' if same else ' MISMATCH'}")
        print(f"B{B} H{H} L{L}: " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
