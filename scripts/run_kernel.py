"""Launch one forward configuration a few times (for rocprofv3 runs).

    python scripts/run_kernel.py [config] [iters]

configs: c2, c3 (FA-v1), c4 (split-KV, KV_TILES_PER_BLOCK = 4, the library's grouping), c4g4 /
c4g1 (C4 with 4 / 1 key blocks per workgroup: 4 / 16 partials per query tile), b1h1l16k (a
shape the library splits itself: 4 partials per query tile since round 4's plan, 2 before),
b1h2l16k (2 partials per tile; 1 before), b1h1l16k_unsplit (the same shape,
one workgroup per query tile), b1h2l4k / _unsplit (4 partials per tile / none), c5 (one rank's
C5 partial kernel shape, FA-v1 form), b2h2l16k (16 partials per tile: the fused chain's walk),
d384 / d512 (the d-tiled kernel at B32 H8 L1024).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from exploring_flash_attention_amd import ops  # noqa: E402

CFG = {"c2": (32, 8, 1024, 32, "v1", None), "c3": (32, 8, 1024, 128, "v1", None),
       "c4": (32, 8, 4096, 128, "v2", None), "c4g4": (32, 8, 4096, 128, "v2", 4),
       "c4g1": (32, 8, 4096, 128, "v2", 1), "b1h1l16k": (1, 1, 16384, 128, "v2", None),
       "b1h1l16k_unsplit": (1, 1, 16384, 128, "v2", 64),
       "b1h2l16k": (1, 2, 16384, 128, "v2", None), "c5": (32, 8, 16384, 128, "v1", None),
       "b1h2l4k": (1, 2, 4096, 128, "v2", None), "b1h2l4k_unsplit": (1, 2, 4096, 128, "v2", 16),
       "b2h2l16k": (2, 2, 16384, 128, "v2", 4),
       "d384": (32, 8, 1024, 384, "td", None), "d512": (32, 8, 1024, 512, "td", None)}
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, H, L, d, var, grp = CFG[name]
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
out = torch.empty_like(q)
ws = None
if var == "v2":
    nb, _ = ops.v2_workspace_bytes(B, H, L, d, 4, q.dtype, blocks_per_workgroup=grp)
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
for _ in range(iters):
    if var == "v1":
        ops.attention_v1(q, k, v, out=out)
    elif var == "td":  # the d-tiled kernel, 128-column K / V chunks
        ops.attention_tiled_d(q, k, v, 128, 128, out=out)
    else:
        ops.attention_v2(q, k, v, 4, out=out, workspace=ws, blocks_per_workgroup=grp)
torch.cuda.synchronize()
print("done", name, iters)
