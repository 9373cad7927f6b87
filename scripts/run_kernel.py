"""Launch one forward configuration a few times (for rocprofv3 runs).

    python scripts/run_kernel.py [c2|c3|c4|c5] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from exploring_flash_attention_amd import ops  # noqa: E402

CFG = {"c2": (32, 8, 1024, 32, "v1"), "c3": (32, 8, 1024, 128, "v1"),
       "c4": (32, 8, 4096, 128, "v2"), "c5": (32, 8, 16384, 128, "v1")}
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, H, L, d, var = CFG[name]
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
for _ in range(iters):
    if var == "v1":
        ops.attention_v1(q, k, v)
    else:
        ops.attention_v2(q, k, v, 4)
torch.cuda.synchronize()
print("done", name, iters)
