"""Time FA-v2 (split-KV, in-kernel combine) over split sizes and partial dtypes.

    python scripts/v2_sweep.py [B H L d]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from exploring_flash_attention_amd import ops  # noqa: E402

B, H, L, d = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (32, 8, 4096, 128)
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
flops = 4.0 * B * H * L * L * d
ref = ops.attention_v1(q, k, v)
for _ in range(100):
    ops.attention_v1(q, k, v)
for kvt in (1, 2, 4, 8, 16, "auto"):
    for pd in (torch.float32, torch.bfloat16):
        nb, ns = ops.v2_workspace_bytes(B, H, L, d, kvt, q.dtype, pd)
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            o = ops.attention_v2(q, k, v, kvt, partial_dtype=pd, workspace=ws)
        n = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            ops.attention_v2(q, k, v, kvt, partial_dtype=pd, workspace=ws)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        err = (o.float() - ref.float()).abs().max().item()
        print(f"kvtpb={kvt!s:>4} splits={ns:3d} partial={str(pd)[6:]:8s} ws={nb / 1e9:6.2f} GB "
              f"{ms:8.3f} ms {flops / ms / 1e9:8.1f} TFLOP/s  maxdiff_vs_v1 {err:.1e}", flush=True)
        del ws
