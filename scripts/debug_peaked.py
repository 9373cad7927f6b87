# Peaked-row error vs the rounding floor (P and O rounded to the input type), per head dim.
# python scripts/debug_peaked.py  (GPU)
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
from exploring_flash_attention_amd import ops
from oracle.batched import attention_fp64
gpu = torch.device("cuda", 0)
for dtype in (torch.bfloat16, torch.float16):
  for d in (32, 64, 128, 256):
    for order in ("rising", "falling", "none"):
        g = torch.Generator().manual_seed(31)
        B, H, L = 1, 2, 1000
        q, k, v = (torch.randn(B, H, L, d, generator=g) for _ in range(3))
        ramp = torch.arange(L, dtype=torch.float32) / 16.0
        if order == "falling": ramp = ramp.flip(0)
        if order != "none":
            q[..., 0] = 16.0 * (d / 128) ** 0.5
            k[..., 0] = ramp
        q, k, v = (x.to(dtype) for x in (q, k, v))
        ref = attention_fp64(q.double().numpy(), k.double().numpy(), v.double().numpy())
        s = (q.double() @ k.double().transpose(-1, -2)) / d ** 0.5
        p = torch.exp(s - s.amax(-1, keepdim=True))
        emu = ((p.to(dtype).double() @ v.double()) / p.sum(-1, keepdim=True)).to(dtype).double()
        emu_err = (emu - torch.from_numpy(ref)).abs().max().item()
        o = ops.attention_v1(q.to(gpu), k.to(gpu), v.to(gpu)); torch.cuda.synchronize()
        err = np.abs(o.double().cpu().numpy() - ref).max()
        # where is the max error: row, col
        e = np.abs(o.double().cpu().numpy() - ref); idx = np.unravel_index(e.argmax(), e.shape)
        print(f"{str(dtype)[6:]} d={d} {order:7s} err={err:.2e} emu={emu_err:.2e} ratio={err/emu_err:.1f} at {idx} ref={ref[idx]:.3f}")
