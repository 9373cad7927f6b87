"""Compare one build of libfa_mi355x.so with a torch fp32 attention on a small shape and
print where the errors are (rows / columns pattern).  Debug aid for kernel variants.

    python scripts/debug_cmp.py lib.so [B H L d]
"""
import ctypes
import sys

import torch

lib = ctypes.CDLL(sys.argv[1])
lib.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
B, H, L, d = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (1, 1, 256, 128)
g = torch.Generator(device="cuda").manual_seed(0)
for name, scale in (("randn", 1.0), ("peaked", 4.0)):
    q, k, v = (torch.randn(B, H, L, d, device="cuda", generator=g) for _ in range(3))
    q = q * scale
    qb, kb, vb = (t.to(torch.bfloat16) for t in (q, k, v))
    o = torch.empty_like(qb)
    st = lib.fa_fwd_v1(qb.data_ptr(), kb.data_ptr(), vb.data_ptr(), o.data_ptr(), B, H, L, d, 1,
                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert st == 0
    ref = torch.softmax(qb.float() @ kb.float().transpose(-1, -2) / d ** 0.5, -1) @ vb.float()
    err = (o.float() - ref).abs()[0, 0]
    print(f"[{name}] max err {err.max().item():.3e}")
    rows = err.max(dim=1).values
    bad = (rows > 2e-2).nonzero().flatten().tolist()
    print(f"  bad rows ({len(bad)}): {bad[:64]}")
    cols = err.max(dim=0).values
    badc = (cols > 2e-2).nonzero().flatten().tolist()
    print(f"  bad cols ({len(badc)}): {badc[:64]}")
    if bad:
        r = bad[0]
        print("  row", r, "ratio o/ref first 16:", (o.float()[0, 0, r, :16] / ref[0, 0, r, :16]).tolist())
