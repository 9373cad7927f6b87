"""Launch fa_fwd_v1 of a given libfa_mi355x.so build a few times at one shape (for rocprofv3
PMC passes over A/B builds, e.g. scripts/build_lite.sh outputs).

    python scripts/run_lib.py LIB.so B,H,L,d [iters]
"""
import ctypes
import sys

import torch


def main():
    lib = ctypes.CDLL(sys.argv[1])
    B, H, L, d = (int(x) for x in sys.argv[2].split(","))
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    lib.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(iters):
        assert lib.fa_fwd_v1(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, 1, s) == 0
    torch.cuda.synchronize()
    print("done", sys.argv[2], iters)


if __name__ == "__main__":
    main()
