"""Compare two libfa_mi355x.so builds' forward outputs on a set of shapes (A/B correctness aid):
both against a torch fp32 reference and against each other, for fa_fwd_v1 and
fa_fwd_v1_tiled_d with several tile pairs.

    python scripts/cmp_libs.py A.so B.so [d]
"""
import ctypes
import sys

import torch


def main():
    libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 384
    for h in libs:
        h.fa_fwd_v1_tiled_d.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    worst = 0.0
    for (B, H, L, dt) in [(2, 3, 200, torch.bfloat16), (1, 2, 1000, torch.bfloat16), (2, 2, 256, torch.float16),
                          (1, 1, 64, torch.bfloat16), (1, 2, 130, torch.float16), (4, 4, 1024, torch.bfloat16)]:
        g = torch.Generator(device="cuda").manual_seed(L + B)
        q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=dt, generator=g) for _ in range(3))
        ref = torch.softmax(q.float() @ k.float().transpose(-1, -2) / d ** 0.5, dim=-1) @ v.float()
        code = 1 if dt == torch.bfloat16 else 0
        for tq, tv in [(128, 128), (64, 64), (32, 64), (64, 32), (32, 32)]:
            outs = []
            for h in libs:
                o = torch.empty_like(q)
                st = h.fa_fwd_v1_tiled_d(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, tq, tv,
                                         code, stream)
                assert st == 0, st
                outs.append(o)
            torch.cuda.synchronize()
            errs = [(o.float() - ref).abs().max().item() for o in outs]
            ab = (outs[0].float() - outs[1].float()).abs().max().item()
            worst = max(worst, errs[1])
            print(f"B{B} H{H} L{L} {str(dt)[6:]} tiles {tq}/{tv}: err A {errs[0]:.2e} B {errs[1]:.2e} |A-B| {ab:.2e}",
                  flush=True)
    print("worst B err", worst)
    assert worst < 1e-2


if __name__ == "__main__":
    main()
