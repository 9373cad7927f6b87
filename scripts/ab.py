"""Interleaved A/B timing of several builds of libfa_mi355x.so in ONE process.

    python scripts/ab.py [--config c3] [--rounds 10] lib_a.so lib_b.so ...

Each round times every library once (20 launches, HIP events), rounds interleaved so
clock / thermal drift hits all variants alike (cdna_hip_programming.md §5.4 rule 24).
Also checks each variant's output against the first one.
"""
import argparse
import ctypes
import statistics

import torch

CFG = {"c2": (32, 8, 1024, 32), "c3": (32, 8, 1024, 128), "c3s": (32, 8, 4096, 128),
       "c4": (32, 8, 4096, 128), "d256": (32, 8, 1024, 256), "d64": (32, 8, 1024, 64),
       "c3r": (32, 8, 1000, 128), "l512": (32, 8, 512, 128), "l2048": (32, 8, 2048, 128), "l8192": (8, 8, 8192, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--acc", action="store_true", help="also report the error against fp32")
    ap.add_argument("--all", action="store_true", help="print every round's time per library")
    ap.add_argument("--kvtpb", type=int, default=0, help="time fa_fwd_v2 with this kv_tiles_per_block")
    ap.add_argument("--bpw", type=int, default=0,
                    help="with --kvtpb: blocks_per_workgroup of fa_fwd_v2_ex (0 = the library's grouping)")
    ap.add_argument("--shape", default="", help="B,H,L,d instead of --config")
    ap.add_argument("--partial", action="store_true",
                    help="time fa_fwd_partial over all keys (scaled fp16 partials: the C5 per-rank kernel)")
    args = ap.parse_args()
    B, H, L, d = tuple(int(x) for x in args.shape.split(",")) if args.shape else CFG[args.config]
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    outs = [torch.empty_like(q) for _ in args.libs]
    libs = []
    for p in args.libs:
        h = ctypes.CDLL(p)
        h.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
        h.fa_fwd_v2.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 +
                                [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
        h.fa_fwd_partial.argtypes = ([ctypes.c_void_p] * 5 + [ctypes.c_int64] * 6 +
                                     [ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
        h.fa_fwd_v2_workspace_size.argtypes = [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [
            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
        h.fa_fwd_v2_workspace_size_ex.argtypes = [ctypes.c_int64] * 4 + [ctypes.c_int] * 4 + [
            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
        h.fa_fwd_v2_ex.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int] * 4 +
                                   [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_void_p] * 3 +
                                   [ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
        libs.append(h)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = None
    if args.kvtpb:  # FA-v2 split-KV (in-kernel combine), scaled fp16 partials
        nb, ns = ctypes.c_size_t(), ctypes.c_int()
        assert libs[0].fa_fwd_v2_workspace_size_ex(B, H, L, d, args.kvtpb, args.bpw, 1, 4, ctypes.byref(nb),
                                                   ctypes.byref(ns)) == 0
        ws = torch.zeros(nb.value, dtype=torch.uint8, device="cuda")  # (zeroed: A/B builds without the counter reset)
        print(f"v2: kv_tiles_per_block {args.kvtpb}, {ns.value} splits, workspace {nb.value / 1e9:.2f} GB")

    part = None
    if args.partial:
        part = [(torch.empty(B, H, L, d, dtype=torch.float16, device="cuda"),
                 torch.empty(B, H, L, 2, dtype=torch.float32, device="cuda")) for _ in libs]

    def run(i):
        if part is not None:
            st = libs[i].fa_fwd_partial(q.data_ptr(), k.data_ptr(), v.data_ptr(), part[i][0].data_ptr(),
                                        part[i][1].data_ptr(), B, H, L, L, d, L, 1, 4, stream)
            outs[i] = part[i][0]
        elif ws is not None:
            st = libs[i].fa_fwd_v2_ex(q.data_ptr(), k.data_ptr(), v.data_ptr(), outs[i].data_ptr(), B, H, L, d,
                                      min(32, d), min(32, d), args.kvtpb, args.bpw, ws.data_ptr(), ws.numel(),
                                      None, None, None, 1.0 / d ** 0.5, 1, 4, stream)
        else:
            st = libs[i].fa_fwd_v1(q.data_ptr(), k.data_ptr(), v.data_ptr(), outs[i].data_ptr(), B, H, L, d, 1, stream)
        assert st == 0, st

    for i in range(len(libs)):
        for _ in range(5):
            run(i)
    for _ in range(args.warmup):  # clock ramp: ~50 ms of back-to-back work first
        run(0)
    torch.cuda.synchronize()
    times = [[] for _ in libs]
    for _ in range(args.rounds):
        for i in range(len(libs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / args.iters)
    flops = 4.0 * B * H * L * L * d
    ref = None
    if args.acc:  # fp32 reference of the first 4 heads (scores materialised)
        qf, kf, vf = (x[:1, :4].float() for x in (q, k, v))
        ref = torch.softmax(qf @ kf.transpose(-1, -2) / d ** 0.5, dim=-1) @ vf
    for i, p in enumerate(args.libs):
        med = statistics.median(times[i])
        diff = (outs[i].float() - outs[0].float()).abs().max().item()
        acc = ""
        if ref is not None:
            err = (outs[i][:1, :4].float() - ref).abs()
            acc = f"  vs_fp32 max {err.max().item():.2e} mean {err.mean().item():.2e}"
        print(f"{p}: median {med * 1e3:.1f} us  min {min(times[i]) * 1e3:.1f} us  "
              f"{flops / (med * 1e-3) / 1e12:.1f} TFLOP/s  maxdiff_vs_0 {diff:.2e}{acc}", flush=True)
        if args.all:
            print("   rounds:", " ".join(f"{t * 1e3:.1f}" for t in times[i]), flush=True)


if __name__ == "__main__":
    main()
