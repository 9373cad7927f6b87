"""Our forward against the ROCm vendor flash-attention kernels PyTorch ships, in ONE process.

    python scripts/vendor_sdpa.py [--configs c3 c2 c4] [--rounds 8] [--json out.json]

torch.nn.functional.scaled_dot_product_attention is the reference's own PyTorch path
(flash_attention_v1/pytorch_imp.py:12).  On ROCm its flash backend is AOTriton by default and
composable_kernel (CK) when preferred (torch.backends.cuda.preferred_rocm_fa_library).  Each
variant is timed over interleaved rounds (HIP events on the current stream, the clock settled
first by ~0.2 s of back-to-back work) on the same bf16 [B, H, L, d] inputs, and its output is
compared with ours.  A backend that refuses the shape is reported as such.
"""
import argparse
import json
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from exploring_flash_attention_amd import ops  # noqa: E402

CFG = {"c2": (32, 8, 1024, 32), "c3": (32, 8, 1024, 128), "c4": (32, 8, 4096, 128),
       "d64": (32, 8, 1024, 64), "l2048": (32, 8, 2048, 128), "b1h1l16k": (1, 1, 16384, 128)}


def sdpa_fn(lib):
    from torch.nn.attention import SDPBackend, sdpa_kernel

    def run(q, k, v):
        torch.backends.cuda.preferred_rocm_fa_library(lib)
        with sdpa_kernel([SDPBackend.FLASH_ATTENTION]):
            return F.scaled_dot_product_attention(q, k, v)
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c3", "c2", "c4"])
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    results = {}
    for cfg in args.configs:
        B, H, L, d = CFG[cfg]
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
        flops = 4.0 * B * H * L * L * d
        iters = max(5, min(50, int(1e13 / flops)))
        ours_out = torch.empty_like(q)
        variants = {"ours": lambda: ops.attention_v1(q, k, v, out=ours_out)}
        for lib in ("aotriton", "ck"):
            fn = sdpa_fn(lib)
            try:
                o = fn(q, k, v)
                torch.cuda.synchronize()
                variants[f"sdpa_flash_{lib}"] = (lambda fn=fn: fn(q, k, v))
                results.setdefault(cfg, {})[f"sdpa_flash_{lib}_maxdiff_vs_ours"] = None
                del o
            except Exception as exc:  # noqa: BLE001 -- reported
                results.setdefault(cfg, {})[f"sdpa_flash_{lib}"] = {"error": f"{type(exc).__name__}: {exc}"[:200]}
        torch.backends.cuda.preferred_rocm_fa_library("default")
        t0 = time.perf_counter()  # clock settle
        while time.perf_counter() - t0 < 0.2:
            for fn in variants.values():
                fn()
            torch.cuda.synchronize()
        times = {n: [] for n in variants}
        outs = {}
        for _ in range(args.rounds):
            for n, fn in variants.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    r = fn()
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / iters)
                outs[n] = ours_out if n == "ours" else r
        rec = results.setdefault(cfg, {"B": B, "H": H, "L": L, "d": d})
        rec.update({"B": B, "H": H, "L": L, "d": d})
        for n in variants:
            med = statistics.median(times[n])
            rec[n] = {"ms": round(med, 4), "min_ms": round(min(times[n]), 4),
                      "tflops": round(flops / (med * 1e-3) / 1e12, 1)}
            if n != "ours":
                rec[n]["maxdiff_vs_ours"] = float((outs[n].float() - ours_out.float()).abs().max())
                rec[n]["ours_speedup"] = round(med / statistics.median(times["ours"]), 3)
                rec.pop(f"{n}_maxdiff_vs_ours", None)
        print(cfg, json.dumps(rec), flush=True)
        del q, k, v, outs, variants
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
