"""MFMA ceiling on random vs constant operands, both shapes the kernels issue (libfa_probe.so).

    python scripts/mfma_peak.py > profiles/r05_mfma_peak_16x16x32.json

One JSON line per (shape, operand pattern, waves per SIMD): TFLOP/s over 20 back-to-back (~0.1 s each)
launches after 10 untimed ones, and the shader clock the chip held (csrc/fa_probe.hip).
"""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {0: "v_mfma_f32_32x32x16_bf16", 1: "v_mfma_f32_16x16x32_bf16"}
PATTERNS = {0: "constant small values", 1: "random, new (A, B) every MFMA",
            2: "random, A repeated in pairs (fa_fwd16_kernel's QK^T / P.V order)", 3: "random values, both constant"}


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "exploring_flash_attention_amd", "_lib", "libfa_probe.so"))
    lib.fa_probe_mfma_ceiling.argtypes = [ctypes.c_int] * 6 + [ctypes.POINTER(ctypes.c_double)]
    out = (ctypes.c_double * 3)()
    for shape in (1, 0):
        for pat in (1, 2, 3, 0):
            for wps in (2, 1):
                iters = 4000 if shape == 1 else 2000  # same FLOPs per launch for both shapes
                rc = lib.fa_probe_mfma_ceiling(shape, pat, wps, iters, 10, 20, out)
                assert rc == 0, rc
                print(json.dumps({"shape": SHAPES[shape], "operands": PATTERNS[pat], "waves_per_simd": wps,
                                  "tflops": round(out[0], 1), "held_clock_mhz": round(out[1]),
                                  "frac_of_2500": round(out[0] / 2500.0, 4),
                                  "loop": "4 independent accumulation chains per wave, nothing else"}), flush=True)


if __name__ == "__main__":
    main()
