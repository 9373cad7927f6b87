"""Compact picture of a kernel's KV-loop step in the ISA (diagnostic).

    python scripts/isa_shape.py file.s [kernel-symbol-substring]

One letter per instruction between the loop header and the first two barriers:
M mfma, e v_exp, f v_fma, a v_add, x v_maximum3, c v_cvt_pk, r ds_read, D buffer_load (DMA),
w s_waitcnt, B s_cbranch, | s_barrier, v other VALU, s other SALU, n s_nop.
"""
import sys

CODES = [("v_mfma", "M"), ("v_exp", "e"), ("v_fma", "f"), ("v_pk_fma", "F"), ("v_add", "a"), ("v_pk_add", "A"),
         ("v_maximum", "x"), ("v_cvt_pk", "c"), ("ds_read", "r"), ("buffer_load", "D"), ("s_waitcnt", "w"),
         ("s_cbranch", "B"), ("s_barrier", "|"), ("s_nop", "n"), ("v_", "v"), ("s_", "s")]


def main():
    path = sys.argv[1]
    sym = sys.argv[2] if len(sys.argv) > 2 else "fa_fwd_kernelIDF16bDF16bLi128ELi0ELb0ELb0"
    lines = open(path).read().split("\n")
    start = next(i for i, x in enumerate(lines) if sym in x and x.split(":")[0].endswith("E") and x.endswith(
        x.split(":")[0] + ": ; @" + x.split(":")[0]) is False or (sym in x and x.startswith("_Z") and ":" in x))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    k = lines[start:end]
    hdr = next(i for i, x in enumerate(k) if "Loop Header" in x)
    bars = [i for i in range(hdr, len(k)) if "s_barrier" in k[i]]
    prev = hdr
    for b in bars[:2]:
        out = []
        for x in k[prev:b + 1]:
            t = x.strip().split()
            if not t or t[0].startswith((";", ".")):
                continue
            out.append(next((c for p, c in CODES if t[0].startswith(p)), ""))
        print("".join(out))
        print({c: "".join(out).count(c) for c in "MefaxcrDwn"})
        prev = b + 1


if __name__ == "__main__":
    main()
