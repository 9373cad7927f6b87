"""Check the hand-counted `s_waitcnt vmcnt(N)` + `s_barrier` pairs of the chained d = 128 kernel
(fa_fwd16_chain.hpp) in its gfx950 ISA.

    python scripts/check_vmcnt.py file.s        # exit status 1 on a violation

vmcnt(N) lets the N youngest vector-memory operations (loads, stores and LDS-DMA pieces count
together, in issue order; MI355X_MICROARCH.md) stay in flight.  The kernel counts N by hand in
three places; each is correct only if code generation issued at least N operations of the
intended kind after the LDS-DMA pieces the barrier must see landed:
  * EPI step (an item's first step):  N = the previous item's O stores issued behind the step's
    DMA pieces -- the N youngest must all be stores;
  * QNEXT step:                       N = 8 loads of the next item's Q^T issued in phase B, after
    the step's DMA pieces -- the N youngest must all be plain (non-LDS) loads;
  * the first prologue:               N = 2 * DPW: V(0) and K(1) may stay in flight, Q and K(0)
    must not -- the N youngest must all be LDS-DMA pieces and a plain (Q) load or further
    pieces (K(0)) must lie behind them.
A wait preceded, before N operations are found, by a compiler-placed vmcnt(0) is moot (the
fused walk's per-tile prologue: the compiler drains its Q^T loads there); one whose N youngest
operations are not all in the straight-line code before it (a label in between, several paths
reaching it) is reported as a violation -- it cannot be checked from one path.
"""
import re
import sys

VMEM = re.compile(r"(buffer_|global_|flat_|scratch_)")


def kind(line):
    op = line.split()[0]
    if " lds" in line:
        return "dma"
    if "store" in op or "atomic" in op:
        return "store"
    return "load"


def check(path):
    lines = open(path).read().split("\n")
    kernel, bad, rows = None, 0, []
    for i, ln in enumerate(lines):
        if re.match(r"^_ZN\w+:", ln):
            kernel = ln.split(":")[0]
        m = re.match(r"\s*s_waitcnt vmcnt\((\d+)\)\s*$", ln)
        if not m or kernel is None or "chain" not in kernel:
            continue
        nxt = [x for x in lines[i + 1:i + 4] if x.strip() and not x.strip().startswith(";")]
        if not nxt or "s_barrier" not in nxt[0]:
            continue  # a compiler-placed wait
        n = int(m.group(1))
        if n == 0:
            continue
        kinds, j, crossed, drained = [], i - 1, False, False
        while j > 0 and len(kinds) < n + 1:
            s = lines[j]
            if re.match(r"\s*s_waitcnt vmcnt\(0\)\s*$", s):
                drained = True  # everything older has landed: the hand count is moot
                break
            if s.startswith(".LBB") or s.startswith("_ZN"):
                crossed = True
                break
            t = s.strip()
            if t and VMEM.match(t):
                kinds.append(kind(t))
            j -= 1
        young = kinds[:n]
        older = kinds[n] if len(kinds) > n else None
        if drained and len(young) < n:
            verdict = "drained by an earlier vmcnt(0): ok"
        elif crossed and len(young) < n:
            verdict = "VIOLATION (path-dependent: not all N operations in straight-line code)"
            bad += 1
        elif all(k == "store" for k in young):
            verdict = "EPI: ok" if older in ("dma", "store", None) else "EPI: ok (over-waits)"
        elif all(k == "load" for k in young):
            verdict = "QNEXT: ok"
        elif all(k == "dma" for k in young) and older in ("dma", "load"):
            verdict = "prologue: ok"
        else:
            verdict = "VIOLATION"
            bad += 1
        rows.append(f"{kernel[:48]} line {i + 1}: vmcnt({n}) youngest {young} older {older} -> {verdict}")
    return bad, rows


def main():
    bad, rows = check(sys.argv[1])
    print("\n".join(rows))
    print(f"{len(rows)} hand-counted waits, {bad} violations")
    sys.exit(1 if bad or not rows else 0)


if __name__ == "__main__":
    main()
