"""Tail model of the chained C3 grid (fa_fwd16_chain.hpp): what rebalancing the last items
could buy, before any GPU time is spent on it.

    python scripts/tail_model.py            # table -> profiles/r06/tail_model.txt

Measured inputs (profiles/r05/seam/stamps_c3_chain*.txt):
  * 2 workgroups per CU, 4 items of 16 KV steps each; a step takes ~1.70 us of a workgroup's
    life while the CU's other workgroup runs (2640-3000 cycles at ~1.7 GHz);
  * seam per item ~2900 cycles = 1.0 step;
  * the first-dispatched workgroup of a CU ends a median 10.1 us before its partner: while
    both run it gets 0.541 of the CU's rate (solves 4 items by X - 5 us, the partner 4 by
    X + 5 us with 0.88 of the pair rate alone at the end);
  * a workgroup alone on its CU runs at 0.88 of the pair's rate (round-3 measurement);
  * per-XCD loop-end medians 108.8 ... 114.6 us: the XCDs' speeds differ by that ratio.
Dynamic variants: the last items cut into `parts` key ranges claimed from one global queue,
each costing 16/parts steps + the seam + `split` steps (partial store + combine of a split
tile) + `claim` steps (a returning device-scope atomic under load: ~6k cycles = ~2 steps,
round 2's measurement).  The split cost measured in round 6 (scripts/split_stamps.py,
profiles/r06/split_stamps_*.txt): loop end -> hand-off verdict 1.1-2.4 us, the combine of 2
partials + O 2.7 + 0.4 us -> ~2.6 steps of 1.7 us on the last piece of a tile (the `measured`
rows); 0.5 is a lower bound.
"""
import os
import statistics

STEP_US = 1.70          # one workgroup's step while the CU is shared
SEAM = 1.0              # steps of seam per item
SHARE_A = 0.541         # the first-dispatched workgroup's share of its CU
ALONE = 0.88            # a lone workgroup's rate, relative to the pair's
XCD_MEDIANS = [111.5, 112.2, 108.8, 113.4, 110.5, 114.6, 112.7, 114.0]  # us, stamps_c3_chain_pairs
CUS_PER_XCD = 32


def simulate(static_items=4, parts=1, split=0.0, claim=0.0, dt=0.01):
    """Loop-end times (us) of all 512 workgroups: `static_items` items from the static lists,
    then (parts > 1) the remaining items' key ranges from a global queue."""
    mean = statistics.mean(XCD_MEDIANS)
    wgs = []
    for xm in XCD_MEDIANS:
        speed = mean / xm
        for _ in range(CUS_PER_XCD):
            wgs.append({"speed": speed, "share": SHARE_A, "static": static_items, "done": False})
            wgs.append({"speed": speed, "share": 1 - SHARE_A, "static": static_items, "done": False})
    total_items = 4 * len(wgs)
    pool = (total_items - static_items * len(wgs)) * parts if parts > 1 else 0

    def next_work(w):
        nonlocal pool
        if w["static"] > 0:
            w["static"] -= 1
            return 16 + SEAM
        if pool > 0:
            pool -= 1
            return 16 / parts + SEAM + split + claim
        return None

    for w in wgs:
        w["rem"] = next_work(w)
    t, active = 0.0, len(wgs)
    while active:
        for i in range(0, len(wgs), 2):
            a, b = wgs[i], wgs[i + 1]
            both = not a["done"] and not b["done"]
            for w in (a, b):
                if w["done"]:
                    continue
                rate = (2 * w["share"] if both else 2 * ALONE) * w["speed"] / STEP_US  # steps per us
                w["rem"] -= rate * dt
                while w["rem"] <= 0:
                    nw = next_work(w)
                    if nw is None:
                        w["done"], w["end"] = True, t
                        active -= 1
                        break
                    w["rem"] += nw
        t += dt
    ends = [w["end"] for w in wgs]
    return max(ends), statistics.median(ends), min(ends)


def main():
    rows = [("static lists (shipped)", dict())]
    for k in (3, 2):
        for parts in (2, 4):
            for split, claim in ((0.0, 0.0), (0.5, 0.0), (0.5, 2.0), (2.6, 0.0), (2.6, 2.0)):
                rows.append((f"{k} static + {4 - k} items as {parts} key ranges, split {split}, claim {claim}",
                             dict(static_items=k, parts=parts, split=split, claim=claim)))
    out = ["C3 chained grid, modelled loop ends (us): max (= the kernel's end) / median / min",
           "seam {:.1f} step per item; a key-range piece pays the seam again plus split + claim steps".format(SEAM)]
    for name, kw in rows:
        mx, med, mn = simulate(**kw)
        out.append(f"  {name:62s} {mx:6.1f} / {med:6.1f} / {mn:6.1f}")
    # the bound: the same work perfectly balanced over every CU's pair rate, no overheads
    mean = statistics.mean(XCD_MEDIANS)
    rate = sum(2 * (mean / xm) / STEP_US * CUS_PER_XCD for xm in XCD_MEDIANS)  # steps per us, all CUs
    work = 4 * 2 * CUS_PER_XCD * len(XCD_MEDIANS) * (16 + SEAM)
    out.append(f"  bound: the same work spread perfectly over every CU (no split cost)  {work / rate:6.1f}")
    text = "\n".join(out)
    print(text)
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06",
                       "tail_model.txt")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        f.write(text + "\n")


if __name__ == "__main__":
    main()
