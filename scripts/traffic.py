"""Summarise the PMC passes of scripts/profile_pmc.sh into per-launch HBM traffic.

    python scripts/traffic.py gpurun_out/pmc_c3 c3 [out.json [source label]]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts exactly half
the bytes of a wide (16 B/lane) coalesced read stream -- every read of the forward kernel
is one (buffer_load_dwordx4, buffer_load_dwordx4 ... lds) -- so the read side is doubled
(MI355X_MICROARCH.md, HBM).  WRITE_SIZE is exact for 16-B-per-lane stores and is taken as
is for the kernel's 8-B stores (uncalibrated).
"""
import csv
import glob
import json
import os
import re
import sys


def main():
    d, cfg = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    vals, kernels = {}, set()
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if not re.search(r"fa_fwd(16|16_chain|_dtp?)?_kernel", r["Kernel_Name"]):
                continue
            kernels.add(r["Kernel_Name"].split("(")[0])
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    fetch = mean.get("FETCH_SIZE")
    write = mean.get("WRITE_SIZE")
    rec = {"counters_mean": mean, "kernels": sorted(kernels)}
    if fetch is not None and write is not None:
        rec["read_bytes_per_launch"] = 2 * fetch * 1024
        rec["write_bytes_per_launch"] = write * 1024
        rec["bytes_per_launch"] = 2 * fetch * 1024 + write * 1024
        rec["method"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024, rocprofv3 --pmc, separate passes"
    res = {cfg: rec}
    if out:
        old = {}
        if os.path.exists(out):
            old = json.load(open(out))
        prev = old.get(cfg, {})
        # keep the entry's labels (kernel, algorithmic bytes), record where the new counters
        # came from and what the entry said before
        for key in ("kernel", "algorithmic_bytes"):
            if key in prev:
                rec[key] = prev[key]
        if "algorithmic_bytes" in rec and "bytes_per_launch" in rec:
            rec["ratio_to_algorithmic"] = round(rec["bytes_per_launch"] / rec["algorithmic_bytes"], 3)
        rec["source"] = sys.argv[4] if len(sys.argv) > 4 else d
        if "bytes_per_launch" in prev:
            rec["previous"] = {k: prev[k] for k in ("bytes_per_launch", "kernel", "source") if k in prev}
        old[cfg] = rec
        json.dump(old, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
