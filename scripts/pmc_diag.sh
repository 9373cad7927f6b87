#!/bin/bash
# Issue / wait breakdown PMC passes of one config (diagnostic): gpurun_out/pmc_diag_<cfg>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=${1:-c3}
OUT=gpurun_out/pmc_diag_$CFG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for group in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d $OUT/p$i -o run --output-format csv -- \
     python scripts/run_kernel.py $CFG 5 > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "fa_fwd_kernel" in row.get("Kernel_Name", "") or "fa_fwd16_kernel" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
