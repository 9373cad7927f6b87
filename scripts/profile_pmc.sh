#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only, never with sys/runtime trace)
# over scripts/run_kernel.py.  Usage: bash scripts/profile_pmc.sh [config] [name] ; output
# gpurun_out/pmc_<name>/ (name defaults to the config)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=${1:-c3}
NAME=${2:-$CFG}
OUT=gpurun_out/pmc_$NAME
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $group -d $OUT/p$i -o run --output-format csv -- \
     python scripts/run_kernel.py $CFG 5 > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i ($group) rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc ;; esac
done
