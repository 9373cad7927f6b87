#!/bin/bash
# SQ counters of the forward kernel for several builds of libfa_mi355x.so (A/B attribution).
# usage: bash scripts/pmc_compare.sh c3 lib1.so lib2.so ...   ->  gpurun_out/pmcab/<n>_p<i>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=$1; shift
OUT=gpurun_out/pmcab
mkdir -p $OUT
export TMPDIR=/tmp
n=0
for lib in "$@"; do
  n=$((n+1)); i=0
  for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
               "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    FA_MI355X_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d $OUT/${n}_p$i -o run \
        --output-format csv -- python scripts/run_kernel.py $CFG 5 > $OUT/${n}_p$i.log 2>&1; rc=$?
    echo "lib $lib pass $i rc=$rc"
    case $rc in 0) ;; *) tail -5 $OUT/${n}_p$i.log; exit $rc ;; esac
  done
done
