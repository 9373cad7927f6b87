#!/bin/bash
# A batch of GPU steps in one gpurun call (STEPS="tests bench peak ab stamps pmc" ...), each under
# its own time limit; stops at the first crash / timeout (exit codes other than 0 and 1).
#   AB_LIBS="lbase.so lpin.so" AB_CONFIGS="c3 c4" STAMP_LIBS="lstamp_base.so:c3" PMC_CONFIGS="c3"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_crash() {
  case "$1" in 0|1) return 0 ;; *) echo "STEP $2 exited $1 -- stopping"; exit "$1" ;; esac
}
for s in ${STEPS:-tests}; do
  case "$s" in
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -4 $OUT/smoke.log; stop_if_crash $rc smoke ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x \
          > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -6 $OUT/pytest_gpu.log; stop_if_crash $rc tests ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_if_crash $rc bench ;;
    peak)
      timeout -k 10 60 ./scripts/bin/mfma_peak > $OUT/mfma_peak.json; rc=$?
      echo "peak rc=$rc"; cat $OUT/mfma_peak.json; stop_if_crash $rc peak ;;
    ab)
      libs=()
      for n in ${AB_LIBS}; do libs+=("exploring_flash_attention_amd/_lib/ab/$n"); done
      for c in ${AB_CONFIGS:-c3}; do
        echo "== ab $c"
        timeout -k 10 240 python scripts/ab.py --config $c --rounds ${ROUNDS:-10} ${AB_ARGS:-} "${libs[@]}" \
            > $OUT/ab_$c.log 2>&1; rc=$?
        grep -v amdgpu.ids $OUT/ab_$c.log; stop_if_crash $rc ab
      done ;;
    stamps)
      for lc in ${STAMP_LIBS}; do
        lib=${lc%%:*}; cfg=${lc##*:}
        echo "== stamps $lib $cfg"
        timeout -k 10 120 python scripts/stamps.py --config $cfg exploring_flash_attention_amd/_lib/ab/$lib \
            > $OUT/stamps_${lib%.so}_$cfg.log 2>&1; rc=$?
        grep -v amdgpu.ids $OUT/stamps_${lib%.so}_$cfg.log; stop_if_crash $rc stamps
      done ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python bench.py --no-cpu-baseline --no-extra > $OUT/prof_bench.json 2> $OUT/prof.log; rc=$?
      echo "prof rc=$rc"; cat $OUT/prof_bench.json; stop_if_crash $rc prof
      find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -5 ;;
    pmc)
      for cfg in ${PMC_CONFIGS:-c3}; do
        bash scripts/profile_pmc.sh $cfg; rc=$?
        stop_if_crash $rc pmc
        python scripts/traffic.py $OUT/pmc_$cfg $cfg $OUT/hbm_traffic_r03.json | head -30
      done ;;
  esac
done
