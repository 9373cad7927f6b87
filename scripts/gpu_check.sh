#!/bin/bash
# One GPU-box pass: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first crash / timeout (exit codes 124, 134, 137, 139) so a faulting
# kernel is never launched twice in one call.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_if_crash() {  # $1 = exit code, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "STEP $2 exited $1 -- stopping"; exit "$1" ;;
  esac
}
STEPS="${STEPS:-smoke tests bench prof}"
for s in $STEPS; do
  case "$s" in
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -5 $OUT/smoke.log; stop_if_crash $rc smoke
      [ $rc -eq 0 ] || exit 1 ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread ${PYTEST_ARGS:--x} > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log; stop_if_crash $rc tests ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err; stop_if_crash $rc bench ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python bench.py --no-cpu-baseline --no-extra > $OUT/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -3 $OUT/prof.log; stop_if_crash $rc prof
      find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20 ;;
  esac
done
