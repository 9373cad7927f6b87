#!/bin/bash
# Targeted GPU pass: the given pytest selection, then (optionally) the bench.
#   TESTS="tests/test_fullsize.py" BENCH=1 bash scripts/gpu_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_quick.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/pytest_quick.log | tail -30
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
