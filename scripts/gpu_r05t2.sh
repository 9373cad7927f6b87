# round 5: the long split tests incl. the queued arrival-first shape
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05t2
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -v -k "long_sequence" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|long split" $O/tests.log | tail -12; exit $rc
