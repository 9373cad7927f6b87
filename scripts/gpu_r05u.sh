# round 5, call u (u2): GPU suite
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05u2
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL|Error" $O/tests.log | tail -30; exit $rc
