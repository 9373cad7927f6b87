# round 5, calls n / final: GPU suite, smoke, default bench
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05final
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -22 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cat $O/bench.json; exit $rc
