set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05a
export PYTHONPATH=$PWD
timeout -k 10 120 python -u scripts/mfma_peak.py > gpurun_out/r05a/mfma_peak.json 2> gpurun_out/r05a/mfma_peak.err || exit $?
cat gpurun_out/r05a/mfma_peak.json
timeout -k 10 400 python -u -m pytest tests/test_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a/fullsize.log 2>&1; rc=$?
tail -25 gpurun_out/r05a/fullsize.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/dtile_sweep.py > gpurun_out/r05a/dtile_sweep.txt 2>&1 || exit $?
cat gpurun_out/r05a/dtile_sweep.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err; rc=$?
cat gpurun_out/r05a/bench.json; tail -3 gpurun_out/r05a/bench.err; exit $rc
