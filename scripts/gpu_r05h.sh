# round 5, call h: fused-chain A/B, then the full GPU suite, MFMA ceiling, d-tile sweep, bench
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05h
mkdir -p $O
export PYTHONPATH=$PWD
bash scripts/gpu_r05g.sh || exit $?
mkdir -p $O && cp -r gpurun_out/r05g/* $O/ 2>/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mfma_peak.py > $O/mfma_peak.json 2> $O/mfma_peak.err || exit $?
cat $O/mfma_peak.json
timeout -k 10 200 python -u scripts/dtile_sweep.py > $O/dtile_sweep.txt 2>&1 || exit $?
cat $O/dtile_sweep.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -3 $O/bench.err; exit $rc
