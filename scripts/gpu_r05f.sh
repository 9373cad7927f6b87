# round 5, call f: full GPU suite with the chained kernel + new tests, peak, d-tile sweep, bench,
# B1H1 L16k traffic under the new order rule
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05f
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mfma_peak.py > $O/mfma_peak.json 2> $O/mfma_peak.err || exit $?
cat $O/mfma_peak.json
timeout -k 10 200 python -u scripts/dtile_sweep.py > $O/dtile_sweep.txt 2>&1 || exit $?
cat $O/dtile_sweep.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for i in 1 2; do
  grp=$([ $i = 1 ] && echo FETCH_SIZE || echo WRITE_SIZE)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc_b1h1l16k/p$i -o run --output-format csv -- \
     python scripts/run_kernel.py b1h1l16k 5 > $O/pmc_b1h1l16k_p$i.log 2>&1 || exit $?
done
python3 scripts/traffic.py $O/pmc_b1h1l16k b1h1l16k_r05 $O/hbm_traffic_r05.json
