# round 5, call b: chained-kernel A/B, GPU correctness of the product build, then the r05a items
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05b
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
for cfg in c3 l2048 c4; do
  timeout -k 10 240 python -u scripts/ab.py --config $cfg --rounds 10 $L/base.so $L/chain.so $L/chain_notap.so $L/chain_noqpf.so > $O/ab_$cfg.txt 2>&1 || { cat $O/ab_$cfg.txt; exit 1; }
  cat $O/ab_$cfg.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mfma_peak.py > $O/mfma_peak.json 2> $O/mfma_peak.err || exit $?
cat $O/mfma_peak.json
timeout -k 10 200 python -u scripts/dtile_sweep.py > $O/dtile_sweep.txt 2>&1 || exit $?
cat $O/dtile_sweep.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -3 $O/bench.err; exit $rc
