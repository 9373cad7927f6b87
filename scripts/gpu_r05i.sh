# round 5, call i: pair-kernel (d = 384) A/B, fused-chain A/B, full GPU suite, MFMA ceiling, bench
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05i
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
timeout -k 10 300 python -u scripts/ab.py --all --acc --shape 32,8,1024,384 --rounds 8 $L/dt_old.so $L/dt_pair.so > $O/ab_d384.txt 2>&1; rc=$?
cat $O/ab_d384.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab.py --all --acc --shape 8,8,4096,384 --rounds 6 $L/dt_old.so $L/dt_pair.so > $O/ab_d384_l4k.txt 2>&1; rc=$?
cat $O/ab_d384_l4k.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r05g.sh || exit $?
cp gpurun_out/r05g/* $O/ 2>/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mfma_peak.py > $O/mfma_peak.json 2> $O/mfma_peak.err || exit $?
cat $O/mfma_peak.json
timeout -k 10 200 python -u scripts/dtile_sweep.py > $O/dtile_sweep.txt 2>&1 || exit $?
cat $O/dtile_sweep.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -3 $O/bench.err; exit $rc
