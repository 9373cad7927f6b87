# round 5, call q: split-KV hand-off with arrive_first only for key blocks >= 4096 keys (the last
# arriver's own partial from the registers either way); A/B vs the store-first build, PMC bytes
# of the split shapes on the full library, GPU suite.  (Call o, same script shape: arrive_first
# everywhere, plus b2h2l16k / c4g1 -- gpurun_out/r05o.)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05q
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
L=exploring_flash_attention_amd/_lib/ab
V="$L/chain_prev.so $L/chain.so"
timeout -k 10 200 python -u scripts/ab.py --shape 1,1,16384,128 --kvtpb -1 --rounds 10 --all $V > $O/ab_b1h1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 1,2,4096,128 --kvtpb -1 --rounds 10 $V > $O/ab_b1h2l4k.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 4 --rounds 4 --warmup 20 $V > $O/ab_c4g4.txt 2>&1
rc=$?
cat $O/ab_*.txt
[ $rc -eq 0 ] || exit $rc
export PMC_CONFIGS="b1h1l16k b1h2l4k c4g4"
for c in $PMC_CONFIGS; do
  for i in 1 2; do
    grp=$([ $i = 1 ] && echo FETCH_SIZE || echo WRITE_SIZE)
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc_$c/p$i -o run --output-format csv -- \
       python3 scripts/run_kernel.py $c 5 > $O/pmc_${c}_p$i.log 2>&1; rc=$?
    echo "$c pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/traffic.py $O/pmc_$c $c $O/hbm_traffic.json > /dev/null || exit $?
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; exit $rc
