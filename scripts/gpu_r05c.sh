# round 5, call c: where the chained kernel differs (C3), then the A/B of the fixed build
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05c
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
timeout -k 10 120 python -u scripts/debug_chain.py $L/base.so $L/chain.so $L/chain_soff.so > $O/debug.txt 2>&1; rc=$?
cat $O/debug.txt; [ $rc -eq 0 ] || exit $rc
for cfg in c3 l2048; do
  timeout -k 10 240 python -u scripts/ab.py --config $cfg --rounds 10 $L/base.so $L/chain.so > $O/ab_$cfg.txt 2>&1 || { cat $O/ab_$cfg.txt; exit 1; }
  cat $O/ab_$cfg.txt
done
