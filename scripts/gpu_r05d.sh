# round 5, call d: chained kernel (fixed DMA offsets): correctness per item, A/B
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05d
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
timeout -k 10 120 python -u scripts/debug_chain.py $L/base.so $L/chain.so $L/chain_lazy.so > $O/debug.txt 2>&1; rc=$?
cat $O/debug.txt; [ $rc -eq 0 ] || exit $rc
for cfg in c3 l2048 c4; do
  timeout -k 10 300 python -u scripts/ab.py --config $cfg --rounds 12 $L/base.so $L/chain.so $L/chain_notap.so $L/chain_noqpf.so $L/chain_lazy.so > $O/ab_$cfg.txt 2>&1 || { cat $O/ab_$cfg.txt; exit 1; }
  cat $O/ab_$cfg.txt
done
