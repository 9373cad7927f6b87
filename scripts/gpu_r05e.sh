# round 5, call e: chained kernel A/B on a longer interleave (every round printed)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05e
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/base.so $L/chain.so $L/chain_notap.so $L/chain_noqpf.so $L/chain_notap_noqpf.so $L/chain_tap8.so $L/chain_tap11.so"
for cfg in c3 l2048 c3 c4; do
  timeout -k 10 300 python -u scripts/ab.py --all --config $cfg --rounds 16 $V > $O/ab_$cfg.txt 2>&1 || { cat $O/ab_$cfg.txt; exit 1; }
  cat $O/ab_$cfg.txt
done
