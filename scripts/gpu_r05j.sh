# round 5, call j: why the fused chain is slow (debug variants, wrong results by design)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05j
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/base.so $L/chain.so $L/nocomb.so $L/noatom.so $L/noepi.so"
timeout -k 10 300 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 4 $V > $O/ab_b2h2.txt 2>&1; cat $O/ab_b2h2.txt
timeout -k 10 400 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 4 --rounds 3 --warmup 20 $V > $O/ab_c4g4.txt 2>&1; cat $O/ab_c4g4.txt
