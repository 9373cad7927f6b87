# round 5, call m: 4-deep combine in the one-shot kernel too (base_old -> base), and the walk
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05m
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/base_old.so $L/base.so $L/chain.so"
timeout -k 10 200 python -u scripts/ab.py --shape 1,1,16384,128 --kvtpb -1 --rounds 8 --all $V > $O/ab_b1h1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 1,2,4096,128 --kvtpb -1 --rounds 8 $V > $O/ab_b1h2l4k.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb -1 --rounds 6 $V > $O/ab_b2h2auto.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 1 --rounds 3 --warmup 20 $V > $O/ab_c4g1.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb -1 --rounds 3 --warmup 20 $V > $O/ab_c4auto.txt 2>&1
rc=$?
cat $O/ab_*.txt
exit $rc
