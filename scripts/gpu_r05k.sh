# round 5, call k: the fused chain as a walk over each tile's key blocks (A/B vs one-shot), then the GPU suite
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05k
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/base.so $L/chain.so"
timeout -k 10 200 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 6 $V > $O/ab_b2h2.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 1 --rounds 4 --warmup 20 $V > $O/ab_c4g1.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 4 --rounds 4 --warmup 20 $V > $O/ab_c4g4.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --config c3 --rounds 6 $V > $O/ab_c3.txt 2>&1
rc=$?
cat $O/ab_*.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -25 $O/tests.log
exit $rc
