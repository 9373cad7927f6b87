# round 5, call z4: per-item alternating issue priority between the two workgroups of a CU (pb1) vs none (pb0)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05z4
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/pb0.so $L/pb1.so"
timeout -k 10 200 python -u scripts/ab.py --config c3 --rounds 10 $V > $O/ab_c3.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --config l2048 --rounds 6 $V > $O/ab_l2048.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 32,8,4096,128 --rounds 4 --warmup 30 $V > $O/ab_c4.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 1 --rounds 4 --warmup 20 $V > $O/ab_c4g1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 6 $V > $O/ab_b2h2.txt 2>&1
rc=$?
cat $O/ab_*.txt | grep -v amdgpu.ids
exit $rc
