# round 5, call w: the walk combine: maxima in one trip (pipe0), the sums double-buffered one (up1) or two (up2) blocks at a time
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05w
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/walk.so $L/pipe0.so $L/up1.so $L/up2.so"
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 1 --rounds 4 --warmup 20 $V > $O/ab_c4g1.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 4 --rounds 4 --warmup 20 $V > $O/ab_c4g4.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 6 $V > $O/ab_b2h2.txt 2>&1
rc=$?
cat $O/ab_*.txt | grep -v amdgpu.ids
exit $rc
