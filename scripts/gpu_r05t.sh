# round 5, call t: split-KV combine in one load batch at <= 4 partials (both kernels) and the
# walk's next K / V tiles issued before its combine; A/B against the previous commit (head)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05t
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/head.so $L/ov0.so $L/ov2.so"
timeout -k 10 200 python -u scripts/ab.py --shape 1,1,16384,128 --kvtpb -1 --rounds 10 $V > $O/ab_b1h1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 1,2,4096,128 --kvtpb -1 --rounds 10 $V > $O/ab_b1h2l4k.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 4 --rounds 4 --warmup 20 $V > $O/ab_c4g4.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --config c4 --kvtpb 4 --bpw 1 --rounds 4 --warmup 20 $V > $O/ab_c4g1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 6 $V > $O/ab_b2h2.txt 2>&1
rc=$?
cat $O/ab_*.txt | grep -v amdgpu.ids
exit $rc
