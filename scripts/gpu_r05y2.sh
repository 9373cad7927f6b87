# round 5, call y2: is the seam the next Q^T load? a probe that reuses the item's Q^T (wrong outputs)
# items' Q (and K / V)?  Timing probes that read Q and / or K / V of 8 heads only (wrong outputs)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05y2
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
V="$L/base.so $L/noq.so"
timeout -k 10 200 python -u scripts/ab.py --config c3 --rounds 8 $V > $O/ab_c3.txt 2>&1 &&
timeout -k 10 200 python -u scripts/ab.py --shape 32,8,4096,128 --rounds 4 --warmup 30 $V > $O/ab_c4.txt 2>&1
rc=$?
cat $O/ab_*.txt | grep -v amdgpu.ids
exit $rc
