# round 5, call s2: per-step stamps of the chained kernel at C3 and L = 2048
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05s3
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 120 python -u scripts/chain_stamps.py exploring_flash_attention_amd/_lib/ab/stamps.so --config c3 > $O/stamps_c3.txt 2>&1 &&
timeout -k 10 120 python -u scripts/chain_stamps.py exploring_flash_attention_amd/_lib/ab/stamps.so --config l2048 > $O/stamps_l2048.txt 2>&1
rc=$?; cat $O/stamps_*.txt | grep -v amdgpu.ids; exit $rc
