# round 5, call x: where C3's time goes on the chained grid -- time vs items per workgroup at
# L = 1024 (B = 32, 64, 128) and vs steps per item (L = 2048, 4096 at 16 items per workgroup)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05x
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/libfa_mi355x.so
for sh in 32,8,1024,128 64,8,1024,128 128,8,1024,128 256,8,1024,128 32,8,2048,128 16,8,4096,128 32,8,4096,128; do
  timeout -k 10 120 python -u scripts/ab.py --shape $sh --rounds 6 $L > $O/t_$sh.txt 2>&1 || exit $?
  echo "$sh $(grep median $O/t_$sh.txt)"
done
