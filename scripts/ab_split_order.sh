#!/bin/bash
# A/B of the fused split-KV work order (query tile fastest vs split fastest) on the split shapes
# of bench.py's extras: lite builds qfast.so / sfast.so (scripts/build_lite.sh 128 ...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=exploring_flash_attention_amd/_lib/ab
run() {
  echo "== $*"
  timeout -k 10 200 python scripts/ab.py --rounds ${ROUNDS:-8} "$@" $L/qfast.so $L/sfast.so 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  [ $rc -eq 0 ] || { echo "ab.py exited $rc -- stopping"; exit $rc; }
}
run --config c4 --kvtpb 4 --bpw 1 --iters 5 --warmup 30
run --config c4 --kvtpb 4 --bpw 4 --iters 5 --warmup 30
run --shape 1,1,16384,128 --kvtpb 4 --iters 50
run --shape 1,2,4096,128 --kvtpb 4 --iters 100
run --shape 2,2,16384,128 --kvtpb 4 --bpw 16 --iters 20
