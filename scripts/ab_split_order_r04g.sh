#!/bin/bash
# A/B of the fused split-KV work order on the shapes round 4's plan now splits further
# (B1 H1 L16384: 4 partials per tile; B1 H2 L16384: 2), qfast.so / sfast.so as in
# scripts/ab_split_order.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=exploring_flash_attention_amd/_lib/ab
run() {
  echo "== $*"
  timeout -k 10 200 python scripts/ab.py --rounds ${ROUNDS:-8} "$@" $L/qfast.so $L/sfast.so 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  [ $rc -eq 0 ] || { echo "ab.py exited $rc -- stopping"; exit $rc; }
}
run --shape 1,1,16384,128 --kvtpb 1 --iters 50
run --shape 1,2,16384,128 --kvtpb 1 --iters 50
run --shape 1,4,16384,128 --kvtpb 1 --iters 30
run --shape 1,1,32768,128 --kvtpb 1 --iters 20
