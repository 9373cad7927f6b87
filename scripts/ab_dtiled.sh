#!/bin/bash
# A/B of d-tiled kernel builds (scripts/build_lite_dt.sh) at B32 H8 L1024, d = 384 and 512.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=exploring_flash_attention_amd/_lib/ab
libs=(); for n in "$@"; do libs+=("$L/$n.so"); done
for d in 384 512; do
  echo "== d=$d"
  timeout -k 10 200 python scripts/ab.py --shape 32,8,1024,$d --rounds 6 --iters 10 --warmup 20 "${libs[@]}" 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "ab.py exited $rc"; exit $rc; }
done
