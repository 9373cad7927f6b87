#!/bin/bash
# A/B timing of the builds under exploring_flash_attention_amd/_lib/ab/ on several configs.
# usage: CONFIGS="c3 c2" bash scripts/ab_run.sh base.so tail.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
libs=()
for n in "$@"; do libs+=("exploring_flash_attention_amd/_lib/ab/$n"); done
for c in ${CONFIGS:-c3}; do
  echo "== $c"
  timeout -k 10 240 python scripts/ab.py --config $c --rounds ${ROUNDS:-10} ${AB_ARGS:-} "${libs[@]}" 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  [ $rc -eq 0 ] || { echo "ab.py exited $rc -- stopping"; exit $rc; }
done
