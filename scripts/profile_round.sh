#!/bin/bash
# Round profile set, written under gpurun_out/round/ (then copied to profiles/<round>/ by hand):
#   kernel_stats.csv  rocprofv3 --kernel-trace --stats over the default bench (C3)
#   pmc_<cfg>/        PMC passes (scripts/profile_pmc.sh) of each config named, and their
#                     per-launch L2 egress merged into a copy of profiles/hbm_traffic.json
#   bash scripts/profile_round.sh <source label> [configs...]   (default configs: c3 c2 c4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
LABEL=${1:-round}; shift || true
CFGS=${*:-c3 c2 c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-extra > $OUT/prof_bench.json 2> $OUT/prof.log; rc=$?
echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cp profiles/hbm_traffic.json $OUT/hbm_traffic.json 2>/dev/null
for cfg in $CFGS; do
  bash scripts/profile_pmc.sh $cfg || exit $?
  python scripts/traffic.py gpurun_out/pmc_$cfg $cfg $OUT/hbm_traffic.json "$LABEL pmc_$cfg" > /dev/null || exit $?
done
head -3 $OUT/kernel_stats.csv
python - <<'PY'
import json
d = json.load(open("gpurun_out/round/hbm_traffic.json"))
for k, v in d.items():
    print(k, v.get("bytes_per_launch"), v.get("ratio_to_algorithmic"), v.get("source"))
PY
