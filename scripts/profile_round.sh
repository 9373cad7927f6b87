#!/bin/bash
# Round profile set, written under gpurun_out/round/ (then copied to profiles/ by hand):
#   kernel_stats.csv  rocprofv3 --kernel-trace --stats over the default bench (C3)
#   pmc_c3/, pmc_c2/  PMC passes (scripts/profile_pmc.sh), hbm_traffic.json from them
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-extra > $OUT/prof_bench.json 2> $OUT/prof.log; rc=$?
echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cp profiles/hbm_traffic.json $OUT/hbm_traffic.json 2>/dev/null
for cfg in c3 c2 c4; do
  bash scripts/profile_pmc.sh $cfg || exit $?
  python scripts/traffic.py gpurun_out/pmc_$cfg $cfg $OUT/hbm_traffic.json > /dev/null || exit $?
done
# C4 with 4 key blocks per workgroup (4 partials per query tile through the workspace), and a
# shape the library splits itself (B1 H1 L16384: 2 partials per query tile)
for cfg in c4g4 b1h1l16k; do
  bash scripts/profile_pmc.sh $cfg || exit $?
  python scripts/traffic.py gpurun_out/pmc_$cfg $cfg $OUT/hbm_traffic.json > /dev/null || exit $?
done
cat $OUT/kernel_stats.csv | head -3
python - <<'PY'
import json
d = json.load(open("gpurun_out/round/hbm_traffic.json"))
for k, v in d.items():
    print(k, v.get("bytes_per_launch"))
PY
