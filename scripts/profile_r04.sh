#!/bin/bash
# Round-4 profile set on one box: rocprofv3 kernel stats of the driver's bench command, then the
# PMC passes (scripts/profile_pmc.sh) of C3 and the split-KV / d-tiled shapes, summarised per
# launch by scripts/traffic.py into gpurun_out/hbm_traffic_r04.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r04
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04 -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 500 --warmup 300 --no-cpu-baseline > gpurun_out/prof_r04/bench.json 2> gpurun_out/prof_r04/bench.err
rc=$?; echo "kernel stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${PMC_CONFIGS:-c3 b1h1l16k b1h2l4k c4g1 d512}; do
  bash scripts/profile_pmc.sh $c r04_$c || exit $?
  python3 scripts/traffic.py gpurun_out/pmc_r04_$c $c gpurun_out/hbm_traffic_r04.json > /dev/null || exit $?
done
echo profile_r04 done
