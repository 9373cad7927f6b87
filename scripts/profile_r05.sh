#!/bin/bash
# Round-5 profile set on one box: rocprofv3 kernel stats of the 500-step bench (the headline
# kernel's average launch must agree with the bench's HIP-event kernel_ms), then FETCH_SIZE /
# WRITE_SIZE passes (one counter group per pass, --kernel-trace only) of C3, the split shapes and
# d = 384, summarised per launch by scripts/traffic.py into gpurun_out/r05p/hbm_traffic_r05.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 500 --warmup 300 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench.err
rc=$?; echo "kernel stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${PMC_CONFIGS:-c3 b1h1l16k b2h2l16k c4g1 c4g4 d384 d512}; do
  for i in 1 2; do
    grp=$([ $i = 1 ] && echo FETCH_SIZE || echo WRITE_SIZE)
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc_$c/p$i -o run --output-format csv -- \
       python3 scripts/run_kernel.py $c 5 > $O/pmc_${c}_p$i.log 2>&1; rc=$?
    echo "$c pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/traffic.py $O/pmc_$c $c $O/hbm_traffic_r05.json > /dev/null || exit $?
done
echo profile_r05 done
