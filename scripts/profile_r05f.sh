#!/bin/bash
# Round-5 final profile set: rocprofv3 kernel stats of the C3 headline alone (500 steps, no
# extras: its average must agree with the bench line's kernel_ms), the driver's default bench
# command, and FETCH_SIZE / WRITE_SIZE passes of the shapes whose traffic entries predate this
# round's kernels (c2, c4 = the chained grid at one partial, the unsplit low-parallelism shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o run --output-format csv -- \
    python3 bench.py --steps 500 --warmup 300 --no-extra --no-cpu-baseline > $O/c3_prof_bench.json 2> $O/c3_prof_bench.err
rc=$?; echo "c3 kernel stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${PMC_CONFIGS:-c2 c4 b1h1l16k_unsplit b1h2l4k_unsplit}; do
  for i in 1 2; do
    grp=$([ $i = 1 ] && echo FETCH_SIZE || echo WRITE_SIZE)
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc_$c/p$i -o run --output-format csv -- \
       python3 scripts/run_kernel.py $c 5 > $O/pmc_${c}_p$i.log 2>&1; rc=$?
    echo "$c pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/traffic.py $O/pmc_$c $c $O/hbm_traffic.json > /dev/null || exit $?
done
timeout -k 10 600 python3 -u bench.py > $O/bench_driver_default.json 2> $O/bench_driver_default.err
rc=$?; echo "bench rc=$rc"; cat $O/bench_driver_default.json; exit $rc
