#!/bin/bash
# GPU steps for one gpurun call, one mode per argument (each GPU step under its own time limit, chained so that
# the first failure ends the call).  Output under gpurun_out/<tag>/.
#   bash scripts/gpu_steps.sh <tag> tests|bench|ab|pmc ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
AB=exploring_flash_attention_amd/_lib/ab
for mode in "$@"; do
  case $mode in
    tests)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
          > $OUT/tests.log 2>&1; rc=$?
      tail -3 $OUT/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      echo "bench rc=$rc"; head -c 600 $OUT/bench.json; echo; [ $rc -eq 0 ] || exit $rc ;;
    ab:*)  # ab:<config>:<lib1,lib2,...>
      IFS=: read -r _ cfg libs <<< "$mode"
      paths=$(echo $libs | tr ',' '\n' | sed "s|^|$AB/|; s|$|.so|" | tr '\n' ' ')
      timeout -k 10 300 python scripts/ab.py --config $cfg --rounds 10 $paths > $OUT/ab_$cfg.txt 2>&1; rc=$?
      echo "ab $cfg rc=$rc"; tail -8 $OUT/ab_$cfg.txt; [ $rc -eq 0 ] || exit $rc ;;
    abx:*)  # abx:<tag>:<lib1,lib2,...>:<ab.py arguments, '+' for spaces>
      IFS=: read -r _ tg libs xargs <<< "$mode"
      paths=$(echo $libs | tr ',' '\n' | sed "s|^|$AB/|; s|$|.so|" | tr '\n' ' ')
      timeout -k 10 300 python scripts/ab.py --rounds 10 $(echo $xargs | tr '+' ' ') $paths > $OUT/ab_$tg.txt 2>&1; rc=$?
      echo "ab $tg rc=$rc"; tail -8 $OUT/ab_$tg.txt; [ $rc -eq 0 ] || exit $rc ;;
    cmp:*)  # cmp:<libA>:<libB>:<d>  (scripts/cmp_libs.py)
      IFS=: read -r _ la lb dd <<< "$mode"
      timeout -k 10 300 python scripts/cmp_libs.py $AB/$la.so $AB/$lb.so $dd > $OUT/cmp_${la}_${lb}.txt 2>&1; rc=$?
      echo "cmp $la $lb rc=$rc"; tail -4 $OUT/cmp_${la}_${lb}.txt; [ $rc -eq 0 ] || exit $rc ;;
    pmc:*)  # pmc:<lib>:<B,H,L,d>:<counters, comma separated>
      IFS=: read -r _ lib shape ctrs <<< "$mode"
      name=${lib}_$(echo $shape | tr ',' '_')_$(echo $ctrs | tr ',' '_')
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $(echo $ctrs | tr ',' ' ') -d $OUT/pmc/$name -o run \
          --output-format csv -- python scripts/run_lib.py $AB/$lib.so $shape 5 > $OUT/pmc_$name.log 2>&1; rc=$?
      echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$name.log; exit $rc; } ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
done
