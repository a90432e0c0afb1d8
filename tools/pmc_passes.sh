#!/bin/bash
# Run one rocprofv3 --pmc pass per argument group over `python3 bench.py $BENCH_ARGS`
# (each pass its own run, --kernel-trace only, killed after 120 s), into gpurun_out/pmc_<tag>/.
# Usage: BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline" tools/pmc_passes.sh <tag> "C1 C2 .." "C3 .." ...
set -u
TAG=$1; shift
ARGS=${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for pass in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass -T --output-format csv -d $OUT/p$i -o p$i -- \
      python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($pass) rc=$rc"
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
done
echo done
