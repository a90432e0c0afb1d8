#!/bin/bash
# Same-box A/B of two library builds (run from the repo root on the GPU box):
#   tools/ab_builds.sh <tag> <rounds> <bench args...>
# alternates FHH_LIB_PATH=ab_builds/libfhh_base.so and ab_builds/libfhh_new.so for <rounds>
# rounds of `python bench.py <bench args>`, one JSON line each into gpurun_out/ab_<tag>/.
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for b in base new; do
    FHH_LIB_PATH=ab_builds/libfhh_$b.so timeout -k 10 300 python3 -u bench.py "$@" > $OUT/${b}_$r.json 2> $OUT/${b}_$r.err
    rc=$?
    echo "round $r $b rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
