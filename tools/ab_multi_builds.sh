#!/bin/bash
# Same-box A/B of several library builds (run from the repo root on the GPU box):
#   tools/ab_multi_builds.sh <tag> "<build names>" <bench args...>
# runs `python bench.py <bench args>` once per ab_builds/libfhh_<name>.so, one JSON line each
# into gpurun_out/ab_<tag>/<name>_<position>.json (a name may repeat: alternating rounds)
set -u
TAG=$1; NAMES=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
i=0
for b in $NAMES; do
  i=$((i+1))
  FHH_LIB_PATH=ab_builds/libfhh_$b.so timeout -k 10 300 python3 -u bench.py "$@" > $OUT/${b}_$i.json 2> $OUT/${b}_$i.err
  rc=$?
  echo "$b rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
