#!/bin/bash
# Same-box rocprof A/B of library builds (run from the repo root on the GPU box):
#   tools/ab_rocprof.sh <tag> "<build names>" <bench args...>
# one `rocprofv3 --kernel-trace --stats` of `python3 bench.py <bench args>` per
# ab_builds/libfhh_<name>.so (a name may repeat), kernel stats into gpurun_out/abp_<tag>/<name>_<i>_*.
set -u
TAG=$1; NAMES=$2; shift 2
OUT=gpurun_out/abp_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for b in $NAMES; do
  i=$((i+1))
  FHH_LIB_PATH=ab_builds/libfhh_$b.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT -o ${b}_$i -- python3 -u bench.py "$@" > $OUT/${b}_$i.json 2> $OUT/${b}_$i.err
  rc=$?
  echo "$b rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
