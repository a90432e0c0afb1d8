#!/bin/bash
# Kernel-level A/B over several library builds (run from the repo root on the GPU box):
#   tools/ab_multi.sh <tag> <rounds> "<build names>" <python script + args...>
# rocprofv3 --kernel-trace --stats of `python3 <script>` with FHH_LIB_PATH = ab_builds/libfhh_<b>.so
# for every build b, alternated for <rounds> rounds; per-kernel stats CSVs into gpurun_out/abm_<tag>/.
set -u
TAG=$1; ROUNDS=$2; BUILDS=$3; shift 3
export TMPDIR=/tmp
OUT=gpurun_out/abm_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for b in $BUILDS; do
    FHH_LIB_PATH=ab_builds/libfhh_$b.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/tmp_${b}_$r -o run -- python3 "$@" > $OUT/${b}_$r.log 2>&1
    rc=$?
    echo "round $r $b rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    find $OUT/tmp_${b}_$r -name "*kernel_stats.csv" -exec cp {} $OUT/${b}_${r}_kernel_stats.csv \;
    rm -rf $OUT/tmp_${b}_$r
  done
done
