#!/bin/bash
# Same-box kernel-level A/B of two library builds (run from the repo root on the GPU box):
#   tools/ab_kernels.sh <tag> <rounds> <bench args...>
# rocprofv3 --kernel-trace --stats of `python3 bench.py <args>` with FHH_LIB_PATH =
# ab_builds/libfhh_base.so and ab_builds/libfhh_new.so alternately; keeps only the per-kernel
# stats CSV of each run (gpurun_out/abk_<tag>/<build>_<round>_kernel_stats.csv).
# AB_BUILDS="base new new2 ..." alternates more builds (ab_builds/libfhh_<name>.so); AB_SCRIPT=tools/x.py
# profiles that script instead of bench.py.
set -u
TAG=$1; ROUNDS=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/abk_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for b in ${AB_BUILDS:-base new}; do
    FHH_LIB_PATH=ab_builds/libfhh_$b.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/tmp_${b}_$r -o run -- python3 ${AB_SCRIPT:-bench.py} "$@" > $OUT/${b}_$r.log 2>&1
    rc=$?
    echo "round $r $b rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    find $OUT/tmp_${b}_$r -name "*kernel_stats.csv" -exec cp {} $OUT/${b}_${r}_kernel_stats.csv \;
    rm -rf $OUT/tmp_${b}_$r
  done
done
