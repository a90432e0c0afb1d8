#!/bin/bash
# Same-box kernel-level A/B of environment settings of ONE build (run from the repo root on the GPU box):
#   tools/ab_env.sh <tag> <rounds> "<VAR=val ...>" "<VAR=val ...>" ... -- <python args...>
# For every round and every setting: rocprofv3 --kernel-trace --stats of `python3 <python args>` with the
# setting's variables exported; keeps the per-kernel stats CSV and the log of each run
# (gpurun_out/abe_<tag>/s<k>_<round>_kernel_stats.csv, s<k>_<round>.log; s<k> = k-th setting).
set -u
TAG=$1; ROUNDS=$2; shift 2
SETTINGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETTINGS+=("$1"); shift; done
shift
export TMPDIR=/tmp
OUT=gpurun_out/abe_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for k in "${!SETTINGS[@]}"; do
    (
      for kv in ${SETTINGS[$k]}; do export "$kv"; done
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tmp_${k}_$r -o run \
          -- python3 "$@" > $OUT/s${k}_$r.log 2>&1
    )
    rc=$?
    echo "round $r setting $k [${SETTINGS[$k]}] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    find $OUT/tmp_${k}_$r -name "*kernel_stats.csv" -exec cp {} $OUT/s${k}_${r}_kernel_stats.csv \;
    rm -rf $OUT/tmp_${k}_$r
  done
done
