#!/bin/bash
# r06 A/B of the ChaCha expand variants (ab_builds/libfhh_<v>.so): rocprofv3 kernel stats of tools/ot_micro.py
set -u
O=gpurun_out/${1:-r06_abot}; shift
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in "$@"; do
    FHH_LIB_PATH=ab_builds/libfhh_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp_${v}_$r -o run \
      -- python3 tools/ot_micro.py 67108864 3 > $O/${v}_$r.log 2>&1 || exit $?
    find $O/tmp_${v}_$r -name "*kernel_stats.csv" -exec cp {} $O/${v}_${r}_kernel_stats.csv \;
    rm -rf $O/tmp_${v}_$r
    echo "round $r $v done"
  done
done
