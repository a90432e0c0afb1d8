#!/bin/bash
# r03h: the real protocol's crawl (GC + OT extension every level) at the metric's 1M clients on the
# current tree, with rocprofv3 kernel stats.
set -u
O=${1:-gpurun_out/r03h}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gc ot --steps 1 --warmup 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "gcot1m rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/prof
echo done
