#!/bin/bash
# r03d: the producer / consumer k_sketch_fe (impl 4): GPU parity of every sketch form, then a same-box
# A/B of configs[4] (bench --workload sketch) impl 0 vs impl 4, alternating, rocprof kernel stats.
set -u
O=gpurun_out/r03d; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step sketch_tests bash -c "timeout -k 10 400 python -u -m pytest tests/test_sketch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sketch_tests.log 2>&1"
for r in 1 2; do
  for impl in 0 4 5; do
    step "ab r$r impl$impl" bash -c "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp_${impl}_$r -o run -- python3 bench.py --workload sketch --sketch-impl $impl --steps 2 --warmup 1 > $O/impl${impl}_$r.json 2> $O/impl${impl}_$r.err"
    find $O/tmp_${impl}_$r -name "*kernel_stats.csv" -exec cp {} $O/impl${impl}_${r}_kernel_stats.csv \;
    rm -rf $O/tmp_${impl}_$r
  done
done
echo done
