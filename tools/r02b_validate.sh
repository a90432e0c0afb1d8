#!/bin/bash
# r02b validation of the tree on one MI355X: full GPU suite, smoke, default bench, profile passes.
set -u
O=gpurun_out/r02b; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests bash -c "timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1"
step smoke bash -c "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
step bench bash -c "timeout -k 10 400 python bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.err"
step profile tools/profile.sh r02b
echo done
