#!/bin/bash
# The driver's round-end sequence on the final tree: GPU suite, smoke, the default bench line.
set -u
O=${1:-gpurun_out/r02_final}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests bash -c "timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1"
step smoke bash -c "timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
step bench bash -c "timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err"
echo done
