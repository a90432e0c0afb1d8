#!/bin/bash
# r03e: the default sketch launch plan with its tail in the producer / consumer form: GPU parity of
# every sketch form, then a same-box rocprof A/B of configs[4] against the session-start build.
set -u
O=gpurun_out/r03e; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step sketch_tests bash -c "timeout -k 10 400 python -u -m pytest tests/test_sketch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sketch_tests.log 2>&1"
step ab bash tools/ab_kernels.sh sketch_r03e 2 --workload sketch --steps 2 --warmup 1
echo done
