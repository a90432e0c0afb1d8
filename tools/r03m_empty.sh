#!/bin/bash
# r03m: GC / OT kernels leave empty workgroups before the LDS table fill: GC / OT / party parity with
# the new build, then a same-box rocprof A/B of the 1M-client GC + OT crawl (one round each).
set -u
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
mkdir -p gpurun_out/r03m
step tests bash -c "FHH_LIB_PATH=ab_builds/libfhh_new.so timeout -k 10 400 python -u -m pytest tests/test_ot.py tests/test_gc.py tests/test_party.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1"
step ab bash tools/ab_kernels.sh empty_r03m 1 --gc ot --steps 1 --warmup 0 --no-cpu-baseline
echo done
