#!/bin/bash
# r03b: GC/OT kernel changes on the GPU: the GC/OT/party parity tests with the new build, a
# rocprof-level same-box A/B of the configs[1] GC + OT crawl (ab_builds/libfhh_{base,new}.so),
# then the driver's round-end sequence on the tree (GPU suite, smoke, bench).
set -u
O=gpurun_out/r03b; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gc_tests bash -c "FHH_LIB_PATH=ab_builds/libfhh_new.so timeout -k 10 400 python -u -m pytest tests/test_gc.py tests/test_ot.py tests/test_party.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gc_tests.log 2>&1"
step ab bash tools/ab_kernels.sh gc_r03b 2 --clients 100000 --gc ot --steps 1 --warmup 1 --no-cpu-baseline
step final bash tools/r02_final.sh $O/final
echo done
