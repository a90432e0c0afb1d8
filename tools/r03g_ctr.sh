#!/bin/bash
# r03g: AES-CTR blocks sharing rounds 1-2 (OT expand, sketch keystream): parity of the OT / GC /
# party / sketch GPU tests with the new build, the RCCL bootstrap + fallback test, then same-box
# rocprof A/Bs of the configs[1] GC + OT crawl and of configs[4] (base = the previous build).
set -u
O=gpurun_out/r03g; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests bash -c "FHH_LIB_PATH=ab_builds/libfhh_new.so timeout -k 10 500 python -u -m pytest tests/test_ot.py tests/test_gc.py tests/test_party.py tests/test_sketch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1"
step rccl bash -c "timeout -k 10 400 python -u -m pytest tests/test_bench_sharding.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/sharding.log 2>&1"
step ab_gc bash tools/ab_kernels.sh gc_r03g 2 --clients 100000 --gc ot --steps 1 --warmup 1 --no-cpu-baseline
step ab_sk bash tools/ab_kernels.sh sk_r03g 2 --workload sketch --steps 2 --warmup 1
echo done
