#!/bin/bash
# r03c: OT kernel A/B (sender expand in two passes per tile, receive hash choice word per tile)
# and the VALU multiply-add microbenchmark (k_sketch_fe's FE products).
set -u
O=gpurun_out/r03c; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step ot_tests bash -c "FHH_LIB_PATH=ab_builds/libfhh_new.so timeout -k 10 400 python -u -m pytest tests/test_gc.py tests/test_ot.py tests/test_party.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/ot_tests.log 2>&1"
step micro bash -c "FHH_LIB_PATH=ab_builds/libfhh_new.so timeout -k 10 120 python3 -c '
import ctypes, fuzzyheavyhitters_amd as fhh
r = ctypes.c_double()
for w, name in [(0, \"v_xor_b32 8w\"), (2, \"v_bitop3_b32 8w\"), (5, \"v_mad_u64_u32 8w\"), (6, \"v_mad_u64_u32 4w\")]:
    fhh.lib().fhh_microbench(0, w, ctypes.byref(r))
    print(name, r.value / 1e12, \"T lane-ops/s\")
' > $O/micro.txt 2>&1"
step ab bash tools/ab_kernels.sh ot_r03c 2 --clients 100000 --gc ot --steps 1 --warmup 1 --no-cpu-baseline
echo done
