#!/bin/bash
# r03j: OT hashes with the Y / x0 blocks in flight through global_load_lds during the AES:
# OT / GC / party GPU parity with that build, then the OT-extension microbenchmark A/B.
set -u
O=gpurun_out/r03j; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests bash -c "FHH_LIB_PATH=ab_builds/libfhh_glds.so timeout -k 10 400 python -u -m pytest tests/test_ot.py tests/test_gc.py tests/test_party.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1"
step ab bash tools/ab_multi.sh otglds 2 "new glds" tools/ot_micro.py 33554432 3
echo done
