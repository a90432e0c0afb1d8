#!/bin/bash
# r02c: GPU suite on the v52 default, then extra workload lines (configs[1] at d = 2, GC + OT with
# real base OTs after the fused hashes).
set -u
O=gpurun_out/r02c; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests bash -c "timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1"
step d2_100k bash -c "timeout -k 10 300 python bench.py --clients 100000 --dims 2 --steps 3 --no-cpu-baseline > $O/d2_100k.json 2> $O/d2_100k.err"
step gcot_co15 bash -c "timeout -k 10 300 python bench.py --clients 100000 --mode fe --gc ot --base-ot --steps 2 --no-cpu-baseline > $O/gcot_co15.json 2> $O/gcot_co15.err"
step gcot_ideal bash -c "timeout -k 10 300 python bench.py --clients 100000 --mode fe --gc ot --steps 2 --no-cpu-baseline > $O/gcot_ideal.json 2> $O/gcot_ideal.err"
step ab bash -c "tools/ab_bench_variants.sh gpurun_out/ab53 52 53 2 > $O/ab53.log 2>&1"
echo done
