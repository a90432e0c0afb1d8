#!/bin/bash
# PMC A/B of k_expand variants at the bench workload (run from the repo root on the GPU box):
#   tools/pmc_variants.sh <tag> <variant>...   -> gpurun_out/pmcv_<tag>/v<variant>_{a,b}/
# pass a: clock (GRBM_GUI_ACTIVE), VALU / LDS instructions, waits; pass b: instruction cache.
# Stops at the first pass that times out / aborts / faults.
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmcv_$TAG
mkdir -p $OUT
for V in "$@"; do
  for P in a b; do
    if [ $P = a ]; then C="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; else C="SQC_ICACHE_HITS SQC_ICACHE_MISSES"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -T --output-format csv -d $OUT/v${V}_$P -o p -- \
        python3 bench.py --variant $V --steps 1 --warmup 1 --no-cpu-baseline > $OUT/v${V}_$P.log 2>&1
    rc=$?
    echo "variant $V pass $P rc=$rc"
    case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
  done
done
echo done
