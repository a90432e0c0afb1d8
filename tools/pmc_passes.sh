#!/bin/bash
# PMC passes of one bench.py command (run from the repo root on the GPU box), one rocprofv3 run
# per counter group (the hardware cannot collect them together; --kernel-trace only beside --pmc):
#   tools/pmc_passes.sh <tag> <bench args...>   -> gpurun_out/pmc_<tag>/p<k>/...
#   PMC_SCRIPT=tools/ot_micro.py tools/pmc_passes.sh <tag> <script args...>   (another python script)
# Summaries: python tools/pmc_means.py gpurun_out/pmc_<tag> [kernel] --json out.json
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
k=0
for group in "SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
  k=$((k + 1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $OUT/p$k -o p$k -- \
      python3 ${PMC_SCRIPT:-bench.py} "$@" > $OUT/p$k.log 2>&1
  rc=$?
  echo "pass $k ($group) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
