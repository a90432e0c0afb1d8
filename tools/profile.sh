#!/bin/bash
# Profiling passes for bench.py on the GPU box (run from the repo root):
#   1. rocprofv3 --kernel-trace --stats (timing; the committed summary under profiles/)
#   2. separate --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950;
#      SQ counters in their own pass), each with --kernel-trace only.
# Usage: tools/profile.sh <tag> [bench args...]
# Stops at the first pass that times out / aborts / faults (exit 124/134/137/139).
set -u
TAG=${1:-r01}; shift || true
ARGS=${*:---steps 1 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS \
      > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after fatal rc"; exit $rc;; esac
  return 0
}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run trace --kernel-trace --stats
run pmc_fetch --kernel-trace --pmc FETCH_SIZE
run pmc_write --kernel-trace --pmc WRITE_SIZE
run pmc_sq --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS
run pmc_grbm --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT
run pmc_sq2 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY
echo done
