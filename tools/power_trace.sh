#!/bin/bash
# Socket power and clocks sampled once a second (rocm-smi) while a bench runs (default: the metric's
# 1M-client crawl, 15 steps), for DESIGN's power-limit argument. Read-only queries.
#   tools/power_trace.sh [outdir] [bench args...]
set -u
O=${1:-gpurun_out/power}; shift || true
ARGS=${*:---steps 15 --warmup 1 --no-cpu-baseline}
mkdir -p $O
rocm-smi --showmaxpower --json > $O/maxpower.json 2>&1 || true
timeout -k 10 300 python3 -u bench.py $ARGS > $O/bench.json 2> $O/bench.err &
PID=$!
for i in $(seq 1 150); do
  if ! kill -0 $PID 2>/dev/null; then break; fi
  echo "t=$i $(date +%s.%N)" >> $O/smi.txt
  timeout 10 rocm-smi --showpower --showclocks --showuse --json >> $O/smi.txt 2>&1
  sleep 1
done
wait $PID; rc=$?
echo "bench rc=$rc"
exit $rc
