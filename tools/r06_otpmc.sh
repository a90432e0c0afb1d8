#!/bin/bash
# r06: kernel stats + PMC passes of the OT-extension microbenchmark (tools/ot_micro.py)
set -u
O=gpurun_out/${1:-r06_otpmc}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/ot_micro.py 67108864 3 > $O/stats.log 2>&1 || exit $?
find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
k=0
for group in "SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
             "FETCH_SIZE" "WRITE_SIZE"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $O/p$k -o p$k -- \
      python3 tools/ot_micro.py 67108864 3 > $O/p$k.log 2>&1
  rc=$?
  echo "pass $k ($group) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
