set -u
# r06: the Z_2^32 table — GPU tests, then the 1M protocol crawl (k = 2) with FE and Z_2^32 shares
O=gpurun_out/${1:-r06ring}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "ring32 or garbled_table or softspoken or equals_plain" > $O/tests.log 2>&1 || { echo tests failed; exit 1; }
for ring in "" "--table-ring32"; do
  timeout -k 10 300 python3 bench.py --gc ot --base-ot --ot-ss-k 2 $ring --steps 1 --warmup 1 --no-cpu-baseline > $O/bench${ring:+_ring}.json 2> $O/bench${ring:+_ring}.err || { echo bench failed; exit 1; }
  grep timed $O/bench${ring:+_ring}.err
done
echo done
