set -u
# r06 SoftSpoken session: the OT / SoftSpoken / GC crawl GPU tests, then the 1M protocol crawl (IKNP, k = 2, 4)
O=gpurun_out/${1:-r06ss}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_softspoken.py tests/test_ot.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_ot.log 2>&1 || { echo ot tests failed; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gc.py tests/test_party.py -m gpu -x -v --timeout 300 --timeout-method thread -k "softspoken or equals_plain or equals_in_process" > $O/tests_gc.log 2>&1 || { echo gc tests failed; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp -o run -- python3 bench.py --gc ot --base-ot --steps 1 --warmup 0 --no-cpu-baseline --no-protocol-circuit --protocol-ss-k 2,4 > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
find $O/tmp -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/tmp
echo done
