set -u
# r06 A/B session: the GC / OT / party GPU tests, the 1M real-protocol crawl's kernel stats, the driver line
O=gpurun_out/${1:-r06b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gc.py tests/test_party.py tests/test_oracle_crawl.py tests/test_ot.py tests/test_group.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; exit 1; }
tools/gpu_session.sh $O gcot1m bench
