set -u
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ot.py tests/test_gc.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/r06_otpmc.sh r06d_otpmc
