# loop tests with the header-record fuzz cases taken with the poll
set -o pipefail
O=gpurun_out/r03zt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rxloop_tests.log 2>&1 || { tail -40 $O/rxloop_tests.log; exit 1; }
tail -3 $O/rxloop_tests.log
