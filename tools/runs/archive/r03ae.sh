# rx loop with stamped offsets: loop parity tests (ragged bursts across the stamp refresh)
set -o pipefail
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rxloop.py > $O/test_rxloop.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/test_rxloop.log | tail -8; exit $rc
