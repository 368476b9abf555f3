# round 3: new edge tests (frames at the end of the buffer, group streams)
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "frames_at_the_end" tests/test_gpu_group.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
