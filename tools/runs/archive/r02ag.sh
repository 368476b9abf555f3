# GPU tests on the current build (incl. the loop-geometry parity cases)
set -o pipefail
O=gpurun_out/r02ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; exit $rc
