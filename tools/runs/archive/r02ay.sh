# GPU tests with the reference-pinned Toeplitz and transport-hash vectors.
set -o pipefail
O=gpurun_out/r02ay; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
echo rc=0
