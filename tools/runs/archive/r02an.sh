# The driver's default bench command on the final build (with the
# udp64_toeplitz secondary line), timed, then the GPU tests.
set -o pipefail
O=gpurun_out/r02an; mkdir -p $O
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench wall s: $(( $(date +%s) - s ))" > $O/wall.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; exit $rc
