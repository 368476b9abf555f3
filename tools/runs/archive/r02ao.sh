# Re-entry check of HEAD on a fresh box: GPU tests, smoke, the driver's
# default bench command.
set -o pipefail
O=gpurun_out/r02ao; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo rc=0
