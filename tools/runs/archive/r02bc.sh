# Round-end rehearsal on the final tree: the driver's GPU test command,
# smoke, and the driver's default bench command.
set -o pipefail
O=gpurun_out/${RUN:-r02bc}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
s=$(date +%s)
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench wall s: $(( $(date +%s) - s ))" > $O/wall.txt
echo rc=0
