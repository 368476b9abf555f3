set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --no-secondary --no-e2e --steps 20 --warmup 3 > $O/bench_prof.json 2> $O/trace.err
echo rc=$?
