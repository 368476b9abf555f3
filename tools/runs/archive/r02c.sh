set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scaling strong --no-secondary --no-e2e --no-cpu --steps 20 > $O/bench_strong.json 2> $O/bench_strong.err
echo rc=$?
