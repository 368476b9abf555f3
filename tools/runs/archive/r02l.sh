set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress.json 2> $O/ingress.err &&
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err &&
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-e2e --no-cpu > $O/b$i.json 2> $O/b$i.err || exit $?
done
echo rc=$?
