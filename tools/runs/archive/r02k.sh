set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-e2e --no-cpu > $O/b$i.json 2> $O/b$i.err || exit $?
done
echo done
