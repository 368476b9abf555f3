set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scaling strong --no-secondary --no-e2e --no-cpu --steps 20 > $O/bench_strong.json 2> $O/bench_strong.err &&
timeout -k 10 300 python -u bench.py --no-secondary --no-e2e --no-cpu --force-exchange --dist-backend gloo > $O/bench_exchange_n1.json 2> $O/bench_exchange_n1.err
echo rc=$?
