set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu > $O/bench_gloo2.json 2> $O/bench_gloo2.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu --scaling strong --no-e2e > $O/bench_gloo2_strong.json 2> $O/bench_gloo2_strong.err
echo rc=$?
