# bench.py's N>1 path on the current tree: the driver's torchrun command shape
# with 2 gloo ranks sharing the box's one GPU (weak and strong scaling)
set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu \
  > $O/bench_gloo2_weak.json 2> $O/bench_gloo2_weak.err || { tail -30 $O/bench_gloo2_weak.err; exit 1; }
tail -c 1500 $O/bench_gloo2_weak.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu \
  --scaling strong --no-e2e > $O/bench_gloo2_strong.json 2> $O/bench_gloo2_strong.err || { tail -30 $O/bench_gloo2_strong.err; exit 1; }
tail -c 800 $O/bench_gloo2_strong.json
