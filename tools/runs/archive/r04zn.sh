# bench.py's N>1 torchrun path on the final tree (the driver's 8-GPU command
# shape), rehearsed with 2 gloo ranks sharing the one MI355X: weak and strong
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu > $O/r04zn_gloo2.json 2> $O/r04zn_gloo2.err || { tail -20 $O/r04zn_gloo2.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --allow-shared-gpu --scaling strong --no-e2e > $O/r04zn_gloo2_strong.json 2> $O/r04zn_gloo2_strong.err || { tail -20 $O/r04zn_gloo2_strong.err; exit 1; }
tail -c 600 $O/r04zn_gloo2.json; echo; tail -c 400 $O/r04zn_gloo2_strong.json
