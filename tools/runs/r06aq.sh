# round 6, the final tree: the N = 2 line rehearsed on one GPU (two gloo ranks
# sharing it), launcher-less and under torchrun as the driver starts it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 10 --warmup 2 --no-e2e --cpu-budget 10 > gpurun_out/r06aq_bench_gloo2.json 2> gpurun_out/r06aq_bench_gloo2.err || { tail -5 gpurun_out/r06aq_bench_gloo2.err; exit 1; }
head -c 400 gpurun_out/r06aq_bench_gloo2.json; echo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --allow-shared-gpu --no-e2e --cpu-budget 10 > gpurun_out/r06aq_bench_gloo2_torchrun.json 2> gpurun_out/r06aq_bench_gloo2_torchrun.err || { tail -5 gpurun_out/r06aq_bench_gloo2_torchrun.err; exit 1; }
head -c 400 gpurun_out/r06aq_bench_gloo2_torchrun.json; echo
echo r06aq-done
