#!/bin/bash
# multi-GPU step overhead at N=1: RCCL exchange every P steps vs the plain step
export TMPDIR=/tmp
O=gpurun_out/r01/ex
mkdir -p $O
timeout -k 10 200 python bench.py --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/plain.json 2>$O/plain.err || exit $?
for P in 1 16; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29540+P)) bench.py --gpus 1 --force-exchange --exchange-every $P --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/p$P.json 2> $O/p$P.err || exit $?
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 1 --force-exchange --exchange-every 1 --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/p1_hwq8.json 2> $O/p1_hwq8.err || exit $?
for f in $O/*.json; do echo $f; cat $f; done
