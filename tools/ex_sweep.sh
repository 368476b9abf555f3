#!/bin/bash
# multi-GPU step overhead at N=1: RCCL exchange every P steps vs the plain step
export TMPDIR=/tmp
O=gpurun_out/r01/ex
mkdir -p $O
timeout -k 10 200 python bench.py --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/plain.json 2>$O/plain.err || exit $?
for P in 1 8; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29540+P)) bench.py --gpus 1 --force-exchange --exchange-every $P --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/p$P.json 2> $O/p$P.err || exit $?
done
timeout -k 10 200 python bench.py --steps 64 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/plain2.json 2>$O/plain2.err || exit $?
for f in $O/*.json; do echo $f; cat $f; done
