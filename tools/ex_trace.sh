#!/bin/bash
# kernel timeline of the multi-GPU step at N=1 (RCCL world of one, no launcher)
export TMPDIR=/tmp
O=gpurun_out/r01/extrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p1 -o run -- python3 bench.py --force-exchange --exchange-every 1 --steps 32 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/p1.json 2> $O/p1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/plain -o run -- python3 bench.py --steps 32 --warmup 4 --no-secondary --no-e2e --no-cpu > $O/plain.json 2> $O/plain.err || exit $?
find $O -name "*.csv" | head
