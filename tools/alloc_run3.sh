#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
timeout -k 10 300 ./tools/alloc_ab 10 sweep 16 > $O/alloc_sweep.jsonl 2> $O/alloc_sweep.err || exit $?
cat $O/alloc_sweep.jsonl
