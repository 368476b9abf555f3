#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
timeout -k 10 200 ./tools/alloc_ab 20 > $O/alloc_ab.jsonl 2> $O/alloc_ab.err || exit $?
cat $O/alloc_ab.jsonl
timeout -k 10 300 python bench.py --verdict-bytes 8 --no-e2e --no-cpu > $O/bench_v8_first.json 2> $O/bench_v8_first.err || exit $?
timeout -k 10 300 python bench.py --verdict-bytes 4 --no-e2e --no-cpu > $O/bench_v4_first.json 2> $O/bench_v4_first.err || exit $?
