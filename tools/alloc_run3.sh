#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
timeout -k 10 300 ./tools/alloc_ab 10 sweep 16 > $O/alloc_xcdmap.jsonl 2> $O/alloc_xcdmap.err || exit $?
cat $O/alloc_xcdmap.jsonl
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_xcdmap.log 2>&1; tail -2 $O/pytest_xcdmap.log
