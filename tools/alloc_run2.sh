#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
timeout -k 10 200 ./tools/alloc_ab 20 cfirst > $O/alloc_cfirst.jsonl 2> $O/alloc_cfirst.err || exit $?
timeout -k 10 200 ./tools/alloc_ab 20 cfirst > $O/alloc_cfirst2.jsonl 2> $O/alloc_cfirst2.err || exit $?
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -i -E "utcl|tlb|translation" $O/counters.txt | head -40 > $O/counters_tlb.txt || true
cat $O/alloc_cfirst.jsonl $O/alloc_cfirst2.jsonl $O/counters_tlb.txt
