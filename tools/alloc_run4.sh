#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $O/pmc_tlb -o run -- ./tools/alloc_ab 2 sweep 12 > $O/alloc_tlb.jsonl 2> $O/alloc_tlb.err || exit $?
cat $O/alloc_tlb.jsonl
