#!/bin/bash
# halfline timing plus its fabric request counters (one pass per TCC group)
export TMPDIR=/tmp
O=gpurun_out/halfline
mkdir -p $O
timeout -k 10 120 ./tools/halfline 20 > $O/time.jsonl 2> $O/time.err || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $O/req -o run -- ./tools/halfline 1 > $O/req.jsonl 2> $O/req.err || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RD_UNCACHED_32B_sum --output-format csv -d $O/dram -o run -- ./tools/halfline 1 > $O/dram.jsonl 2> $O/dram.err
echo done
