#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r01/v4sweep
mkdir -p $O
CBENCH_PROFILE=0 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:1 0:0:2:0:0:0:1 0:0:2:0:3:0:1 0:0:2:0:5:0:1 0:0:2:0:6:0:1 0:0:0:0:0:0:0 0:0:2:0:0:0:0 > $O/udp64_d2.jsonl || exit $?
cat $O/udp64_d2.jsonl
