#!/bin/bash
# geometry sweep with 4-B verdicts (cbench cfg ABLATE:GRID:DEPTH:THREADS:BPC:SCHED:V4)
export TMPDIR=/tmp
O=gpurun_out/r01/v4sweep
mkdir -p $O
CBENCH_PROFILE=0 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:1 0:0:2:0:0:0:1 0:0:0:512:0:0:1 0:0:2:512:0:0:1 0:0:0:0:2:0:1 0:0:0:0:3:0:1 0:0:0:0:6:0:1 0:0:0:0:8:0:1 0:0:0:1024:0:0:1 > $O/udp64.jsonl || exit $?
CBENCH_PROFILE=0 timeout -k 10 300 ./tools/cbench 1 20 0:0:0:0:0:0:1 0:0:2:0:0:0:1 0:0:0:256:0:0:1 0:0:0:256:3:0:1 0:0:0:0:1:0:1 0:0:0:0:3:0:1 0:0:0:1024:0:0:1 > $O/tcp1500.jsonl || exit $?
cat $O/*.jsonl
mkdir -p $O
CBENCH_PROFILE=0 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:1 0:0:2:0:0:0:1 0:0:2:0:3:0:1 0:0:2:0:5:0:1 0:0:2:0:6:0:1 0:0:0:0:0:0:0 0:0:2:0:0:0:0 > $O/udp64_d2.jsonl || exit $?
cat $O/udp64_d2.jsonl
