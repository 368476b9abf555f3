#!/bin/bash
# 8-B vs 4-B verdicts, interleaved in one process (tools/cbench)
export TMPDIR=/tmp
O=gpurun_out/r01/v4
mkdir -p $O
for WL in 0 1; do
  CBENCH_PROFILE=0 timeout -k 10 150 ./tools/cbench $WL 20 0:0:0:0:0:0:0 0:0:0:0:0:0:1 > $O/cb_wl${WL}.jsonl || exit $?
done
cat $O/*.jsonl
