#!/bin/bash
# per-launch gap: kernel time vs wall time per back-to-back step, with and
# without the per-launch profiling events
export TMPDIR=/tmp
O=gpurun_out/r01/gap
mkdir -p $O
for WL in 0 1; do
  CBENCH_PROFILE=1 timeout -k 10 120 ./tools/cbench $WL 20 0:0:0:0:0:0 > $O/cb_wl${WL}_p1.jsonl || exit $?
  CBENCH_PROFILE=0 timeout -k 10 120 ./tools/cbench $WL 20 0:0:0:0:0:0 > $O/cb_wl${WL}_p0.jsonl || exit $?
done
cat $O/*.jsonl
