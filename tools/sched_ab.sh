#!/bin/bash
# A/B of the static persistent grid vs the dynamic per-XCD tile queue:
# parity with the queue on, then cbench with and without a co-running kernel.
export TMPDIR=/tmp
O=gpurun_out/r01/sched
mkdir -p $O
GCL_TUNE_SCHED=1 timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest_sched1.log 2>&1 || { tail -30 $O/pytest_sched1.log; exit 1; }
tail -2 $O/pytest_sched1.log
for WL in 0 1; do
  timeout -k 10 120 ./tools/cbench $WL 20 0:0:0:0:0:0 0:0:0:0:0:1 > $O/cb_wl${WL}.jsonl || exit $?
  CBENCH_NOISE_US=40 timeout -k 10 120 ./tools/cbench $WL 20 0:0:0:0:0:0 0:0:0:0:0:1 > $O/cb_wl${WL}_noise40.jsonl || exit $?
done
cat $O/*.jsonl
