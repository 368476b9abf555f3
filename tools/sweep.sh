#!/bin/bash
# Tuning sweep over the GCL_TUNE_* knobs (bench.py, no CPU leg).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sweep}
mkdir -p $OUT
for wl in ${WLS:-udp64 tcp1500}; do
 for d in ${DEPTHS:-1 2}; do
  for nt in ${NTS:-0 1}; do
   for bpc in ${BPCS:-0 4}; do
    tag=${wl}_d${d}_nt${nt}_b${bpc}
    GCL_TUNE_DEPTH=$d GCL_TUNE_NT_STORE=$nt GCL_TUNE_BLOCKS_PER_CU=$bpc timeout -k 10 120 \
      python bench.py --workload $wl --steps ${STEPS:-30} --warmup 3 --no-cpu --no-secondary --no-e2e > $OUT/$tag.json 2> $OUT/$tag.err || { echo "FAIL $tag"; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['roofline']['achieved'], d['roofline']['kernel_ms'])"
   done
  done
 done
done
