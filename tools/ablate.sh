#!/bin/bash
# Timing-only ablations of the classify kernel (GCL_TUNE_ABLATE bitmask:
# 1 no flow hash, 2 no IP lookup, 4 no histogram atomic, 8 no flow_tbl gather).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ablate}
mkdir -p $OUT
for wl in ${WLS:-udp64 tcp1500}; do
  for a in ${ABL:-0 1 2 4 8 15}; do
    GCL_TUNE_ABLATE=$a timeout -k 10 120 python bench.py --workload $wl --steps 30 --warmup 3 --no-cpu --no-secondary --no-e2e > $OUT/${wl}_a$a.json 2> $OUT/${wl}_a$a.err || { echo "FAIL $wl $a"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${wl}_a$a.json')); print('$wl', 'ablate=$a', d['value'], d['roofline']['kernel_ms'])"
  done
done
