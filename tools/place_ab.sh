#!/bin/bash
# A/B of the frame-pool placement policy (gcl_dev_alloc_paired vs plain
# hipMalloc) in bench.py, three fresh processes each, interleaved.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/place_ab}
mkdir -p $O
for i in 1 2 3; do
  for p in 1 0; do
    GCL_PAIR_DEBUG=1 GCL_BENCH_PLACEMENT=$p timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 30 > $O/p${p}_$i.json 2> $O/p${p}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/p${p}_$i.json')); s=d['secondary']; print('placement=$p run $i', d['value'], d['roofline']['kernel_ms'], d['placement'].get('probe_us_chosen'), d['placement'].get('probe_us_worst'), '| tcp1500', s['value'], s['roofline']['kernel_ms'], s['placement'].get('probe_us_chosen'), s['placement'].get('probe_us_worst'), '| hsplit', s['header_split_layout']['value'])"
  done
done
