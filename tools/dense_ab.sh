#!/bin/bash
# Dense tile-kernel frame loads, streaming hint (the library default) against
# plain loads (caladan_amd/ab/libgclassify.so, built with
# -DGCL_TILE_LOAD_PLAIN), alternating fresh bench processes on one box:
# udp64 in all three verdict widths and TOEPLITZ, tcp1500, the header split.
#   OUT=gpurun_out/dense_ab bash tools/dense_ab.sh
set -o pipefail
OUT=${OUT:-gpurun_out/dense_ab}
mkdir -p $OUT
for i in 1 2; do
  for v in nt plain; do
    if [ $v = plain ]; then export GCL_LIB=$PWD/caladan_amd/ab/libgclassify.so; else unset GCL_LIB; fi
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-e2e --no-cpu --no-group > $OUT/$v.$i.json 2> $OUT/$v.$i.err || { tail $OUT/$v.$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$v.$i.json').read().strip().splitlines()[-1]); s=d['secondary']
print('$v', $i, d['value'], d['roofline']['kernel_ms'], [o['value'] for o in s['udp64_other_verdicts']], s['udp64_toeplitz']['value'], s['value'], s['roofline']['kernel_ms'], s['header_split_layout']['value'])"
  done
done
