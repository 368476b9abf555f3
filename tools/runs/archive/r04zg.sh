# launch-geometry sweep of the udp64 headline with 1-B verdicts (earlier
# rounds tuned it with 4- and 2-B ones): default (4 x 256 lanes per CU,
# depth 2), 3 blocks per CU, 2 x 512, 1 x 1024, depth 1, the dynamic tile
# queue; fresh processes, two passes
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04zg_geometry.jsonl
for rep in 1 2; do
  for cfg in "default" "GCL_TUNE_BLOCKS_PER_CU=3" "GCL_TUNE_THREADS=512" "GCL_TUNE_THREADS=1024" "GCL_TUNE_DEPTH=1" "GCL_TUNE_SCHED=1"; do
    if [ "$cfg" = default ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 200 python bench.py --no-secondary --no-e2e --no-cpu --no-group > gpurun_out/r04zg_run.json 2> gpurun_out/r04zg_run.err || { tail -5 gpurun_out/r04zg_run.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04zg_run.json').read().strip().splitlines()[-1]); print(json.dumps({'cfg': '$cfg', 'rep': $rep, 'value': d['value'], 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'frac_of_ceiling': d['roofline'].get('frac_of_ceiling'), 'checks': [c.get('kernel_us') for c in d['placement']['kernel_checks']]}))" >> $out
  done
done
cat $out
