# poll issue order (GCL_TUNE_LOOP_ORDER 0: entries then word, 1: word then entries) against the
# share of bursts caught stale, lone-burst latency, and a soak of each order
set -o pipefail
O=gpurun_out/r03zr
mkdir -p $O
for rnd in 1 2 3; do
  for ord in 0 1; do
    for m in plain records; do
      GCL_TUNE_LOOP_ORDER=$ord timeout -k 10 120 ./tools/rxpipe 64 1 1 20000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"order\": $ord, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
    GCL_TUNE_LOOP_ORDER=$ord timeout -k 10 120 ./tools/rxpipe 64 4 8 20000 records | sed "s/^{/{\"mode\": \"records\", \"order\": $ord, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
  done
done
for ord in 0 1; do
  for m in "" records; do
    GCL_TUNE_LOOP_ORDER=$ord timeout -k 10 170 ./tools/loopsoak 3000000 1 2 1 $m | sed "s/^{/{\"order\": $ord, /" >> $O/soak.jsonl || exit 1
    GCL_TUNE_LOOP_ORDER=$ord timeout -k 10 170 ./tools/loopsoak 10000000 4 4 4 $m | sed "s/^{/{\"order\": $ord, /" >> $O/soak.jsonl || exit 1
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zr/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['order'], d['workers'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['bursts_early'], d['bursts_stale'], d['bursts_late'])
for l in open('gpurun_out/r03zr/soak.jsonl'):
    d=json.loads(l); print('soak', d['order'], d['records'], d['workers'], d['mismatches'], d['mpps'], d['bursts_early'], d['bursts_stale'], d['bursts_late'])
PY
