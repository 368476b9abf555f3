# 8-B verdict records (GCL_LOOP_REC8) against 16-B at 16x32 and 8x16, plain offsets, 6 alternating rounds
set -o pipefail
O=gpurun_out/r03zj
mkdir -p $O
for rnd in 1 2 3 4 5 6; do
  for a in "8 16" "16 32"; do
    for m in plain rec8; do
      timeout -k 10 120 ./tools/rxpipe 64 $a 40000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zj/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'], d['deliver_ns_per_pkt'], d['wait_ns_per_pkt'])
PY
