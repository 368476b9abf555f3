# rxpipe with TSC timestamps and the submit/wait/deliver split sampled every 8th burst:
# burst 64 at 1-32 workers, plain offsets and header records, 3 rounds
set -o pipefail
O=gpurun_out/r03zk
mkdir -p $O
for rnd in 1 2 3; do
  for a in "1 1" "4 8" "8 16" "16 32" "32 64"; do
    for m in plain records; do
      timeout -k 10 120 ./tools/rxpipe 64 $a 40000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zk/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'], d['deliver_ns_per_pkt'], d['wait_ns_per_pkt'])
PY
