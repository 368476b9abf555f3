# burst-64 pipeline with more GPU workers (cap raised to 64)
set -o pipefail
O=gpurun_out/r03af
mkdir -p $O
for rep in 1 2 3; do
for cfg in "64 16 32 40000" "64 32 32 60000" "64 32 64 60000" "64 64 64 60000" "64 32 64 60000 inline" "64 64 64 60000 inline"; do
  timeout -k 10 120 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
done
python3 -c "
import json
for l in open('$O/rxpipe.jsonl'):
    d=json.loads(l); print(d['burst'], d['workers'], d['depth'], d['verdicts'][-8:], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['deliver_ns_per_pkt'], d['delivered_check'])"
