# burst-64 pipeline: where the host core's time goes (submit / wait / deliver per packet)
set -o pipefail
O=gpurun_out/r03ag
mkdir -p $O
for rep in 1 2; do
for cfg in "64 1 1 20000" "64 4 8 20000" "64 8 16 40000" "64 16 32 40000" "64 32 64 60000" "64 16 32 40000 inline"; do
  timeout -k 10 120 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
done
python3 -c "
import json
for l in open('$O/rxpipe.jsonl'):
    d=json.loads(l); print(d['burst'], d['workers'], d['depth'], d['verdicts'][-8:], d['mpps_one_core'], d['burst_latency_p50_us'], 'sub', d['submit_ns_per_pkt'], 'wait', d['wait_ns_per_pkt'], 'del', d['deliver_ns_per_pkt'])"
