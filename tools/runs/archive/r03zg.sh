# header records: the writer's prefetch distance and record-line prefetch for ownership
# (GCL_TUNE_LOOP_PF=dist,write) at 4x8 and 16x32, beside plain loops, alternating rounds
set -o pipefail
O=gpurun_out/r03zg
mkdir -p $O
for rnd in 1 2 3; do
  for a in "4 8" "16 32"; do
    timeout -k 10 120 ./tools/rxpipe 64 $a 20000 | sed "s/^{/{\"mode\": \"plain\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    for pf in 2,0 2,1 6,0 6,1; do
      GCL_TUNE_LOOP_PF=$pf timeout -k 10 120 ./tools/rxpipe 64 $a 20000 records | sed "s/^{/{\"mode\": \"records\", \"pf\": \"$pf\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zg/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d.get('pf',''), d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'], d['deliver_ns_per_pkt'], d['wait_ns_per_pkt'])
PY
