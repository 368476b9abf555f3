# header records: the speculative poll window (GCL_TUNE_LOOP_SPEC, 10-ns ticks) against
# plain and inline loops, burst 64 on one host core, alternating rounds
set -o pipefail
O=gpurun_out/r03zc
mkdir -p $O
for rnd in 1 2; do
  for a in "1 1" "4 8" "8 16" "16 32"; do
    for m in plain inline; do
      timeout -k 10 120 ./tools/rxpipe 64 $a 20000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
    for sp in 400 150 60 0; do
      GCL_TUNE_LOOP_SPEC=$sp timeout -k 10 120 ./tools/rxpipe 64 $a 20000 records | sed "s/^{/{\"mode\": \"records\", \"spec\": $sp, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zc/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d.get('spec',''), d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'])
PY
