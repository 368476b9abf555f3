# header records with the register-only writer: the speculative poll window
# (GCL_TUNE_LOOP_SPEC, 10-ns ticks) at 8x16 and 16x32, beside plain loops, alternating rounds
set -o pipefail
O=gpurun_out/r03ze
mkdir -p $O
for rnd in 1 2 3; do
  for a in "8 16" "16 32"; do
    timeout -k 10 120 ./tools/rxpipe 64 $a 20000 | sed "s/^{/{\"mode\": \"plain\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    for sp in 400 150 60 0; do
      GCL_TUNE_LOOP_SPEC=$sp timeout -k 10 120 ./tools/rxpipe 64 $a 20000 records | sed "s/^{/{\"mode\": \"records\", \"spec\": $sp, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03ze/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d.get('spec',''), d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'], d['deliver_ns_per_pkt'], d['wait_ns_per_pkt'])
PY
