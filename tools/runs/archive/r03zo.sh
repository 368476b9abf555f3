# slot-ring allocation (GCL_TUNE_LOOP_ALLOC 0 hipHostMalloc, 1 rounded to 2 MiB, 2 THP mmap +
# hipHostRegister) against lone-burst latency at 64 slots, and 4 slots for reference
set -o pipefail
O=gpurun_out/r03zo
mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag || true
for rnd in 1 2 3; do
  for al in 0 1 2; do
    for m in plain records; do
      GCL_TUNE_LOOP_ALLOC=$al timeout -k 10 120 ./tools/rxpipe 64 1 1 20000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"alloc\": $al, \"slots\": 64, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
  for m in plain records; do
    RXPIPE_SLOTS=4 timeout -k 10 120 ./tools/rxpipe 64 1 1 20000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"alloc\": 0, \"slots\": 4, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
  done
  GCL_TUNE_LOOP_ALLOC=2 timeout -k 10 120 ./tools/rxpipe 64 16 32 40000 | sed "s/^{/{\"mode\": \"plain\", \"alloc\": 2, \"slots\": 64, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
  timeout -k 10 120 ./tools/rxpipe 64 16 32 40000 | sed "s/^{/{\"mode\": \"plain\", \"alloc\": 0, \"slots\": 64, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zo/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['alloc'], d['slots'], d['workers'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'])
PY
