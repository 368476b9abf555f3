# lone-burst latency in rxpipe against the ring's slot count (the bench's loop rows use 16, rxpipe 64)
set -o pipefail
O=gpurun_out/r03zn
mkdir -p $O
for rnd in 1 2 3; do
  for sl in 64 16 4; do
    for m in plain records; do
      RXPIPE_SLOTS=$sl timeout -k 10 120 ./tools/rxpipe 64 1 1 20000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"slots\": $sl, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
  for sl in 64 16; do
    RXPIPE_SLOTS=$sl timeout -k 10 120 ./tools/rxpipe 64 4 8 20000 records | sed "s/^{/{\"mode\": \"records\", \"slots\": $sl, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
  done
done
timeout -k 10 200 python3 -c "
import torch, json, bench, caladan_amd.gclassify as g
print(json.dumps(bench.rxloop_bench(torch.device('cuda:0'), 2)))" > $O/rxloop_bench.json 2> $O/rxloop_bench.err || { tail $O/rxloop_bench.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zn/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['slots'], d['workers'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'])
d=json.load(open('gpurun_out/r03zn/rxloop_bench.json'))
for k,v in d.items():
    if k.startswith('loop_burst64'): print(k, v)
PY
