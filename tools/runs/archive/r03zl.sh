# lone-burst latency in rxpipe: pinned near the GPU (default) vs unpinned, plain and header records
set -o pipefail
O=gpurun_out/r03zl
mkdir -p $O
for rnd in 1 2 3; do
  for pin in 1 0; do
    for m in plain records; do
      RXPIPE_PIN=$pin GCL_LOOP_DEBUG=1 timeout -k 10 120 ./tools/rxpipe 64 1 1 20000 $( [ $m = plain ] || echo $m ) 2>>$O/dbg.txt | sed "s/^{/{\"mode\": \"$m\", \"pin\": $pin, \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zl/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['pin'], d['mode'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['host_cpu'])
PY
sort $O/dbg.txt | uniq -c | head
cat /sys/devices/system/node/online; lscpu | grep -i "numa node" | head
