# rxpipe burst-64 rows, pinned (last GPU-local CPU) vs unpinned, interleaved
set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
for rep in 1 2 3; do
for pin in 1 0; do
for cfg in "64 4 8 20000" "64 8 16 40000" "64 16 32 40000" "64 16 32 40000 inline"; do
  RXPIPE_PIN=$pin timeout -k 10 120 ./tools/rxpipe $cfg | sed "s/^{/{\"pin\": $pin, /" >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
done
done
nproc; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; taskset -pc $$
python3 -c "
import json
for l in open('$O/rxpipe.jsonl'):
    d=json.loads(l); print(d['pin'], d['burst'], d['workers'], d['depth'], d['verdicts'][:30], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['host_cpu'])"
