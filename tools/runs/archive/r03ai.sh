# rx loop host side: prefetch of the next burst's verdict records (new) vs none (np), interleaved
set -o pipefail
O=gpurun_out/r03ai${RUN:-}
mkdir -p $O
for rep in 1 2 3 4; do
for cfg in "64 1 1 20000" "64 8 16 40000" "64 16 32 40000" "64 32 64 60000"; do
  for v in np new; do
    exe=./tools/rxpipe; [ $v = np ] && exe=./tools/_scratch/rxpipe_np
    timeout -k 10 120 $exe $cfg | sed "s/^{/{\"v\": \"$v\", /" >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
  done
done
done
python3 - <<PY
import json, collections
rows = collections.defaultdict(list)
for l in open('$O/rxpipe.jsonl'):
    d = json.loads(l)
    rows[(d['burst'], d['workers'], d['depth'], d['v'])].append((d['mpps_one_core'], d['burst_latency_p50_us'], d['wait_ns_per_pkt'], d['deliver_ns_per_pkt']))
for k in sorted(rows):
    m = sorted(x[0] for x in rows[k]); w = sorted(x[2] for x in rows[k]); dl = sorted(x[3] for x in rows[k])
    print(k, 'mpps', m, 'wait med', w[len(w)//2], 'deliver med', dl[len(dl)//2])
PY
