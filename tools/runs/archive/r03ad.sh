# rx loop variants, interleaved in one call: old (HEAD before round 3's poll
# change), vb (stop flag beside every poll, offsets polled always), new (stop
# beside every 8th poll, offsets polled for the first 4 us of a wait)
set -o pipefail
O=gpurun_out/r03ad
mkdir -p $O
for rep in 1 2 3 4 5 6; do
for cfg in "64 1 1 20000" "64 4 8 20000" "64 8 16 40000" "64 16 32 40000"; do
  for v in old vb new; do
    exe=./tools/rxpipe; [ $v = old ] && exe=./tools/_scratch/rxpipe_old; [ $v = vb ] && exe=./tools/_scratch/rxpipe_vb
    timeout -k 10 120 $exe $cfg | sed "s/^{/{\"v\": \"$v\", /" >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
  done
done
done
python3 - <<PY
import json, collections
rows = collections.defaultdict(list)
for l in open('$O/rxpipe.jsonl'):
    d = json.loads(l)
    rows[(d['burst'], d['workers'], d['depth'], d['v'])].append((d['mpps_one_core'], d['burst_latency_p50_us']))
for k in sorted(rows):
    m = sorted(x[0] for x in rows[k]); p = sorted(x[1] for x in rows[k])
    print(k, 'mpps med', m[len(m)//2], 'all', m, 'p50 med', p[len(p)//2])
PY
