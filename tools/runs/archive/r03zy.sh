# the bench's loop rows interleaved in three rounds (median by p50), the driver's command
set -o pipefail
O=gpurun_out/r03zy
mkdir -p $O
s=$(date +%s)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "wall_s $(( $(date +%s) - s ))"
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['e2e']['rxloop'].items(): print(k, v)
for r in d['e2e']['rx_burst_pipeline']['runs']: print(r.get('burst'), r.get('workers'), r.get('depth'), r.get('verdicts'), r.get('mpps_one_core'), r.get('mpps_samples'), r.get('burst_latency_p50_us'))"
