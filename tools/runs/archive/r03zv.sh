# the driver's bench command with the pipeline rows as medians of three processes; wall time
set -o pipefail
O=gpurun_out/r03zv
mkdir -p $O
s=$(date +%s)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "wall_s $(( $(date +%s) - s ))"
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for r in d['e2e']['rx_burst_pipeline']['runs']: print(r.get('burst'), r.get('workers'), r.get('depth'), r.get('verdicts'), r.get('mpps_one_core'), r.get('mpps_samples'), r.get('burst_latency_p50_us'))
print(d['cpu_baseline']['nic_mode']['1core_lrpc_mpps'])"
