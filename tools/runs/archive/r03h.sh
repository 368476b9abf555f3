# round 3: the driver's sequence on the current tree: smoke, then the bench
# line with the driver's flags
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['group'], d['secondary']['value'], d['secondary']['roofline']['frac'])
print(json.dumps(d['e2e']['rx_burst_pipeline'])[:1500])
print(d['e2e']['ingress_pool']['integrated_nic_working_set']['roofline']['kernel_ms'], d['e2e']['ingress_pool']['integrated_nic']['roofline']['frac'])
print(d['placement']['kernel_checks'], d['secondary']['header_split_layout']['placement'].get('kernel_checks'))
print(d['cpu_baseline']['nic_mode'])
"
echo done
