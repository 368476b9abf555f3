set -o pipefail
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-secondary --no-e2e --no-cpu --group-node-force > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['group']['value'], d.get('group_node'))"
