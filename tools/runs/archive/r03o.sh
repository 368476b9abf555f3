# round 3: cache hints of the pair kernel's loads on the working set / random pool
set -o pipefail
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 600 python -u tools/ws_ab.py 3 ld1=GCL_TUNE_PAIR_LOADS:1 ld2=GCL_TUNE_PAIR_LOADS:2 ld3=GCL_TUNE_PAIR_LOADS:3 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ws_ab.jsonl'):
    r=json.loads(l); d[(r['set'],r['row'])].append((r['kernel_us'], r.get('verdicts_match_default')))
for k,v in sorted(d.items()): print(k, v)
"
