# round 3: what the verdict stores cost the pair kernel on the working set
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 600 python -u tools/ws_ab.py 3 pair_abl=GCL_TUNE_ABLATE:128 no_store=GCL_TUNE_ABLATE:512 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ws_ab.jsonl'):
    r=json.loads(l); d[(r['set'],r['row'])].append((r['kernel_us'], r.get('verdicts_match_default')))
for k,v in sorted(d.items()): print(k, v)
"
echo done
