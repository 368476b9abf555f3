# round 3: verdict store policy on the pair kernel's working-set row
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python -u tools/ws_ab.py 3 st_plain=GCL_TUNE_NT_STORE:0 st_nt=GCL_TUNE_NT_STORE:1 pair8=GCL_TUNE_PAIR:2 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ws_ab.jsonl'):
    r=json.loads(l); d[(r['set'],r['row'])].append((r['kernel_us'], r.get('verdicts_match_default')))
for k,v in sorted(d.items()): print(k, v)
"
echo done
