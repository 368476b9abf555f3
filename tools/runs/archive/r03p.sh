# round 3: plain vs non-temporal frame loads in the pair kernel, same process;
# then bench's GENERAL rows (device, zero-copy, trace replay) on the plain build
set -o pipefail
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python -u tools/ws_ab.py 3 ntl=GCL_TUNE_PAIR_LOADS:1 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ws_ab.jsonl'):
    r=json.loads(l); d[(r['set'],r['row'])].append((r['kernel_us'], r.get('verdicts_match_default')))
for k,v in sorted(d.items()): print(k, v)
"
timeout -k 10 600 python -u tools/general_ab.py 2 > $O/general_ab.jsonl 2> $O/general_ab.err || { tail $O/general_ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/general_ab.jsonl'):
    d=json.loads(l); i=d['ingress_pool']
    print(d['round'], d['GCL_TUNE_PAIR'], i['integrated_nic']['roofline']['kernel_ms'], i['integrated_nic']['zerocopy_mpps'], i['jenkins_offs_only']['kernel_ms'], i['integrated_nic_working_set']['roofline']['kernel_ms'], d['trace_replay']['zerocopy_mpps'])
"
