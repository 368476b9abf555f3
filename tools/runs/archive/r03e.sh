# round 3: the pair kernel on bench's GENERAL rows (device, zero-copy, trace)
# and its SQ counters on the working set
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 600 python -u tools/general_ab.py 2 > $O/general_ab.jsonl 2> $O/general_ab.err || { tail $O/general_ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/general_ab.jsonl'):
    d=json.loads(l); i=d['ingress_pool']
    print(d['round'], d['GCL_TUNE_PAIR'], i['integrated_nic']['roofline']['kernel_ms'], i['integrated_nic']['zerocopy_mpps'], i['jenkins_offs_only']['kernel_ms'], i['integrated_nic_working_set']['roofline']['kernel_ms'], d['trace_replay']['zerocopy_mpps'])
"
GCL_TUNE_PAIR=1 WL=ingress_ws OUT=gpurun_out/sq_r03_pair timeout -k 10 600 bash tools/sqprof.sh > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
echo done
