# round 3: ARP target as one dword read (pair + tile kernels): parity, then
# bench's GENERAL rows A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u tools/general_ab.py 3 > $O/general_ab.jsonl 2> $O/general_ab.err || { tail $O/general_ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/general_ab.jsonl'):
    d=json.loads(l); i=d['ingress_pool']
    print(d['round'], d['GCL_TUNE_PAIR'], i['integrated_nic']['roofline']['kernel_ms'], i['integrated_nic']['zerocopy_mpps'], i['jenkins_offs_only']['kernel_ms'], i['integrated_nic_working_set']['roofline']['kernel_ms'], d['trace_replay']['zerocopy_mpps'])
"
echo done
