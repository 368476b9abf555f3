# round 5: the CPU baseline with classify-only and classify + lrpc_send timed
# with the 1-core cells before the all-cores ones -- r05j still had the lrpc
# cell 3 % above classify-only -- via the driver's bench command
set -o pipefail
mkdir -p gpurun_out
GCL_BENCH_DETAIL=gpurun_out/r05k_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r05k_bench.json 2> gpurun_out/r05k_bench.err || { tail -5 gpurun_out/r05k_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/r05k_bench_detail.json'))['cpu_baseline']
for s,v in d['streams'].items():
    for m in ('nic_mode','jenkins_mode'):
        x=v[m]; print(s, m, x['1core_mpps'], x['1core_lrpc_mpps'], x['all_cores_mpps'], x['spread_1core'], x['spread_all_cores'])
"
