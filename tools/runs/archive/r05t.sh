# round 5, final tree: the one-process multi-GPU step forced onto the one GPU
# (group_node), and the launcher-less --gpus 2 rehearsal (gloo, shared GPU)
set -o pipefail
mkdir -p gpurun_out
GCL_BENCH_DETAIL=gpurun_out/r05t_gn_detail.json timeout -k 10 500 python bench.py --group-node-force --no-cpu --no-secondary --no-e2e > gpurun_out/r05t_group_node.json 2> gpurun_out/r05t_group_node.err || { tail -5 gpurun_out/r05t_group_node.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05t_group_node.json')); print(d['value'], d.get('group'), d.get('group_node'))"
GCL_BENCH_DETAIL=gpurun_out/r05t_gloo2_detail.json timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 20 --warmup 2 > gpurun_out/r05t_gloo2.json 2> gpurun_out/r05t_gloo2.err || { tail -5 gpurun_out/r05t_gloo2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05t_gloo2.json')); print(d['n_gpus'], d['value'], d.get('counts_check'), d.get('kernel_only',{}).get('value'), len(json.dumps(d)))"
