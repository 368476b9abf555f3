# round 6: the pair kernel at 2 x 256 lanes per CU (the default now) against
# 2 x 512: parity, the A/B on the ingress rows, then the driver's bench command
# (its zero-copy ingress row runs the pair kernel over PCIe)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06aw_tests.log 2>&1 || { tail -30 gpurun_out/r06aw_tests.log; exit 1; }
tail -1 gpurun_out/r06aw_tests.log
FORMS='[{}, {"threads": 512}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/pair_lean_ab.py 3 > gpurun_out/r06aw_pair_ab_$i.jsonl 2> gpurun_out/r06aw_pair_ab_$i.err || { tail -5 gpurun_out/r06aw_pair_ab_$i.err; exit 1; }
done
python - gpurun_out/r06aw_pair_ab_*.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for l in open(f):
        r = json.loads(l)
        if "kernel_us" in r:
            agg[(r["row"], r["form"])].append(r["kernel_us"])
        elif r.get("check") != "ok":
            print(r)
for k in sorted(agg):
    print(k, agg[k])
PY
GCL_BENCH_DETAIL=gpurun_out/r06aw_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06aw_bench.json 2> gpurun_out/r06aw_bench.err || { tail -5 gpurun_out/r06aw_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06aw_bench.json").readline())
e = d["e2e"]
print("udp64", d["value"], d["roofline"]["frac"], "tcp1500", d["secondary"]["value"], "ws", e["ingress_working_set_nic"], "ingress", e["ingress_integrated_nic"], "mixed", e["mixed"], e["mixed_trace_replay_mpps"])
PY
echo r06aw-done
