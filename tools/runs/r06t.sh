# round 6: classify_pair_kernel's 32-bit form (gcl_tune.pair_i32): the pair /
# offsets / ingress parity tests, then the A/B on the integrated ingress rows
# (random pool, working set) in three fresh processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06t_tests.log 2>&1 || { tail -30 gpurun_out/r06t_tests.log; exit 1; }
tail -1 gpurun_out/r06t_tests.log
for i in 1 2 3; do
  AB_KNOB=pair_i32 timeout -k 10 300 python tools/pair_lean_ab.py 3 > gpurun_out/r06t_i32_ab_$i.jsonl 2> gpurun_out/r06t_i32_ab_$i.err || { tail -5 gpurun_out/r06t_i32_ab_$i.err; exit 1; }
  python - gpurun_out/r06t_i32_ab_$i.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows:
    if "kernel_us" in r:
        agg[(r["row"], r["form"])].append(r["kernel_us"])
    else:
        print(r)
for k in sorted(agg):
    print(k, agg[k])
PY
done
echo r06t-done
