# round 6: the pair kernel's 32-bit form with scalar tile tests, straight-line
# pair_src and range-checked frame loads (no select per load), classify_lean
# with the verdict width known: parity, the pair_i32 A/B on the ingress rows in
# three fresh processes, then the bench line with timed_launches' 10-ms window
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ak_tests.log 2>&1 || { tail -30 gpurun_out/r06ak_tests.log; exit 1; }
tail -1 gpurun_out/r06ak_tests.log
for i in 1 2 3; do
  AB_KNOB=pair_i32 timeout -k 10 300 python tools/pair_lean_ab.py 3 > gpurun_out/r06ak_i32_ab_$i.jsonl 2> gpurun_out/r06ak_i32_ab_$i.err || { tail -5 gpurun_out/r06ak_i32_ab_$i.err; exit 1; }
  python - gpurun_out/r06ak_i32_ab_$i.jsonl <<'PY'
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
timeout -k 10 900 python -u bench.py > gpurun_out/r06ak_bench.json 2> gpurun_out/r06ak_bench.err || { tail -20 gpurun_out/r06ak_bench.err; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/r06ak_bench_detail.json
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06ak_bench.json").readline())
e = d["e2e"]
print("udp64", d["value"], d["roofline"]["frac"], "ws", e["ingress_working_set_nic"], "ingress", e["ingress_integrated_nic"]["device_resident_mpps"])
PY
echo r06ak-done
