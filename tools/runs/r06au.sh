# round 6: wide slots (stride > 64) on 256-lane tiles at depth 1, two blocks
# per CU (the default now) against the former 2 x 512 at depth 2; parity, the
# A/B in two fresh processes, then the driver's bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06au_tests.log 2>&1 || { tail -30 gpurun_out/r06au_tests.log; exit 1; }
tail -1 gpurun_out/r06au_tests.log
FORMS='[{}, {"threads": 512, "depth": 2}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/tile_ab.py tcp1500 > gpurun_out/r06au_ab_$i.jsonl 2> gpurun_out/r06au_ab_$i.err || { tail -5 gpurun_out/r06au_ab_$i.err; exit 1; }
done
python - gpurun_out/r06au_ab_*.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for l in open(f):
        r = json.loads(l)
        if "check" in r:
            if r["check"] != "ok": print("MISMATCH", r)
            continue
        for k, v in r.items():
            if k.startswith("form="):
                agg[(r["workload"], k)].append((v["kernel_us"], v["probe_us"]))
for k in sorted(agg):
    print(k, agg[k])
PY
GCL_BENCH_DETAIL=gpurun_out/r06au_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06au_bench.json 2> gpurun_out/r06au_bench.err || { tail -5 gpurun_out/r06au_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06au_bench.json").readline())
s = d["secondary"]
print("udp64", d["value"], d["roofline"]["frac"], "tcp1500", s["value"], s["roofline"]["frac"], s["roofline"]["frac_of_ceiling"], s["roofline"]["kernel_ms"])
PY
echo r06au-done
