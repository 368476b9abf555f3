# round 6: table staging with every lane's loads issued before its LDS stores
# (stage_tables), against the r06ar numbers of the loop it replaces; and the
# 1024-runtime geometry for tcp1500: 2 x 256 at depth 2 / 1, 2 x 512 at depth 1,
# 1 x 1024
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06as_tests.log 2>&1 || { tail -30 gpurun_out/r06as_tests.log; exit 1; }
tail -1 gpurun_out/r06as_tests.log
FORMS='[{}, {"tables": 1}, {"threads": 256}, {"threads": 256, "depth": 1}, {"threads": 512, "depth": 1}, {"threads": 1024, "blocks_per_cu": 1, "depth": 1}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/tile_ab.py tcp1500_hsplit tcp1500 > gpurun_out/r06as_geo_ab_$i.jsonl 2> gpurun_out/r06as_geo_ab_$i.err || { tail -5 gpurun_out/r06as_geo_ab_$i.err; exit 1; }
done
python - gpurun_out/r06as_geo_ab_*.jsonl <<'PY'
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
echo r06as-done
