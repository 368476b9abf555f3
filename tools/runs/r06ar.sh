# round 6: where the header-split launch's fixed costs go (0.87 of the 512-MiB
# read speed of light): the default against per-packet verdict stores, tables
# in HBM (no LDS staging), depth 2, 256-lane tiles, one block per CU
set -o pipefail
mkdir -p gpurun_out
FORMS='[{}, {"defer": 0}, {"tables": 1}, {"depth": 2}, {"threads": 256}, {"blocks_per_cu": 1}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/tile_ab.py tcp1500_hsplit tcp1500 > gpurun_out/r06ar_hsplit_ab_$i.jsonl 2> gpurun_out/r06ar_hsplit_ab_$i.err || { tail -5 gpurun_out/r06ar_hsplit_ab_$i.err; exit 1; }
done
python - gpurun_out/r06ar_hsplit_ab_*.jsonl <<'PY'
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
        agg[(r["workload"], "minimal")].append(r["minimal_probe_us"])
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06ar-done
