# round 6: the pair kernel's geometry under its round-6 forms (lean waves,
# 32-bit): 4 x 256 (default) against 2 x 512 and 1 x 1024 lanes per CU, on
# the integrated ingress rows, three fresh processes
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{},{"threads":512,"blocks_per_cu":2},{"threads":1024,"blocks_per_cu":1},{"threads":256,"blocks_per_cu":2}]'
for i in 1 2 3; do
  timeout -k 10 300 python tools/pair_lean_ab.py 2 > gpurun_out/r06ac_pair_geo_$i.jsonl 2> gpurun_out/r06ac_pair_geo_$i.err || { tail -5 gpurun_out/r06ac_pair_geo_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r06ac_pair_geo_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if "kernel_us" in d:
            agg[(d["row"], d["form"])].append(d["kernel_us"])
        elif d.get("check") != "ok":
            print("CHECK", d)
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06ac-done
