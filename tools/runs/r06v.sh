# round 6: the headline geometry, several knobs per form (tile_ab AB_FORMS):
# 4 x 256 (today) against 2 x 512, each at depth 2 and 1, three fresh processes
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{"threads":256},{"threads":512},{"threads":256,"depth":1},{"threads":512,"depth":1}]'
for i in 1 2 3; do
  timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06v_geo_$i.jsonl 2> gpurun_out/r06v_geo_$i.err || { tail -5 gpurun_out/r06v_geo_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
wins = collections.Counter()
for f in sorted(glob.glob("gpurun_out/r06v_geo_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if "round" in d:
            ks = [k for k in d if k.startswith("form=")]
            best = min(ks, key=lambda k: d[k]["kernel_us"])
            wins[best] += 1
            for k in ks:
                agg[k].append(d[k]["kernel_us"])
        elif d.get("check") != "ok":
            print("CHECK", d)
        else:
            print(d)
for k in sorted(agg):
    print(k, agg[k])
print("fastest per round:", dict(wins))
PY
echo r06v-done
