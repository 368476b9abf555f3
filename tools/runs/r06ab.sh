# round 6: beyond 2 x 512 -- one 1024-lane block per CU (its verdicts fit LDS
# + registers in one write phase) at depth 1 and 2, and the lean waves off
# under the new geometry; udp64 1-B, three fresh processes
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{},{"threads":1024,"depth":1,"blocks_per_cu":1},{"threads":1024,"depth":2,"blocks_per_cu":1},{"tile_lean":0}]'
for i in 1 2 3; do
  AB_ROUNDS=2 timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06ab_geo_$i.jsonl 2> gpurun_out/r06ab_geo_$i.err || { tail -5 gpurun_out/r06ab_geo_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list); wins = collections.Counter()
for f in sorted(glob.glob("gpurun_out/r06ab_geo_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if "round" in d:
            ks = [k for k in d if k.startswith("form=")]
            wins[min(ks, key=lambda k: d[k]["kernel_us"])] += 1
            for k in ks:
                agg[k].append((d[k]["kernel_us"], d[k]["probe_us"]))
        elif d.get("check") != "ok":
            print("CHECK", d)
for k in sorted(agg):
    print(k, agg[k])
print("fastest per round:", dict(wins))
PY
echo r06ab-done
