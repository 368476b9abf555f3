# round 6: what made 512 lanes at depth 1 fastest -- the tile size, the
# depth, or a grid of two block generations (blocks_per_cu stays 4 while 2
# blocks of 512 fit): udp64 1-B, three fresh processes
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{},{"threads":512,"depth":1},{"threads":512,"depth":1,"blocks_per_cu":2},{"threads":256,"depth":1,"grid":2048},{"threads":512,"depth":2,"blocks_per_cu":2},{"threads":256,"depth":2,"grid":2048},{"threads":512,"depth":1,"grid":1536}]'
for i in 1 2 3; do
  AB_ROUNDS=2 timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06x_geo_$i.jsonl 2> gpurun_out/r06x_geo_$i.err || { tail -5 gpurun_out/r06x_geo_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list); probe = collections.defaultdict(list)
wins = collections.Counter()
for f in sorted(glob.glob("gpurun_out/r06x_geo_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if "round" in d:
            ks = [k for k in d if k.startswith("form=")]
            wins[min(ks, key=lambda k: d[k]["kernel_us"])] += 1
            for k in ks:
                agg[k].append(d[k]["kernel_us"]); probe[k].append(d[k]["probe_us"])
        elif d.get("check") != "ok":
            print("CHECK", d)
for k in sorted(agg):
    print(k, agg[k], "probe", probe[k])
print("fastest per round:", dict(wins))
PY
echo r06x-done
