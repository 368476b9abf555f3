# round 6: the new dense geometry as the default (2 x 512 lanes per CU, depth
# 1 where a dense slab's block defers its verdicts): the whole GPU suite, then
# the default against round 5's 4 x 256 at depth 2 on udp64 and tcp1500,
# three fresh processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06z_gputests.log 2>&1 || { tail -30 gpurun_out/r06z_gputests.log; exit 1; }
tail -1 gpurun_out/r06z_gputests.log
export AB_FORMS='[{},{"threads":256,"depth":2,"blocks_per_cu":4}]'
for i in 1 2 3; do
  AB_ROUNDS=2 timeout -k 10 300 python tools/tile_ab.py udp64 tcp1500 > gpurun_out/r06z_geo_$i.jsonl 2> gpurun_out/r06z_geo_$i.err || { tail -5 gpurun_out/r06z_geo_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r06z_geo_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if "round" in d:
            for k in d:
                if k.startswith("form="):
                    agg[(d["workload"], k)].append((d[k]["kernel_us"], d[k]["probe_us"], d[k]["frac"]))
        elif d.get("check") != "ok":
            print("CHECK", d)
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06z-done
