# round 6: the headline's launch geometry re-checked with the round-6 forms
# (lean waves, deferred verdicts with the staged register flush): threads
# 256 / 512 / 1024 and depth 1 / 2, each beside its kernel-shape ceiling,
# two fresh processes per knob
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  AB_KNOB=threads AB_VALUES=256,512,1024 timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06u_threads_$i.jsonl 2> gpurun_out/r06u_threads_$i.err || { tail -5 gpurun_out/r06u_threads_$i.err; exit 1; }
  AB_KNOB=depth AB_VALUES=2,1 timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06u_depth_$i.jsonl 2> gpurun_out/r06u_depth_$i.err || { tail -5 gpurun_out/r06u_depth_$i.err; exit 1; }
done
python - <<'PY'
import json, glob, collections
for kn in ("threads", "depth"):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/r06u_{kn}_*.jsonl")):
        for l in open(f):
            d = json.loads(l)
            if "round" in d:
                for k, v in d.items():
                    if "=" in k:
                        agg[k].append((v["kernel_us"], v["probe_us"]))
            elif d.get("check") != "ok":
                print("CHECK", d)
    for k in sorted(agg):
        print(k, agg[k])
PY
echo r06u-done
