# round 6: 512-lane blocks at 2 per CU (one block generation), depth 1 and 2,
# against today's policy on the other dense rows: tcp1500, header split, udp64
# 2-/4-/8-B verdicts, TOEPLITZ; two fresh processes each
set -o pipefail
mkdir -p gpurun_out
F='[{},{"threads":512,"depth":1,"blocks_per_cu":2},{"threads":512,"depth":2,"blocks_per_cu":2}]'
run() { # tag, env..., workload
  local tag=$1; shift
  for i in 1 2; do
    env AB_FORMS="$F" AB_ROUNDS=2 "$@" timeout -k 10 300 python tools/tile_ab.py $WL > gpurun_out/r06y_${tag}_$i.jsonl 2> gpurun_out/r06y_${tag}_$i.err || { tail -5 gpurun_out/r06y_${tag}_$i.err; return 1; }
  done
}
WL=tcp1500 run tcp1500 AB_VBYTES=2 && WL=tcp1500_hsplit run hsplit AB_VBYTES=2 && \
WL=udp64 run udp64_v2 AB_VBYTES=2 && WL=udp64 run udp64_v4 AB_VBYTES=4 && WL=udp64 run udp64_v8 AB_VBYTES=8 && \
WL=udp64 run udp64_toep AB_HASH=toeplitz || exit 1
python - <<'PY'
import json, glob, collections
for tag in ("tcp1500", "hsplit", "udp64_v2", "udp64_v4", "udp64_v8", "udp64_toep"):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/r06y_{tag}_*.jsonl")):
        for l in open(f):
            d = json.loads(l)
            if "round" in d:
                for k in d:
                    if k.startswith("form="):
                        agg[k].append(d[k]["kernel_us"])
            elif d.get("check") != "ok":
                print("CHECK", tag, d)
    print(tag, {k: v for k, v in sorted(agg.items())})
PY
echo r06y-done
