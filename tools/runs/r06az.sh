# round 6: lines in flight for udp64 with per-packet 4-/8-B verdicts (no
# deferral, depth 2): 2 x 512 at depth 2 (default) against 2 x 256 at depth 2
# and at depth 1; two fresh processes each
set -o pipefail
mkdir -p gpurun_out
F='[{}, {"threads": 256}, {"threads": 256, "depth": 1}]'
for vb in 4 8; do
  for i in 1 2; do
    AB_FORMS="$F" AB_VBYTES=$vb timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06az_v${vb}_$i.jsonl 2> gpurun_out/r06az_v${vb}_$i.err || { tail -5 gpurun_out/r06az_v${vb}_$i.err; exit 1; }
  done
done
python - gpurun_out/r06az_v*.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    tag = f.split("_")[-2]
    for l in open(f):
        r = json.loads(l)
        if "check" in r:
            if r["check"] != "ok": print("MISMATCH", r)
            continue
        for k, v in r.items():
            if k.startswith("form="):
                agg[(tag, k)].append((v["kernel_us"], v["probe_us"]))
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06az-done
