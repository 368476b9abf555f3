# round 6: lines in flight per CU for the pair kernel (the r06au finding for
# wide slots): 2 x 512 (default) against 2 x 256 and 1 x 512 (half the lines
# in flight) and 4 x 256, on the ingress random pool and working set
set -o pipefail
mkdir -p gpurun_out
FORMS='[{}, {"threads": 256}, {"threads": 512, "blocks_per_cu": 1}, {"threads": 256, "blocks_per_cu": 4}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/pair_lean_ab.py 3 > gpurun_out/r06av_pair_ab_$i.jsonl 2> gpurun_out/r06av_pair_ab_$i.err || { tail -5 gpurun_out/r06av_pair_ab_$i.err; exit 1; }
done
python - gpurun_out/r06av_pair_ab_*.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for l in open(f):
        r = json.loads(l)
        if "kernel_us" in r:
            agg[(r["row"], r["form"])].append(r["kernel_us"])
        elif r.get("check") != "ok":
            print(r)
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06av-done
