# round 6: classify_kernel's verdict registers 10 -> 16 dwords per lane (32
# tiles of 2-B verdicts past a full LDS buffer), so the 1024-runtime contexts
# (7 tiles of LDS room beside their 37-KiB tables) write their verdicts once,
# after the reads, rather than once mid-run; against r06as (10 registers):
# tcp1500 172.3-173.2 us, header split 86.1-86.3; udp64 307-309 (r06am)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06at_tests.log 2>&1 || { tail -30 gpurun_out/r06at_tests.log; exit 1; }
tail -1 gpurun_out/r06at_tests.log
FORMS='[{}, {"threads": 256, "depth": 1}]'
for i in 1 2; do
  AB_FORMS="$FORMS" timeout -k 10 300 python tools/tile_ab.py udp64 tcp1500 tcp1500_hsplit > gpurun_out/r06at_ab_$i.jsonl 2> gpurun_out/r06at_ab_$i.err || { tail -5 gpurun_out/r06at_ab_$i.err; exit 1; }
done
python - gpurun_out/r06at_ab_*.jsonl <<'PY'
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
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06at-done
