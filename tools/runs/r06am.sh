# round 6: classify_kernel's tile order (gcl_tune.tile_order): round-robin (0)
# against one contiguous run per block (1), after tools/read_sol found
# block-contiguous streaming reads ~5 % faster than grid-stride ones.  Parity
# of the deferred-flush and tune cases, then the A/B in three fresh processes
# (udp64 1-B and tcp1500 2-B), and udp64 4-B once
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deferred_flushes or ctx_tune or narrow or access_probe" > gpurun_out/r06am_tests.log 2>&1 || { tail -30 gpurun_out/r06am_tests.log; exit 1; }
tail -1 gpurun_out/r06am_tests.log
for i in 1 2 3; do
  AB_KNOB=tile_order timeout -k 10 300 python tools/tile_ab.py udp64 tcp1500 > gpurun_out/r06am_order_ab_$i.jsonl 2> gpurun_out/r06am_order_ab_$i.err || { tail -5 gpurun_out/r06am_order_ab_$i.err; exit 1; }
done
AB_KNOB=tile_order AB_VBYTES=4 timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06am_order_ab_v4.jsonl 2> gpurun_out/r06am_order_ab_v4.err || { tail -5 gpurun_out/r06am_order_ab_v4.err; exit 1; }
python - gpurun_out/r06am_order_ab_*.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for l in open(f):
        r = json.loads(l)
        if "check" in r:
            if r["check"] != "ok": print("MISMATCH", f, r)
            continue
        tag = r["workload"] + ("_v4" if f.endswith("v4.jsonl") else "")
        for k, v in r.items():
            if k.startswith("tile_order="):
                agg[(tag, k)].append((v["kernel_us"], v["probe_us"]))
for k in sorted(agg):
    print(k, agg[k])
PY
echo r06am-done
