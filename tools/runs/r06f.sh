# round 6: the cold-header pipeline rows with the pool in 2 MiB pages and the records submit prefetching 16 headers ahead; then the hot-header records rows for the prefetch change
# (rxpipe RXPIPE_POOL=ingress records / stamped offsets, tools/cpupipe classify / + lrpc_send,
# three fresh processes per row, through bench.py's own leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -c '
import json, bench
out = bench.ingress_pipeline_bench()
print(json.dumps(out))
' > gpurun_out/r06f_ingress.json 2> gpurun_out/r06f_ingress.err || { tail -20 gpurun_out/r06f_ingress.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06f_ingress.json").read().strip().splitlines()[-1])
for r in d["gpu"] + d["cpu"]:
    print({k: r.get(k) for k in ("pipeline", "workers", "batch", "record", "mpps", "mpps_one_core", "mpps_samples", "nic_wait_frac", "p50_us", "error")})
PY

for i in 1 2 3; do
  for cfg in "1 1 20000" "4 8 20000"; do
    RXPIPE_HASH=nic timeout -k 10 120 tools/rxpipe 64 $cfg records > gpurun_out/r06f_hot_$i.json 2>&1 || { cat gpurun_out/r06f_hot_$i.json; exit 1; }
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print("hot", d["workers"], d["depth"], d["mpps_one_core"], d["burst_latency_p50_us"], d["submit_ns_per_pkt"], d["deliver_ns_per_pkt"])' gpurun_out/r06f_hot_$i.json
  done
done
echo r06f-done
