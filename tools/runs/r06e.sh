# round 6: the cold-header pipeline rows after the NIC
# threads moved off the dataplane core: rxpipe RXPIPE_POOL=ingress (records,
# stamped offsets) and tools/cpupipe (classify, + lrpc_send) on identical
# inputs, three fresh processes per row, through bench.py's own leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -c '
import json, bench
out = bench.ingress_pipeline_bench()
print(json.dumps(out))
' > gpurun_out/r06e_ingress.json 2> gpurun_out/r06e_ingress.err || { tail -20 gpurun_out/r06e_ingress.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06e_ingress.json").read().strip().splitlines()[-1])
for r in d["gpu"] + d["cpu"]:
    print({k: r.get(k) for k in ("pipeline", "workers", "batch", "record", "mpps", "mpps_one_core", "mpps_samples", "nic_wait_frac", "p50_us", "error")})
PY
echo r06e-done
