# round 6: SQ instruction mix of the final tree's udp64 tile kernel and the
# working-set pair kernel
set -o pipefail
mkdir -p gpurun_out
WL=udp64 OUT=gpurun_out/sq_r06s timeout -k 10 600 bash tools/sqprof.sh > gpurun_out/r06s_sq_udp64.log 2>&1 || { tail -5 gpurun_out/r06s_sq_udp64.log; exit 1; }
WL=ingress_ws OUT=gpurun_out/sq_r06s timeout -k 10 600 bash tools/sqprof.sh > gpurun_out/r06s_sq_ws.log 2>&1 || { tail -5 gpurun_out/r06s_sq_ws.log; exit 1; }
python tools/sq_summary.py gpurun_out/sq_r06s udp64 > gpurun_out/r06s_sq_udp64.json && python tools/sq_summary.py gpurun_out/sq_r06s ingress_ws > gpurun_out/r06s_sq_ws.json
python - <<'PY'
import json
for f in ("gpurun_out/r06s_sq_udp64.json", "gpurun_out/r06s_sq_ws.json"):
    d = json.load(open(f))
    print(f, d.get("kernel"), d.get("waves_per_launch"), json.dumps(d.get("per_wave")), json.dumps(d.get("over_wave_cycles")))
PY
echo r06s-done
