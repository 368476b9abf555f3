# round 6: the integrated working-set row against its kernel-shape ceiling,
# and its SQ instruction mix
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ingress_run.py 20 --ws-only > gpurun_out/r06k_ws.json 2> gpurun_out/r06k_ws.err || { tail -5 gpurun_out/r06k_ws.err; exit 1; }
python -c 'import json; d=json.loads(open("gpurun_out/r06k_ws.json").read().strip().splitlines()[-1]); r=d["integrated_nic_working_set"]; print(r["device_resident_mpps"], r["roofline"])'
WL=ingress_ws OUT=gpurun_out/sq_r06k timeout -k 10 900 bash tools/sqprof.sh > gpurun_out/r06k_sq.log 2>&1 || { tail -5 gpurun_out/r06k_sq.log; exit 1; }
python tools/sq_summary.py gpurun_out/sq_r06k ingress_ws > gpurun_out/r06k_sq_ws.json && cat gpurun_out/r06k_sq_ws.json
echo r06k-done
