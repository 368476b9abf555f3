# round 6: classify_pair_kernel without the eager waits (offset clamp at its
# use, every loaded dword live until the exchange): pair-kernel parity, then
# the ingress-pool leg three times (random pool, working set, their ceilings)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or offsets or fuzz or ingress or golden or access_probe" > gpurun_out/r06l_tests.log 2>&1 || { tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/ingress_run.py 20 > gpurun_out/r06l_ingress_$i.json 2> gpurun_out/r06l_ingress_$i.err || { tail -5 gpurun_out/r06l_ingress_$i.err; exit 1; }
  python - gpurun_out/r06l_ingress_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("integrated_nic", "jenkins_offs_only", "integrated_nic_working_set"):
    r = d.get(k, {})
    rf = r.get("roofline", {})
    print(k, r.get("device_resident_mpps"), r.get("counts_check"), {x: rf.get(x) for x in ("frac", "kernel_ms", "ceiling_ms", "frac_of_ceiling")}, r.get("kernel_ms"))
PY
done
echo r06l-done
