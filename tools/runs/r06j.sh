# round 6: the pair kernel's probe mode (gcl_access_probe for batches with
# offsets): the probe tests, then the ingress-pool leg alone twice (its
# frac_of_ceiling against the kernel-shape ceiling)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "access_probe or pair_lean or offsets" > gpurun_out/r06j_tests.log 2>&1 || { tail -30 gpurun_out/r06j_tests.log; exit 1; }
tail -1 gpurun_out/r06j_tests.log
for i in 1 2; do
  timeout -k 10 300 python tools/ingress_run.py 20 > gpurun_out/r06j_ingress_$i.json 2> gpurun_out/r06j_ingress_$i.err || { tail -5 gpurun_out/r06j_ingress_$i.err; exit 1; }
  python - gpurun_out/r06j_ingress_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def walk(x, p=""):
    if isinstance(x, dict):
        if "frac_of_ceiling" in x or "device_resident_mpps" in x:
            print(p, {k: x.get(k) for k in ("device_resident_mpps", "kernel_ms", "frac", "ceiling_ms", "frac_of_ceiling")},
                  {k: x["roofline"].get(k) for k in ("frac", "kernel_ms", "ceiling_ms", "frac_of_ceiling")} if "roofline" in x else "")
        for k, v in x.items():
            walk(v, p + "/" + k)
walk(d)
PY
done
echo r06j-done
