# Spread dummy loads, tile kernel default, quad kernel behind GCL_TUNE_QUAD:
# GPU tests (quad fuzz + loop geometries), the driver's bench command, ingress.
set -o pipefail
O=gpurun_out/r02au; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/ingress_run.py 10 > $O/ingress_$i.json 2> $O/ingress_$i.err || exit $?
done
echo rc=0
