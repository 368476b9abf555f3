# Register-header GENERAL kernel (classify_quad_kernel): GPU tests with it as
# the default, then the ingress rows alternating GCL_TUNE_QUAD=1/0 in fresh
# processes.
set -o pipefail
O=gpurun_out/r02ap; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  for q in 1 0; do
    GCL_TUNE_QUAD=$q timeout -k 10 300 python3 -u tools/ingress_run.py 10 > $O/ingress_q${q}_$i.json 2> $O/ingress_q${q}_$i.err || exit $?
  done
done
echo rc=0
