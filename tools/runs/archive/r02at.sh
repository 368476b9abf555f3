# Dummy loads spread onto lines the kernel already reads (default) vs one
# shared address (GCL_TUNE_ABLATE=256), both GENERAL kernels, ingress rows;
# GPU tests first.
set -o pipefail
O=gpurun_out/r02at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  for q in 1 0; do
    for a in 0 256; do
      GCL_TUNE_QUAD=$q GCL_TUNE_ABLATE=$a timeout -k 10 200 python3 -u tools/ingress_run.py 10 > $O/q${q}_a${a}_$i.json 2> $O/q${q}_a${a}_$i.err || exit $?
    done
  done
done
echo rc=0
