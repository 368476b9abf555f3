# rx loop: staggered multi-wave polling of the slot word (GCL_LOOP_POLLERS
# 4, default) vs one poller (1); loop GPU tests first.
set -o pipefail
O=gpurun_out/r02ax; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  for p in 4 1 2; do
    GCL_LOOP_POLLERS=$p timeout -k 10 200 python3 -u tools/rxloop_run.py 2000 > $O/p${p}_$i.json 2> $O/p${p}_$i.err || exit $?
  done
done
echo rc=0
