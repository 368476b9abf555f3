# Buffer loads: dense tiles (GCL_TUNE_LDAUX default 18 = sc1 nt; 2 = nt;
# -1 = the former global_load nt) and GENERAL chunks (GCL_TUNE_GBUF=1).
# GPU tests first (dense default), a GENERAL-buffer parity pass, then
# udp64 / tcp1500 kernel-only lines and the ingress rows, fresh processes.
set -o pipefail
O=gpurun_out/r02bj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
GCL_TUNE_GBUF=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_gbuf.log 2>&1 || { tail -30 $O/gpu_tests_gbuf.log; exit 1; }
tail -1 $O/gpu_tests_gbuf.log
for i in 1 2; do
  for a in 18 2 -1; do
    GCL_TUNE_LDAUX=$a timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 100 > $O/udp_a${a}_$i.json 2> $O/udp_a${a}_$i.err || exit $?
    GCL_TUNE_LDAUX=$a timeout -k 10 300 python3 -u bench.py --workload tcp1500 --no-cpu --no-secondary --no-e2e --steps 100 > $O/tcp_a${a}_$i.json 2> $O/tcp_a${a}_$i.err || exit $?
  done
  for gb in 0 1; do
    for a in 18 2; do
      GCL_TUNE_GBUF=$gb GCL_TUNE_LDAUX=$a timeout -k 10 300 python3 -u tools/ingress_run.py 10 > $O/ing_g${gb}_a${a}_$i.json 2> $O/ing_g${gb}_a${a}_$i.err || exit $?
    done
  done
done
echo rc=0
