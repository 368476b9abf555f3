# Dense tiles as buffer loads (default sc1 nt = 18; 2 = nt; -1 = the former
# global_load nt): GPU tests on the new default, then udp64 and tcp1500
# kernel-only lines, fresh processes alternating.
set -o pipefail
O=gpurun_out/r02bi; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do
  for a in 18 2 -1; do
    GCL_TUNE_LDAUX=$a timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 100 > $O/udp_a${a}_$i.json 2> $O/udp_a${a}_$i.err || exit $?
    GCL_TUNE_LDAUX=$a timeout -k 10 300 python3 -u bench.py --workload tcp1500 --no-cpu --no-secondary --no-e2e --steps 100 > $O/tcp_a${a}_$i.json 2> $O/tcp_a${a}_$i.err || exit $?
  done
done
echo rc=0
