# round 6, the final tree: the whole GPU suite, smoke, the driver's bench
# command, the 2-rank rehearsal of the N>1 line, and the rocprofv3 passes
# (kernel trace + stats, then separate PMC passes) of udp64 1-B, tcp1500 2-B
# and the integrated ingress shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06n_gputests.log 2>&1 || { tail -30 gpurun_out/r06n_gputests.log; exit 1; }
tail -1 gpurun_out/r06n_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06n_smoke.log 2>&1 || { tail -5 gpurun_out/r06n_smoke.log; exit 1; }
tail -1 gpurun_out/r06n_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r06n_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06n_bench.json 2> gpurun_out/r06n_bench.err || { tail -5 gpurun_out/r06n_bench.err; exit 1; }
wc -c gpurun_out/r06n_bench.json
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 10 --warmup 2 --no-e2e --cpu-budget 10 > gpurun_out/r06n_bench_gloo2.json 2> gpurun_out/r06n_bench_gloo2.err || { tail -5 gpurun_out/r06n_bench_gloo2.err; exit 1; }
head -c 300 gpurun_out/r06n_bench_gloo2.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r06n WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06n_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r06n_prof_udp64.log; exit 1; }
ROUND=r06n WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06n_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r06n_prof_tcp1500.log; exit 1; }
ROUND=r06n WLS=ingress_nic VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06n_prof_ingress.log 2>&1 || { tail -5 gpurun_out/r06n_prof_ingress.log; exit 1; }
echo r06n-done
