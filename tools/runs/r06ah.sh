# round 6, the final tree (plain pools for the deferring contexts): the whole
# GPU suite, smoke, the driver's bench command and the rocprofv3 passes of
# udp64, tcp1500 and the ingress shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ah_gputests.log 2>&1 || { tail -30 gpurun_out/r06ah_gputests.log; exit 1; }
tail -1 gpurun_out/r06ah_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06ah_smoke.log 2>&1 || { tail -5 gpurun_out/r06ah_smoke.log; exit 1; }
tail -1 gpurun_out/r06ah_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r06ah_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06ah_bench.json 2> gpurun_out/r06ah_bench.err || { tail -5 gpurun_out/r06ah_bench.err; exit 1; }
wc -c gpurun_out/r06ah_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r06ah WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ah_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r06ah_prof_udp64.log; exit 1; }
ROUND=r06ah WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ah_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r06ah_prof_tcp1500.log; exit 1; }
ROUND=r06ah WLS=ingress_nic VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ah_prof_ingress.log 2>&1 || { tail -5 gpurun_out/r06ah_prof_ingress.log; exit 1; }
echo r06ah-done
