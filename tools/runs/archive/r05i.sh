# round 5, the final tree: the whole GPU suite, smoke, the driver's bench
# command, then rocprofv3 (kernel trace/stats + PMC passes) of the two
# dominant launches (udp64 1-B, tcp1500 2-B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i_gputests.log 2>&1 || { tail -30 gpurun_out/r05i_gputests.log; exit 1; }
tail -2 gpurun_out/r05i_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05i_smoke.log 2>&1 || { tail -5 gpurun_out/r05i_smoke.log; exit 1; }
tail -1 gpurun_out/r05i_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r05i_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r05i_bench.json 2> gpurun_out/r05i_bench.err || { tail -5 gpurun_out/r05i_bench.err; exit 1; }
wc -c gpurun_out/r05i_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r05 WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r05i_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r05i_prof_udp64.log; exit 1; }
ROUND=r05 WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r05i_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r05i_prof_tcp1500.log; exit 1; }
echo r05i-done
