# round 5, the final tree: the whole GPU suite, smoke and the driver's bench
# command (the loop's 1-ms window for 1-2 workers; the CPU baseline's
# throwaway first cell)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05x_gputests.log 2>&1 || { tail -30 gpurun_out/r05x_gputests.log; exit 1; }
tail -1 gpurun_out/r05x_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05x_smoke.log 2>&1 || { tail -5 gpurun_out/r05x_smoke.log; exit 1; }
tail -1 gpurun_out/r05x_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r05x_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r05x_bench.json 2> gpurun_out/r05x_bench.err || { tail -5 gpurun_out/r05x_bench.err; exit 1; }
wc -c gpurun_out/r05x_bench.json
