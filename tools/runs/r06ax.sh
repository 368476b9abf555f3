# round 6, the final tree (wide slots on 2 x 256 at depth 1, the pair kernel on
# 2 x 256): the whole GPU suite,
# smoke and the driver's bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ax_gputests.log 2>&1 || { tail -30 gpurun_out/r06ax_gputests.log; exit 1; }
tail -1 gpurun_out/r06ax_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06ax_smoke.log 2>&1 || { tail -5 gpurun_out/r06ax_smoke.log; exit 1; }
tail -1 gpurun_out/r06ax_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r06ax_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06ax_bench.json 2> gpurun_out/r06ax_bench.err || { tail -5 gpurun_out/r06ax_bench.err; exit 1; }
wc -c gpurun_out/r06ax_bench.json
echo r06ax-done
