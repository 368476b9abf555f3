# round 6, after the wait-time ring prefetch and the ordered clock in rxpipe: the whole GPU
# suite, smoke and the driver's bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06p_gputests.log 2>&1 || { tail -30 gpurun_out/r06p_gputests.log; exit 1; }
tail -1 gpurun_out/r06p_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06p_smoke.log 2>&1 || { tail -5 gpurun_out/r06p_smoke.log; exit 1; }
tail -1 gpurun_out/r06p_smoke.log
GCL_BENCH_DETAIL=gpurun_out/r06p_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r06p_bench.json 2> gpurun_out/r06p_bench.err || { tail -5 gpurun_out/r06p_bench.err; exit 1; }
wc -c gpurun_out/r06p_bench.json
