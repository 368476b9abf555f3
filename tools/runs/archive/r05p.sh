# round 5, the final tree: the driver's bench command once more (pair kernel
# lean waves, CPU baseline through one loop with the 1-core cells first)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deferred_flushes" > gpurun_out/r05p_flush.log 2>&1 || { tail -30 gpurun_out/r05p_flush.log; exit 1; }
tail -1 gpurun_out/r05p_flush.log
GCL_BENCH_DETAIL=gpurun_out/r05p_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r05p_bench.json 2> gpurun_out/r05p_bench.err || { tail -5 gpurun_out/r05p_bench.err; exit 1; }
wc -c gpurun_out/r05p_bench.json
