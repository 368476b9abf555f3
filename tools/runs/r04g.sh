set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/clock_probe > gpurun_out/r04g_clock.jsonl || exit 1
cat gpurun_out/r04g_clock.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "copy_transport or ingress_pool or end_to_end or access_probe or top_of_u64" --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 || { tail -20 gpurun_out/r04g_tests.log; exit 1; }
tail -2 gpurun_out/r04g_tests.log
bash tools/runs/r04c.sh r04g > /dev/null || exit 1
grep lone gpurun_out/r04g_stages.jsonl
timeout -k 10 400 python bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || { tail -5 gpurun_out/r04g_bench.err; exit 1; }
