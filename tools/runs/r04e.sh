set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -q -k "access_probe or top_of_u64" --timeout 60 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 || { tail -20 gpurun_out/r04e_tests.log; exit 1; }
bash tools/runs/r04c.sh r04e || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { tail -5 gpurun_out/r04e_bench.err; exit 1; }
