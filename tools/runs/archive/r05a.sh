# round 5, first GPU call: the compact bench line (driver's command) and the
# launcher-less --gpus 2 rehearsal (two gloo ranks sharing the one GPU)
set -o pipefail
mkdir -p gpurun_out
GCL_BENCH_DETAIL=gpurun_out/r05a_bench_detail.json timeout -k 10 600 python bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || { tail -5 gpurun_out/r05a_bench.err; exit 1; }
wc -c gpurun_out/r05a_bench.json
GCL_BENCH_DETAIL=gpurun_out/r05a_gloo2_detail.json timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 20 --warmup 2 > gpurun_out/r05a_gloo2.json 2> gpurun_out/r05a_gloo2.err || { tail -5 gpurun_out/r05a_gloo2.err; exit 1; }
cut -c1-600 gpurun_out/r05a_gloo2.json
