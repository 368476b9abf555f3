set -o pipefail
mkdir -p gpurun_out
for mode in records offsets; do
  for b in 64 1; do
    RXPIPE_STAMPS=1 timeout -k 10 60 tools/rxpipe $b 1 1 20000 $( [ $mode = records ] && echo records ) >> gpurun_out/r04_stages.jsonl || exit 1
  done
done
timeout -k 10 400 python bench.py > gpurun_out/r04_bench_a.json 2> gpurun_out/r04_bench_a.err || { tail -5 gpurun_out/r04_bench_a.err; exit 1; }
cat gpurun_out/r04_stages.jsonl
