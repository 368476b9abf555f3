#!/bin/bash
# rocprofv3 passes for bench.py: kernel trace + stats, then one PMC pass per
# counter group (never combined with tracing domains).
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_r01}
ARGS=${ARGS:---steps 20 --warmup 3 --no-cpu}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_write.json 2> $OUT/bench_write.err
echo done
