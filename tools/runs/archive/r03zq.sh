# poll-outcome counters (gcl_rxloop_poll_stats): loop tests, then the stamped-offset and
# header-record soaks with their early / stale / late burst counts
set -o pipefail
O=gpurun_out/r03zq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rxloop_tests.log 2>&1 || { tail -40 $O/rxloop_tests.log; exit 1; }
tail -3 $O/rxloop_tests.log
for m in "" records; do
  for cfg in "3000000 1 2 1" "10000000 4 4 4" "10000000 16 16 16" "10000000 64 64 64"; do
    timeout -k 10 170 ./tools/loopsoak $cfg $m >> $O/soak.jsonl 2>> $O/soak.err || { cat $O/soak.err; tail -2 $O/soak.jsonl; exit 1; }
    tail -1 $O/soak.jsonl
  done
done
for a in "64 1 1 20000" "64 1 1 20000 records" "64 16 32 40000" "64 16 32 40000 records"; do
  timeout -k 10 120 ./tools/rxpipe $a >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
cat $O/rxpipe.jsonl
