# rx loop submit refactor (records / arrays share the publish): the loop tests and a few pipeline rows
set -o pipefail
O=gpurun_out/r03zm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rxloop_tests.log 2>&1 || { tail -40 $O/rxloop_tests.log; exit 1; }
tail -3 $O/rxloop_tests.log
for a in "64 1 1 20000" "64 1 1 20000 records" "64 8 16 40000" "64 8 16 40000 records" "64 32 64 60000" "64 16 32 40000 inline"; do
  timeout -k 10 120 ./tools/rxpipe $a >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
cat $O/rxpipe.jsonl
