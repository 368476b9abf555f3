# final round-3 tree: loop tests, pipeline rows, the whole GPU suite, smoke, default bench
# smoke, the driver's default bench command, and the burst-64 pipeline rows
set -o pipefail
O=gpurun_out/r03zs
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rxloop_tests.log 2>&1 || { tail -40 $O/rxloop_tests.log; exit 1; }
tail -3 $O/rxloop_tests.log
for a in "64 1 1 20000" "64 1 1 20000 inline" "64 1 1 20000 records" "64 4 8 20000" "64 4 8 20000 records" "64 16 32 40000" "64 16 32 40000 inline" "64 16 32 40000 records"; do
  timeout -k 10 120 ./tools/rxpipe $a >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
cat $O/rxpipe.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['e2e']['rxloop']))"
