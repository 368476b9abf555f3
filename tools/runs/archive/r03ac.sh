# rx loop A/B: stop flag read beside every 8th poll, offsets polled for the first 4 us of a wait (new) against the previous loop
# (new) against the previous loop (tools/_scratch/rxpipe_old), alternating
set -o pipefail
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rxloop.py > $O/test_rxloop.log 2>&1 || { tail -30 $O/test_rxloop.log; exit 1; }
tail -2 $O/test_rxloop.log
for rep in 1 2 3; do
for cfg in "64 1 1 20000" "64 4 8 20000" "64 8 16 40000" "64 16 32 40000" "64 16 64 40000"; do
  for v in old new; do
    exe=./tools/rxpipe; [ $v = old ] && exe=./tools/_scratch/rxpipe_old
    timeout -k 10 120 $exe $cfg | sed "s/^{/{\"v\": \"$v\", /" >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
  done
done
done
python3 -c "
import json
for l in open('$O/rxpipe.jsonl'):
    d=json.loads(l); print(d['v'], d['burst'], d['workers'], d['depth'], d['verdicts'][-8:], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['delivered_check'])"
timeout -k 10 200 python -u tools/rxloop_run.py 2000 > $O/rxloop.json 2> $O/rxloop.err || { tail $O/rxloop.err; exit 1; }
cat $O/rxloop.json
