# rxpipe with the dataplane thread pinned near the GPU: repeat the burst-64 rows
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
for rep in 1 2 3; do
for cfg in "64 4 8 20000" "64 8 16 40000" "64 16 32 40000" "64 8 16 40000 inline" "64 16 32 40000 inline"; do
  timeout -k 10 120 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
done
python3 -c "
import json
for l in open('$O/rxpipe.jsonl'):
    d=json.loads(l); print(d['burst'], d['workers'], d['depth'], d['verdicts'][:30], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['host_cpu'])"
timeout -k 10 120 ./tools/grouppipe 1 $((8<<20)) 5 > $O/grouppipe.json 2> $O/grouppipe.err && cat $O/grouppipe.json &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_group.py > $O/test_group.log 2>&1; rc=$?; tail -5 $O/test_group.log; exit $rc
