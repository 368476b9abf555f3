# 8-B verdict records (GCL_LOOP_REC8): the loop tests, then rxpipe plain vs rec8 (and records vs
# records+rec8) at burst 64, alternating rounds
set -o pipefail
O=gpurun_out/r03zi
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rxloop_tests.log 2>&1 || { tail -40 $O/rxloop_tests.log; exit 1; }
tail -3 $O/rxloop_tests.log
for rnd in 1 2 3; do
  for a in "1 1" "4 8" "8 16" "16 32" "32 64"; do
    for m in plain rec8 records records+rec8; do
      timeout -k 10 120 ./tools/rxpipe 64 $a 30000 $( [ $m = plain ] || echo $m ) | sed "s/^{/{\"mode\": \"$m\", \"round\": $rnd, /" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r03zi/ab.jsonl'):
    d=json.loads(l); print(d['round'], d['mode'], d['workers'], d['depth'], d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['submit_ns_per_pkt'], d['deliver_ns_per_pkt'], d['wait_ns_per_pkt'])
PY
