# round 5: the loop's speculative window 1 ms for 1-2 workers by default:
# the loop suite, then rxpipe rows without any knob (sparse lone bursts,
# back to back, 4 x 8, 8 x 16)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05w_looptests.log 2>&1 || { tail -30 gpurun_out/r05w_looptests.log; exit 1; }
tail -1 gpurun_out/r05w_looptests.log
out=gpurun_out/r05w_rows.jsonl
: > $out
for a in "1 1 20000 0" "1 1 20000 rand" "1 1 5000 rand:20000" "4 8 20000 0" "8 16 40000 0"; do
  set -- $a
  r=$(RXPIPE_HASH=nic RXPIPE_GAP_NS=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 records) || { echo "FAIL $a"; exit 1; }
  echo "$r" >> $out
done
python3 -c "
import json
for l in open('gpurun_out/r05w_rows.jsonl'):
    w=json.loads(l); print(w['workers'], w['depth'], w['gap_ns'], w['mpps_one_core'], w['burst_latency_p50_us'], w['burst_latency_p99_us'], w['bursts_late'])
"
