# two polls in flight (GCL_TUNE_LOOP_DUAL: the second poll 68 ticks = 0.68
# us after the first) against one: loop tests with the knob on, then the lone
# burst at random and fixed phases and the shallow rows, NIC hash, records
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_LOOP_DUAL=68 timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread -k "fuzz_vs_oracle or lean or ragged or soak or stamp_wrap" > gpurun_out/r04zi_tests.log 2>&1 || { tail -30 gpurun_out/r04zi_tests.log; exit 1; }
tail -2 gpurun_out/r04zi_tests.log
out=gpurun_out/r04zi_dual.jsonl
for rep in 1 2; do
  for d in 0 68; do
    for gap in rand 0 600; do
      RXPIPE_HASH=nic RXPIPE_GAP_NS=$gap GCL_TUNE_LOOP_DUAL=$d timeout -k 10 60 tools/rxpipe 64 1 1 20000 records | sed "s/^{/{\"dual\": $d, /" >> $out || exit 1
    done
    for cfg in "64 4 8 20000 records" "64 8 16 40000 records" "64 16 32 40000"; do
      RXPIPE_HASH=nic GCL_TUNE_LOOP_DUAL=$d timeout -k 10 60 tools/rxpipe $cfg | sed "s/^{/{\"dual\": $d, /" >> $out || exit 1
    done
  done
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print(d['dual'], d['workers'], d['depth'], d['gap_ns'], 'rec' if 'records' in d['verdicts'] else 'off', d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['bursts_stale'])
"
