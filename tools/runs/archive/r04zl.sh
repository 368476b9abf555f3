# hybrid polling (GCL_TUNE_LOOP_HYBRID: a caught-up worker's first poll some
# ticks after its last records): loop tests with it on, then the lone burst
# back to back and at a random phase, and the shallow rows, NIC hash
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_LOOP_HYBRID=50 timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread -k "fuzz_vs_oracle or lean or ragged or soak or stamp_wrap or pipelined" > gpurun_out/r04zl_tests.log 2>&1 || { tail -30 gpurun_out/r04zl_tests.log; exit 1; }
tail -2 gpurun_out/r04zl_tests.log
out=gpurun_out/r04zl_hybrid.jsonl
for rep in 1 2; do
  for hy in 0 30 50 70 90; do
    for gap in 0 rand; do
      RXPIPE_HASH=nic RXPIPE_GAP_NS=$gap GCL_TUNE_LOOP_HYBRID=$hy timeout -k 10 60 tools/rxpipe 64 1 1 20000 records | sed "s/^{/{\"hybrid\": $hy, /" >> $out || exit 1
    done
    for cfg in "64 4 8 20000 records" "64 8 16 40000 records" "64 16 32 40000"; do
      RXPIPE_HASH=nic GCL_TUNE_LOOP_HYBRID=$hy timeout -k 10 60 tools/rxpipe $cfg | sed "s/^{/{\"hybrid\": $hy, /" >> $out || exit 1
    done
  done
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print(d['hybrid'], d['workers'], d['depth'], d['gap_ns'], 'rec' if 'records' in d['verdicts'] else 'off', d['mpps_one_core'], d['burst_latency_p50_us'], d['burst_latency_p99_us'])
"
