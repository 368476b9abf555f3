# the lone 64-packet burst (header records, NIC hash) against the phase of
# its submit: back to back, fixed gaps between delivery and the next
# submit, and a uniformly random gap (bursts arriving at any phase of the
# worker's polls, as from a NIC); two passes
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04zh_phase.jsonl
for rep in 1 2; do
  for gap in 0 200 400 600 800 1000 1200 1400 rand; do
    RXPIPE_HASH=nic RXPIPE_GAP_NS=$gap timeout -k 10 60 tools/rxpipe 64 1 1 20000 records >> $out || exit 1
  done
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print(d['gap_ns'], d['burst_latency_p50_us'], d['burst_latency_p99_us'], d['wait_ns_per_pkt'])
"
