# round 5: the poll-phase delay's update moved after the records' store and
# the context flags kept in registers (no kernel-argument reloads between a
# hit and the record store): the loop's GPU tests, the lone burst's stage
# stamps, then 1 x 1 rows (records NIC / JENKINS back to back, NIC random
# phase, stamped offsets NIC) in fresh processes, three rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05zt_rxloop_tests.log 2>&1 || { tail -30 gpurun_out/r05zt_rxloop_tests.log; exit 1; }
tail -1 gpurun_out/r05zt_rxloop_tests.log
out=gpurun_out/r05zt_stages.jsonl
: > $out
for h in nic jenkins; do
  for gap in 0 rand; do
    RXPIPE_STAMPS=1 RXPIPE_HASH=$h RXPIPE_GAP_NS=$gap timeout -k 10 60 tools/rxpipe 64 1 1 20000 records > gpurun_out/r05zt_tmp.txt || { cat gpurun_out/r05zt_tmp.txt; exit 1; }
    sed "s/^{/{\"hash\": \"$h\", \"gap\": \"$gap\", /" gpurun_out/r05zt_tmp.txt >> $out
  done
done
grep lone_burst $out
out=gpurun_out/r05zt_rows.jsonl
: > $out
for rnd in 1 2 3; do
  for a in "0 nic records" "0 jenkins records" "rand nic records" "0 nic offs"; do
    set -- $a
    m=$3; [ "$m" = offs ] && m=""
    r=$(RXPIPE_HASH=$2 RXPIPE_GAP_NS=$1 timeout -k 10 90 tools/rxpipe 64 1 1 20000 $m) || { echo "FAIL $a"; exit 1; }
    echo "{\"round\": $rnd, \"row\": $r}" >> $out
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05zt_rows.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["hash"][:5], w["gap_ns"], w["verdicts"][-12:])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"]))
for k in sorted(d, key=str):
    print(k, d[k])
PY
