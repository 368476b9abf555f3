# round 5: the poll-phase delay after its fix for loops without the
# speculative window (a first-poll find counts as on time unless stale): the
# loop's GPU tests, then 1 x 1 rows with the delay off and on -- header
# records back to back and at a random phase, inline headers and stamped
# offsets back to back -- fresh processes, three rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ph_rxloop_tests.log 2>&1 || { tail -30 gpurun_out/r05ph_rxloop_tests.log; exit 1; }
tail -1 gpurun_out/r05ph_rxloop_tests.log
out=gpurun_out/r05ph_phase_fix.jsonl
: > $out
for rnd in 1 2 3; do
  for ph in 0 120,16,1; do
    for a in "0 records" "rand records" "0 inline" "0 offs"; do
      set -- $a
      m=$2; [ "$m" = offs ] && m=""
      r=$(GCL_TUNE_LOOP_PHASE=$ph RXPIPE_HASH=nic RXPIPE_GAP_NS=$1 timeout -k 10 90 tools/rxpipe 64 1 1 20000 $m) || { echo "FAIL phase=$ph $a"; exit 1; }
      echo "{\"round\": $rnd, \"phase\": \"$ph\", \"row\": $r}" >> $out
    done
  done
  echo "round $rnd done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05ph_phase_fix.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["verdicts"][-16:], w["gap_ns"], r["phase"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"], w.get("bursts_early"), w.get("bursts_stale"), w.get("bursts_late")))
for k in sorted(d, key=str):
    print(k, d[k])
PY
