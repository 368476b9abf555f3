# round 5: the poll-phase delay's ceiling and steps around r05y's best
# (120,8,1): back to back, random phase [0, 2) us, sparse [0, 20) us and two
# workers x 2 in flight, NIC hash and header records; forms interleaved in
# fresh processes, three rounds (the loop's tests as in r05y first)
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_LOOP_PHASE=120,32,1 timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05z_rxloop_tests.log 2>&1 || { tail -30 gpurun_out/r05z_rxloop_tests.log; exit 1; }
tail -1 gpurun_out/r05z_rxloop_tests.log
out=gpurun_out/r05z_phase_ab.jsonl
: > $out
for rnd in 1 2 3; do
  for ph in 0 120,8,1 100,8,1 80,8,1 150,8,1 120,16,1 120,32,1; do
    for a in "1 1 20000 0 nic" "1 1 20000 rand nic" "1 1 6000 rand:20000 nic" "2 2 20000 0 nic"; do
      set -- $a
      r=$(GCL_TUNE_LOOP_PHASE=$ph RXPIPE_HASH=$5 RXPIPE_GAP_NS=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 records) || { echo "FAIL phase=$ph $a"; exit 1; }
      echo "{\"round\": $rnd, \"phase\": \"$ph\", \"row\": $r}" >> $out
    done
  done
  echo "round $rnd done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05z_phase_ab.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["workers"], w["gap_ns"], r["phase"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"], w.get("bursts_early"), w.get("bursts_stale"), w.get("bursts_late")))
for k in sorted(d, key=str):
    print(k, d[k])
PY
