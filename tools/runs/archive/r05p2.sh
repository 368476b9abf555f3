# round 5 (the form measured here was removed after it lost): the delayed
# first poll's second sample (GCL_TUNE_LOOP_PHASE2,
# ticks behind the first; 0 = off, the default) with the delay's steps
# (GCL_TUNE_LOOP_PHASE): 1 x 1 header records back to back, at a random
# phase and sparse (NIC), back to back (JENKINS); the loop's GPU tests with
# PHASE2=30 first; forms interleaved in fresh processes, three rounds
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_LOOP_PHASE2=30 timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05p2_rxloop_tests.log 2>&1 || { tail -30 gpurun_out/r05p2_rxloop_tests.log; exit 1; }
tail -1 gpurun_out/r05p2_rxloop_tests.log
out=gpurun_out/r05p2_phase2_ab.jsonl
: > $out
for rnd in 1 2 3; do
  for f in "120,16,1 0" "120,16,1 30" "120,4,2 30" "120,2,2 30" "120,4,2 50"; do
    set -- $f
    ph=$1; p2=$2
    for a in "0 nic" "rand nic" "rand:20000 nic" "0 jenkins"; do
      set -- $a
      nb=20000; [ "$1" = rand:20000 ] && nb=6000
      r=$(GCL_TUNE_LOOP_PHASE=$ph GCL_TUNE_LOOP_PHASE2=$p2 RXPIPE_HASH=$2 RXPIPE_GAP_NS=$1 timeout -k 10 90 tools/rxpipe 64 1 1 $nb records) || { echo "FAIL $ph $p2 $a"; exit 1; }
      echo "{\"round\": $rnd, \"phase\": \"$ph\", \"phase2\": $p2, \"row\": $r}" >> $out
    done
  done
  echo "round $rnd done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05p2_phase2_ab.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["hash"][:5], w["gap_ns"], r["phase"], r["phase2"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"]))
for k in sorted(d, key=str):
    print(k, d[k])
PY
