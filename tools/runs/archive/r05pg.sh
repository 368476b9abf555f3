# round 5: the loop's next-ticket poll issued before a burst is classified
# (GCL_TUNE_LOOP_PREFETCH, 0/1), now only after a burst found by its first
# poll (the host ahead), on the pipelined rows and, forced, on the
# lone burst; the loop's GPU tests with it forced on for every worker count
# first; forms interleaved in fresh processes, three rounds
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_LOOP_PREFETCH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05pg_rxloop_tests.log 2>&1 || { tail -30 gpurun_out/r05pg_rxloop_tests.log; exit 1; }
tail -1 gpurun_out/r05pg_rxloop_tests.log
out=gpurun_out/r05pg_prefetch_ab.jsonl
: > $out
for rnd in 1 2 3; do
  for pf in 0 1; do
    for a in "4 8 20000 0 nic records" "4 8 20000 0 jenkins records" "8 16 40000 0 nic records" "16 32 40000 0 jenkins records" "4 8 20000 0 jenkins offs" "16 32 40000 0 jenkins offs" "1 1 20000 0 nic records" "8 16 40000 0 jenkins records"; do
      set -- $a
      m=$6; [ "$m" = offs ] && m=""
      r=$(GCL_TUNE_LOOP_PREFETCH=$pf RXPIPE_HASH=$5 RXPIPE_GAP_NS=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 $m) || { echo "FAIL pf=$pf $a"; exit 1; }
      echo "{\"round\": $rnd, \"prefetch\": $pf, \"row\": $r}" >> $out
    done
  done
  echo "round $rnd done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05pg_prefetch_ab.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["workers"], w["depth"], w["hash"][:5], w["verdicts"][-14:], w["gap_ns"], r["prefetch"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"], w.get("bursts_early"), w.get("bursts_stale"), w.get("bursts_late")))
for k in sorted(d, key=str):
    print(k, d[k])
PY
