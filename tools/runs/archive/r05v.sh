# round 5: the speculative window, second pass: the default 4 us against an
# effectively unbounded one (1 ms) on sparse lone bursts and on the many-worker
# rows where every idle worker's polls would read its records (4 KiB per poll)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05v_spec_ab.jsonl
: > $out
for rnd in 1 2; do
  for spec in 400 100000; do
    for a in "1 1 5000 rand:20000 records" "2 2 20000 0 records" "4 8 20000 0 records" "8 16 40000 0 records" "16 32 40000 0 records" "16 32 40000 0 offs" "32 64 40000 0 offs"; do
      set -- $a
      f=$5; [ "$f" = offs ] && f=""
      r=$(GCL_TUNE_LOOP_SPEC=$spec RXPIPE_HASH=nic RXPIPE_GAP_NS=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 $f) || { echo "FAIL spec=$spec $a"; exit 1; }
      echo "{\"round\": $rnd, \"spec\": $spec, \"row\": $r}" >> $out
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05v_spec_ab.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["workers"], w["depth"], w["gap_ns"], w["verdicts"][:24], r["spec"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"], w.get("bursts_late")))
for k in sorted(d, key=str):
    print(k, d[k])
PY
