# round 5: the loop's speculative window (GCL_TUNE_LOOP_SPEC, 10-ns ticks;
# default 400 = 4 us: how long after its last burst a worker polls the
# header records with the word) against sparser lone-burst traffic (random
# gaps of [0, 2) / [0, 5) / [0, 10) us) and the pipelined rows, rows
# interleaved in fresh processes, two rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05u_spec_ab.jsonl
: > $out
for rnd in 1 2; do
  for spec in 400 1000 100000; do
    for a in "1 1 20000 rand" "1 1 10000 rand:5000" "1 1 6000 rand:10000" "1 1 20000 0" "4 8 20000 0" "8 16 40000 0"; do
      set -- $a
      r=$(GCL_TUNE_LOOP_SPEC=$spec RXPIPE_HASH=nic RXPIPE_GAP_NS=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 records) || { echo "FAIL spec=$spec $a"; exit 1; }
      echo "{\"round\": $rnd, \"spec\": $spec, \"row\": $r}" >> $out
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05u_spec_ab.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["workers"], w["depth"], w["gap_ns"], r["spec"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"], w.get("bursts_late")))
for k in sorted(d, key=str):
    print(k, d[k])
PY
