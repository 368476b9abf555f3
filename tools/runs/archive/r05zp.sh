# round 5: the poll-phase delay forced on for the pipelined rows (4 x 8 and
# 8 x 16, GCL_TUNE_LOOP_PHASE=120,16,1) against the default (off above 2
# workers); fresh processes, three rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05zp_phase_pipe.jsonl
: > $out
for rnd in 1 2 3; do
  for ph in default 120,16,1; do
    for a in "4 8 20000 nic records" "4 8 20000 jenkins records" "8 16 40000 nic records" "4 8 20000 jenkins offs"; do
      set -- $a
      m=$5; [ "$m" = offs ] && m=""
      if [ "$ph" = default ]; then
        r=$(RXPIPE_HASH=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 $m) || { echo "FAIL $ph $a"; exit 1; }
      else
        r=$(GCL_TUNE_LOOP_PHASE=$ph RXPIPE_HASH=$4 timeout -k 10 90 tools/rxpipe 64 $1 $2 $3 $m) || { echo "FAIL $ph $a"; exit 1; }
      fi
      echo "{\"round\": $rnd, \"phase\": \"$ph\", \"row\": $r}" >> $out
    done
  done
  echo "round $rnd done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05zp_phase_pipe.jsonl"):
    r = json.loads(l); w = r["row"]
    d[(w["workers"], w["depth"], w["hash"][:5], w["verdicts"][-12:], r["phase"])].append((w["mpps_one_core"], w["burst_latency_p50_us"], w["burst_latency_p99_us"]))
for k in sorted(d, key=str):
    print(k, d[k])
PY
