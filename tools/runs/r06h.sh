# round 6: rec_prefetch 2 / 16 / 64 once more, six interleaved rounds of fresh
# processes: hot-header lone burst (the bench's records_1x1_nic row) and cold
# headers 1 x 1 and 4 x 8
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r06h_recpf.jsonl
: > $out
for i in 1 2 3 4 5 6; do
  for pf in 2 16 64; do
    for kind in hot ingress4 ingress1; do
      case $kind in
        hot) env="RXPIPE_HASH=nic"; cfg="1 1 20000";;
        ingress4) env="RXPIPE_HASH=nic RXPIPE_POOL=ingress"; cfg="4 8 20000";;
        ingress1) env="RXPIPE_HASH=nic RXPIPE_POOL=ingress"; cfg="1 1 20000";;
      esac
      env $env GCL_TUNE_REC_PREFETCH=$pf timeout -k 10 120 tools/rxpipe 64 $cfg records > gpurun_out/r06h_one.json 2>&1 || { cat gpurun_out/r06h_one.json; exit 1; }
      python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d["rec_prefetch"]=int(sys.argv[2]); d["round"]=int(sys.argv[3]); d["pool_kind"]=sys.argv[4]; print(json.dumps(d))' gpurun_out/r06h_one.json $pf $i $kind >> $out
    done
  done
done
python - <<'PY'
import json, collections, statistics as st
rows = [json.loads(l) for l in open("gpurun_out/r06h_recpf.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["pool_kind"], r["rec_prefetch"])].append((r["mpps_one_core"], r["burst_latency_p50_us"], r["submit_ns_per_pkt"]))
for k in sorted(agg):
    v = agg[k]
    print(k, "mpps med", st.median(x[0] for x in v), "p50 med", st.median(x[1] for x in v), "submit med", st.median(x[2] for x in v))
PY
echo r06h-done
