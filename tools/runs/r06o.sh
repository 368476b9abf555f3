# round 6: gcl_host_prefetch_rxq during a lone wait (RXPIPE_RING_PREFETCH)
# 0 / 1, with rxpipe's clock now rdtscp (ordered), six interleaved rounds of
# fresh processes: hot lone burst NIC and JENKINS, cold lone burst
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r06o_ringpf.jsonl
: > $out
for i in 1 2 3 4 5 6; do
  for pf in 0 1; do
    for kind in hot_nic hot_jenkins cold_nic; do
      case $kind in
        hot_nic) env="RXPIPE_HASH=nic"; cfg="1 1 20000";;
        hot_jenkins) env="RXPIPE_HASH=jenkins"; cfg="1 1 20000";;
        cold_nic) env="RXPIPE_HASH=nic RXPIPE_POOL=ingress"; cfg="1 1 20000";;
      esac
      env $env RXPIPE_RING_PREFETCH=$pf timeout -k 10 120 tools/rxpipe 64 $cfg records > gpurun_out/r06o_one.json 2>&1 || { cat gpurun_out/r06o_one.json; exit 1; }
      python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d["ring_prefetch"]=int(sys.argv[2]); d["round"]=int(sys.argv[3]); d["kind"]=sys.argv[4]; print(json.dumps(d))' gpurun_out/r06o_one.json $pf $i $kind >> $out
    done
  done
done
python - <<'PY'
import json, collections, statistics as st
rows = [json.loads(l) for l in open("gpurun_out/r06o_ringpf.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["kind"], r["ring_prefetch"])].append(r)
for k in sorted(agg):
    v = agg[k]
    print(k, "p50 med", st.median(x["burst_latency_p50_us"] for x in v), "p99 med", st.median(x["burst_latency_p99_us"] for x in v),
          "mpps med", st.median(x["mpps_one_core"] for x in v), "submit med", st.median(x["submit_ns_per_pkt"] for x in v),
          "deliver med", st.median(x["deliver_ns_per_pkt"] for x in v), "wait med", st.median(x["wait_ns_per_pkt"] for x in v))
PY
echo r06o-done
