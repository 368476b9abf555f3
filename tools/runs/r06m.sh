# round 6: gcl_tune.slot_prefetch (the next slot's lines taken for writing
# while a lone burst is awaited) 0 / 1, six interleaved rounds of fresh
# processes: hot lone burst NIC and JENKINS, 2 x 2, cold lone burst; then the
# loop suite
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r06m_slotpf.jsonl
: > $out
for i in 1 2 3 4 5 6; do
  for pf in 0 1; do
    for kind in hot_nic hot_jenkins hot_2x2 cold_nic; do
      case $kind in
        hot_nic) env="RXPIPE_HASH=nic"; cfg="1 1 20000";;
        hot_jenkins) env="RXPIPE_HASH=jenkins"; cfg="1 1 20000";;
        hot_2x2) env="RXPIPE_HASH=nic"; cfg="2 2 20000";;
        cold_nic) env="RXPIPE_HASH=nic RXPIPE_POOL=ingress"; cfg="1 1 20000";;
      esac
      env $env GCL_TUNE_SLOT_PREFETCH=$pf timeout -k 10 120 tools/rxpipe 64 $cfg records > gpurun_out/r06m_one.json 2>&1 || { cat gpurun_out/r06m_one.json; exit 1; }
      python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d["slot_prefetch"]=int(sys.argv[2]); d["round"]=int(sys.argv[3]); d["kind"]=sys.argv[4]; print(json.dumps(d))' gpurun_out/r06m_one.json $pf $i $kind >> $out
    done
  done
done
python - <<'PY'
import json, collections, statistics as st
rows = [json.loads(l) for l in open("gpurun_out/r06m_slotpf.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["kind"], r["slot_prefetch"])].append(r)
for k in sorted(agg):
    v = agg[k]
    print(k, "p50 med", st.median(x["burst_latency_p50_us"] for x in v), "p99 med", st.median(x["burst_latency_p99_us"] for x in v),
          "mpps med", st.median(x["mpps_one_core"] for x in v), "submit med", st.median(x["submit_ns_per_pkt"] for x in v),
          "deliver med", st.median(x["deliver_ns_per_pkt"] for x in v))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r06m_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06m_tests.log
echo r06m-done rc=$rc
