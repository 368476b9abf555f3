# round 6: the records submit's header prefetch distance (gcl_tune.rec_prefetch
# via GCL_TUNE_REC_PREFETCH) on cold headers (RXPIPE_POOL=ingress) and hot,
# interleaved, three rounds of fresh processes; then the loop suite and the
# tune-validation test with the new field
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r06g_recpf.jsonl
: > $out
for i in 1 2 3; do
  for pf in 2 16 32 64; do
    for cfg in "1 1 20000" "4 8 20000" "8 16 40000"; do
      GCL_TUNE_REC_PREFETCH=$pf RXPIPE_POOL=ingress RXPIPE_HASH=nic timeout -k 10 120 tools/rxpipe 64 $cfg records > gpurun_out/r06g_one.json 2>&1 || { cat gpurun_out/r06g_one.json; exit 1; }
      python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d["rec_prefetch"]=int(sys.argv[2]); d["round"]=int(sys.argv[3]); d["pool_kind"]="ingress"; print(json.dumps(d))' gpurun_out/r06g_one.json $pf $i >> $out
    done
    RXPIPE_HASH=nic GCL_TUNE_REC_PREFETCH=$pf timeout -k 10 120 tools/rxpipe 64 1 1 20000 records > gpurun_out/r06g_one.json 2>&1 || { cat gpurun_out/r06g_one.json; exit 1; }
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d["rec_prefetch"]=int(sys.argv[2]); d["round"]=int(sys.argv[3]); d["pool_kind"]="hot"; print(json.dumps(d))' gpurun_out/r06g_one.json $pf $i >> $out
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r06g_recpf.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["pool_kind"], r["workers"], r["depth"], r["rec_prefetch"])].append((r["mpps_one_core"], r["burst_latency_p50_us"], r["submit_ns_per_pkt"]))
for k in sorted(agg):
    print(k, agg[k])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "fuzz_vs_oracle or ctx_tune" > gpurun_out/r06g_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06g_tests.log
echo r06g-done rc=$rc
