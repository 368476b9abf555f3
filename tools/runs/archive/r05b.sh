# round 5, after pruning the experiment knobs: the GPU suite, smoke, the
# headline kernels under rocprofv3 (kernel times unchanged?), and the first
# A/B of the two-poller burst-64 loop (GCL_TUNE_LOOP_POLLERS 1 vs 2, rxpipe
# rows interleaved in fresh processes, back-to-back and random phase)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_gputests.log 2>&1 || { tail -30 gpurun_out/r05b_gputests.log; exit 1; }
tail -2 gpurun_out/r05b_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1 || { cat gpurun_out/r05b_smoke.log; exit 1; }
cat gpurun_out/r05b_smoke.log
out=gpurun_out/r05b_pollers_ab.jsonl
: > $out
for rnd in 1 2; do
  for np in 1 2; do
    for a in "nic 64 1 1 20000 records" "nic 64 4 8 20000 records" "jenkins 64 1 1 20000 records" "jenkins 64 4 8 20000 records" "jenkins 64 8 16 40000 records" "jenkins 64 1 1 20000" "jenkins 64 4 8 20000"; do
      set -- $a
      h=$1; shift
      for gap in 0 rand; do
        r=$(GCL_TUNE_LOOP_POLLERS=$np RXPIPE_HASH=$h RXPIPE_GAP_NS=$gap timeout -k 10 60 tools/rxpipe "$@") || { echo "FAIL np=$np $a gap=$gap"; exit 1; }
        echo "{\"round\": $rnd, \"pollers\": $np, \"gap\": \"$gap\", \"row\": $r}" >> $out
        [ "$2" = 1 ] || break
      done
    done
  done
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/r05b_pollers_ab.jsonl')]
for r in rows:
    x=r['row']
    print(r['round'], r['pollers'], r['gap'], x['hash'][:7], x['burst'], x['workers'], x['depth'], x['verdicts'][-20:], x['mpps_one_core'], x['burst_latency_p50_us'], x.get('bursts_early'), x.get('bursts_stale'), x.get('bursts_late'))
PY
