# round 5: rxloop64 with the word loaded first (r05c: records read a round
# trip before the word, nearly every lone burst stale) and NP 2's spec window
# from the last post: loop tests, then the pollers A/B (GCL_TUNE_LOOP_POLLERS
# 1 vs 2, rxpipe rows interleaved in fresh processes, back-to-back and
# random phase)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_looptests.log 2>&1 || { tail -30 gpurun_out/r05d_looptests.log; exit 1; }
tail -2 gpurun_out/r05d_looptests.log
out=gpurun_out/r05d_pollers_ab.jsonl
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
echo ab-done
