# round 5 (r05d found no box; this is it plus the dense A/B): rxloop64 with the word loaded first (r05c: records read a round
# trip before the word, nearly every lone burst stale) and NP 2's spec window
# from the last post: loop tests, then the pollers A/B (GCL_TUNE_LOOP_POLLERS
# 1 vs 2, rxpipe rows interleaved in fresh processes, back-to-back and
# random phase)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_looptests.log 2>&1 || { tail -30 gpurun_out/r05e_looptests.log; exit 1; }
tail -2 gpurun_out/r05e_looptests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense" > gpurun_out/r05e_densetests.log 2>&1 || { tail -30 gpurun_out/r05e_densetests.log; exit 1; }
tail -2 gpurun_out/r05e_densetests.log
timeout -k 10 600 python tools/dense_ab.py > gpurun_out/r05e_dense_ab.jsonl 2> gpurun_out/r05e_dense_ab.err || { tail -5 gpurun_out/r05e_dense_ab.err; exit 1; }
cat gpurun_out/r05e_dense_ab.jsonl
out=gpurun_out/r05e_pollers_ab.jsonl
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
