# the loop suite after moving rxloop64's offsets-path side loads behind the
# offset's use (one round trip, not two, for bursts with ol_flags / hash.rss
# arrays); back-to-back lone bursts without stage stamps (the bench's own
# rows): the poller storing the verdict records against the writer wave, NIC
# hash, records and offsets, interleaved three times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zf_tests.log 2>&1 || { tail -30 gpurun_out/r04zf_tests.log; exit 1; }
tail -2 gpurun_out/r04zf_tests.log
out=gpurun_out/r04zf_writer.jsonl
for rep in 1 2 3; do
  for w in 0 1; do
    for cfg in "64 1 1 20000 records" "64 4 8 20000 records" "64 1 1 20000" "64 4 8 20000"; do
      RXPIPE_HASH=nic GCL_TUNE_LOOP_WRITER=$w timeout -k 10 60 tools/rxpipe $cfg | sed "s/^{/{\"writer\": $w, /" >> $out || exit 1
    done
  done
done
cut -c1-200 $out
