# round 5: the lone burst's stages with the poll-phase delay (stage stamps, header
# records, NIC and JENKINS hash, back to back and random phase)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05zs_stages.jsonl
: > $out
for h in nic jenkins; do
  for gap in 0 rand; do
    RXPIPE_STAMPS=1 RXPIPE_HASH=$h RXPIPE_GAP_NS=$gap timeout -k 10 60 tools/rxpipe 64 1 1 20000 records > gpurun_out/r05zs_tmp.txt || { cat gpurun_out/r05zs_tmp.txt; exit 1; }
    sed "s/^{/{\"hash\": \"$h\", \"gap\": \"$gap\", /" gpurun_out/r05zs_tmp.txt >> $out
  done
done
cat $out
