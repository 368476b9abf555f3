#!/bin/bash
# rx_burst replacement on one host core: persistent GPU loop + lrpc post-pass
O=gpurun_out/rxpipe
mkdir -p $O
: > $O/rxpipe.jsonl
for cfg in "64 1 1 20000" "64 4 8 20000" "256 4 8 10000" "1024 8 16 4000" "4096 16 16 1000"; do
  timeout -k 10 60 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || exit 1
done
echo done
