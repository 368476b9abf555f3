# 1-byte verdict stores (timing only, GCL_TUNE_ABLATE 1024) against the
# 2-byte queue verdict, udp64 and tcp1500, same buffers, interleaved rounds
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 120 tools/cbench 0 50 0:0:0:0:0:0:2 1024:0:0:0:0:0:2 >> gpurun_out/r04x_v1_udp64.jsonl || exit 1
done
timeout -k 10 120 tools/cbench 1 50 0:0:0:0:0:0:2 1024:0:0:0:0:0:2 >> gpurun_out/r04x_v1_tcp1500.jsonl || exit 1
cat gpurun_out/r04x_v1_udp64.jsonl gpurun_out/r04x_v1_tcp1500.jsonl
