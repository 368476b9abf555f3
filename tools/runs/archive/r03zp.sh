# soak of the header records (GCL_LOOP_HDR_RECORDS): random 1..64-packet bursts racing the
# workers' polls, every verdict against the batch kernel (tools/loopsoak ... records)
set -o pipefail
O=gpurun_out/r03zp
mkdir -p $O
for cfg in "3000000 1 2 1" "10000000 4 4 4" "10000000 3 8 8" "10000000 16 16 16" "10000000 32 64 64" "10000000 64 64 64"; do
  timeout -k 10 170 ./tools/loopsoak $cfg records >> $O/soak.jsonl 2>> $O/soak.err || { cat $O/soak.err; tail -2 $O/soak.jsonl; exit 1; }
  tail -1 $O/soak.jsonl
done
