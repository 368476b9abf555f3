# soak of the rx loop's stamped offsets: random 1..64-packet bursts at random offsets,
# few slots, tight host loop with pauses; every verdict against the batch kernel's
set -o pipefail
O=gpurun_out/r03al
mkdir -p $O
for cfg in "300000 1 2 1" "1000000 4 4 4" "1000000 3 8 8" "1000000 16 16 16" "1000000 32 64 64"; do
  timeout -k 10 240 ./tools/loopsoak $cfg | tee -a $O/soak.jsonl || exit 1
done
