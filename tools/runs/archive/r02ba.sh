# Experiment: consecutive udp64 steps alternating two streams (kernel tails
# overlap the next step's head) vs one stream; wall-clock value, fresh
# processes alternating.
set -o pipefail
O=gpurun_out/r02ba; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for sN in 1 2; do
    GCL_BENCH_STREAMS=$sN timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 100 > $O/s${sN}_$i.json 2> $O/s${sN}_$i.err || exit $?
  done
done
echo rc=0
