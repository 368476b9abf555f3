# Settle length: the driver's command (--steps 20 --warmup 5) with 30 ms
# (current) vs 300 ms of untimed continuous steps before the timed ones,
# fresh processes alternating; kernel-only lines.
set -o pipefail
O=gpurun_out/r02bg; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for ms in 30 300; do
    GCL_BENCH_SETTLE_MS=$ms timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --no-e2e > $O/s${ms}_$i.json 2> $O/s${ms}_$i.err || exit $?
  done
done
echo rc=0
