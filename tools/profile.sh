#!/bin/bash
# rocprofv3 evidence for one round: per workload a kernel-trace/stats pass and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE), plus membench calibration
# dispatches of known byte counts.  Never mixes --pmc with tracing domains.
set -e
export TMPDIR=/tmp
R=${ROUND:-r01}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
for wl in ${WLS:-udp64 tcp1500}; do
  A="--workload $wl --steps 20 --warmup 3 --no-cpu --no-secondary --no-e2e"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${wl}_trace -o run -- python3 bench.py $A > $OUT/${wl}_bench.json 2> $OUT/${wl}_trace.err
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/${wl}_$c -o run -- python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu --no-secondary --no-e2e > /dev/null 2> $OUT/${wl}_$c.err
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/calib_$c -o run -- ./tools/membench calib > $OUT/calib_$c.jsonl 2> $OUT/calib_$c.err
done
echo profile-done
