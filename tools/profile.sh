#!/bin/bash
# rocprofv3 evidence for one round: per workload and verdict size a
# kernel-trace/stats pass and separate PMC passes (FETCH_SIZE, WRITE_SIZE,
# fabric request counts), plus membench calibration dispatches of known byte
# counts.  Never mixes --pmc with tracing domains; every pass has its own
# time limit and the script stops at the first failure.
#   ROUND=r02 WLS="udp64 tcp1500 ingress_nic" VBS="4" bash tools/profile.sh
set -e
export TMPDIR=/tmp
R=${ROUND:-r02}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
run_cmd() { # workload, vbytes, steps -> the program and its arguments
  if [ "$1" = ingress_nic ]; then
    echo "python3 tools/ingress_run.py $3 --nic-only"
  elif [ "$1" = ingress_ws ]; then
    echo "python3 tools/ingress_run.py $3 --ws-only"
  else
    echo "python3 bench.py --workload $1 --verdict-bytes $2 --no-cpu --no-secondary --no-e2e --no-group --steps $3 --warmup ${WARMUP:-100}"
  fi
}
for vb in ${VBS:-2 4 8}; do
for wl in ${WLS:-udp64 tcp1500}; do
  D=$OUT/${wl}_v${vb}
  if [ -z "$REQ_ONLY" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${D}_trace -o run -- $(run_cmd $wl $vb 20) > ${D}_bench.json 2> ${D}_trace.err
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d ${D}_$c -o run -- $(run_cmd $wl $vb 5) > /dev/null 2> ${D}_$c.err
  done
  fi
  # request sizes at the L2/fabric boundary, for the rocprof-compute gfx950
  # HBM formula (128 x TCC_BUBBLE + 32 x RDREQ_32B + 64 x the other reads;
  # 64 x WRREQ_64B + 32 x the other writes): 4 TCC counters, then 1
  timeout -k 10 300 rocprofv3 --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum --output-format csv -d ${D}_REQ -o run -- $(run_cmd $wl $vb 5) > /dev/null 2> ${D}_REQ.err
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --output-format csv -d ${D}_REQ64 -o run -- $(run_cmd $wl $vb 5) > /dev/null 2> ${D}_REQ64.err
done
done
if [ -x ./tools/membench ] && [ -z "$NO_CALIB" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/calib_$c -o run -- ./tools/membench calib > $OUT/calib_$c.jsonl 2> $OUT/calib_$c.err
  done
fi
echo profile-done
