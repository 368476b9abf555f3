#!/bin/bash
# SQ instruction-mix counters for the classify kernel (one PMC pass per group).
#   WL=udp64|tcp1500|ingress_nic|ingress_ws OUT=gpurun_out/sq bash tools/sqprof.sh
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sq}
mkdir -p $OUT
wl=${WL:-udp64}
case $wl in
  ingress_nic) CMD="python3 tools/ingress_run.py 4 --nic-only" ;;
  ingress_ws) CMD="python3 tools/ingress_run.py 4 --ws-only" ;;
  *) CMD="python3 bench.py --workload $wl --steps 4 --warmup 1 --no-cpu --no-secondary --no-e2e" ;;
esac
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" "SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_LOAD"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/${wl}_g$i -o run -- $CMD > /dev/null 2> $OUT/${wl}_g$i.err
done
echo sq-done
