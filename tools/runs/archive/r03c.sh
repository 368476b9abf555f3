# round 3: what bounds the GENERAL path on the working-set row: knob A/B
# (tools/ws_ab.py) and SQ instruction counters (tools/sqprof.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u tools/ws_ab.py 3 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
cat $O/ws_ab.jsonl
for wl in ingress_ws udp64; do
  WL=$wl OUT=gpurun_out/sq_r03 timeout -k 10 900 bash tools/sqprof.sh > $O/sq_$wl.log 2>&1 || { tail $O/sq_$wl.log; exit 1; }
done
echo done
