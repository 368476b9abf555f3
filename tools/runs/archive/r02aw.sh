# Evidence for the current build (dummy loads spread): the driver's command
# twice, smoke, and the rocprof set (stats + FETCH/WRITE/request PMC passes)
# for udp64, tcp1500 and both ingress rows.
set -o pipefail
O=gpurun_out/r02aw; mkdir -p $O
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 700 python -u bench.py > $O/bench_a.json 2> $O/bench_a.err || exit $?
echo "bench wall s: $(( $(date +%s) - s ))" > $O/wall.txt
timeout -k 10 700 python -u bench.py > $O/bench_b.json 2> $O/bench_b.err || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
ROUND=r02m WLS="udp64 tcp1500 ingress_nic ingress_ws" VBS="2" NO_CALIB=1 timeout -k 10 1000 bash tools/profile.sh > $O/profile.log 2>&1
echo rc=$?
