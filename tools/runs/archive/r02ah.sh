# Evidence for the fixed-load-count build: the driver's bench command twice
# (fresh processes), smoke, and the rocprof set (kernel trace/stats, FETCH /
# WRITE / request-size PMC passes) for udp64, tcp1500 and both ingress rows.
set -o pipefail
O=gpurun_out/r02ah; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > $O/bench_a.json 2> $O/bench_a.err &&
timeout -k 10 700 python -u bench.py > $O/bench_b.json 2> $O/bench_b.err &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
ROUND=r02h WLS="udp64 tcp1500 ingress_nic ingress_ws" VBS="2" NO_CALIB=1 timeout -k 10 900 bash tools/profile.sh > $O/profile.log 2>&1
echo rc=$?
