# Evidence for the final kernel (dense drains at the lookup and the first
# stage): the driver's command twice, strong scaling at N=1, smoke, and the
# rocprof set for udp64, tcp1500 and both ingress rows.
set -o pipefail
O=gpurun_out/r02al; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > $O/bench_a.json 2> $O/bench_a.err &&
timeout -k 10 700 python -u bench.py > $O/bench_b.json 2> $O/bench_b.err &&
timeout -k 10 700 python -u bench.py --scaling strong --no-cpu --no-secondary --no-e2e --steps 10 --warmup 3 > $O/bench_strong.json 2> $O/bench_strong.err &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
ROUND=r02l WLS="udp64 tcp1500 ingress_nic ingress_ws" VBS="2" NO_CALIB=1 timeout -k 10 900 bash tools/profile.sh > $O/profile.log 2>&1
echo rc=$?
