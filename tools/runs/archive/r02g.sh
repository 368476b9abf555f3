set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
ROUND=r02 WLS="udp64 tcp1500 ingress_nic" VBS="4 2" timeout -k 10 1200 bash tools/profile.sh > $O/profile.log 2>&1
echo rc=$?
