set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_a.json 2> $O/ingress_a.err &&
timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_b.json 2> $O/ingress_b.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:2:2 > $O/cb_udp64.jsonl 2> $O/cb_udp64.err
echo rc=$?
