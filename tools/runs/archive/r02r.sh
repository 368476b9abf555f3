set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
GCL_TUNE_OFFS_LDS=0 timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_offs0.json 2> $O/ingress0.err &&
GCL_TUNE_OFFS_LDS=1 timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_offs1.json 2> $O/ingress1.err &&
GCL_TUNE_OFFS_LDS=0 timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_offs0b.json 2> $O/ingress0b.err &&
GCL_TUNE_OFFS_LDS=1 timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress_offs1b.json 2> $O/ingress1b.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:2:2 0:0:0:0:0:0:1:2 > $O/cb_udp64.jsonl 2> $O/cb_udp64.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 1 20 0:0:0:0:0:0:2:2 > $O/cb_tcp1500.jsonl 2> $O/cb_tcp1500.err
echo rc=$?
