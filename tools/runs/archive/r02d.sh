set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 ./tools/pair_ab 10 6 4 > $O/pair_ab.jsonl 2> $O/pair_ab.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 200 ./tools/cbench 0 20 0:0:0:0:0:0:1:2:0 0:0:0:0:0:0:1:2:1 0:0:0:0:0:0:2:2:0 0:0:0:0:0:0:2:2:1 0:0:0:0:0:0:0:2:0 0:0:0:0:0:0:0:2:1 > $O/cb_udp64.jsonl 2> $O/cb_udp64.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 200 ./tools/cbench 1 20 0:0:0:0:0:0:1:2:0 0:0:0:0:0:0:1:2:1 0:0:0:0:0:0:2:2:0 0:0:0:0:0:0:2:2:1 > $O/cb_tcp1500.jsonl 2> $O/cb_tcp1500.err
echo rc=$?
