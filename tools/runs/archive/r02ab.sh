set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
export TMPDIR=/tmp
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:2:2 64:0:0:0:0:0:2:2 4:0:0:0:0:0:2:2 > $O/cb_udp64_flush.jsonl 2> $O/cb.err
echo rc=$?
