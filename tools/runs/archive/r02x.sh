set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
export TMPDIR=/tmp
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 1 20 0:0:0:0:0:0:2:2 64:0:0:0:0:0:2:2 4:0:0:0:0:0:2:2 68:0:0:0:0:0:2:2 2:0:0:0:0:0:2:2 1:0:0:0:0:0:2:2 > $O/cb_tcp1500_ablate.jsonl 2> $O/cb_tcp1500_ablate.err
echo rc=$?
