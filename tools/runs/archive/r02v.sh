set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
export TMPDIR=/tmp
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:2:2 0:0:2:512:0:0:2:2 0:0:1:512:0:0:2:2 0:0:1:1024:0:0:2:2 0:0:2:256:3:0:2:2 0:0:2:256:2:0:2:2 0:0:1:256:0:0:2:2 > $O/cb_udp64_geom.jsonl 2> $O/cb_udp64_geom.err
echo rc=$?
