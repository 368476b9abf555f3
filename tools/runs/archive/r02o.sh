set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
# tcp1500, 2-byte verdicts, write-through: default geometry vs 1024-lane tiles, depth 1/2, grid caps
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 1 20 0:0:0:0:0:0:2:2 0:0:1:0:0:0:2:2 0:0:2:1024:0:0:2:2 0:0:1:1024:0:0:2:2 0:0:2:256:0:0:2:2 0:0:2:512:1:0:2:2 0:0:0:0:0:1:2:2 > $O/cb_tcp1500_geom.jsonl 2> $O/cb_tcp1500_geom.err
echo rc=$?
