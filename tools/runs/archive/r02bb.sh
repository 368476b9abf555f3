# Experiment: one vs two alternating streams for consecutive udp64 steps, in
# one process on the same buffers (tools/streams_ab.py), two processes.
set -o pipefail
O=gpurun_out/r02bb; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/streams_ab.py > $O/ab_$i.json 2> $O/ab_$i.err || exit $?
done
echo rc=0
