# udp64 with 8-B and 4-B verdicts: current build against the old (1c1256a),
# fresh bench.py process each, one box.
set -o pipefail
O=gpurun_out/r02ai; mkdir -p $O
export TMPDIR=/tmp
for v in new old new2 old2; do
  cp tools/_ab/libgclassify_${v%2}.so caladan_amd/libgclassify.so || exit 1
  for vb in 8 4; do
    timeout -k 10 240 python3 bench.py --workload udp64 --verdict-bytes $vb --no-cpu --no-secondary --no-e2e --steps 200 --warmup 20 > $O/bench_v${vb}_$v.json 2> $O/bench_v${vb}_$v.err || exit $?
  done
done
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
