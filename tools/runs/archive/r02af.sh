# Dense layouts: the build with the explicit first-half drain (newa) against
# the old build and the undrained one (new), fresh process each.
set -o pipefail
O=gpurun_out/r02af; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-newa old new newa2 old2}; do
  cp tools/_ab/libgclassify_${v%2}.so caladan_amd/libgclassify.so || exit 1
  for wl in udp64 tcp1500; do
    timeout -k 10 240 python3 bench.py --workload $wl --no-cpu --no-secondary --no-e2e --steps 200 --warmup 20 > $O/bench_${wl}_$v.json 2> $O/bench_${wl}_$v.err || exit $?
  done
done
cp tools/_ab/libgclassify_newa.so caladan_amd/libgclassify.so
echo done
