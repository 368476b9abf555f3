# Tile depth on the dense layouts: new build at GCL_TUNE_DEPTH=1 / 2 (default)
# against the old build, fresh process each.
set -o pipefail
O=gpurun_out/r02ae; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-new_d1 new_d2 old_d0 new_d1b old_d0b}; do
  lib=${v%%_*}; d=${v#*_d}; d=${d%b}
  cp tools/_ab/libgclassify_$lib.so caladan_amd/libgclassify.so || exit 1
  for wl in udp64 tcp1500; do
    if [ "$d" = 0 ]; then unset GCL_TUNE_DEPTH; else export GCL_TUNE_DEPTH=$d; fi
    timeout -k 10 240 python3 bench.py --workload $wl --no-cpu --no-secondary --no-e2e --steps 200 --warmup 20 > $O/bench_${wl}_$v.json 2> $O/bench_${wl}_$v.err || exit $?
  done
done
unset GCL_TUNE_DEPTH
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
