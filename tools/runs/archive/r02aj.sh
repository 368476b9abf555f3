# udp64 verdict-store policy (GCL_TUNE_NT_STORE 0 plain / 1 nontemporal /
# 2 write-through, the default) on the current build against the old build,
# 8-B and 2-B verdicts, fresh bench.py process each, one box.
set -o pipefail
O=gpurun_out/r02aj; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-new_s2 new_s0 new_s1 old_s2 new_s2b old_s2b}; do
  lib=${v%%_*}; st=${v#*_s}; st=${st%b}
  cp tools/_ab/libgclassify_$lib.so caladan_amd/libgclassify.so || exit 1
  for vb in 8 2; do
    GCL_TUNE_NT_STORE=$st timeout -k 10 240 python3 bench.py --workload udp64 --verdict-bytes $vb --no-cpu --no-secondary --no-e2e --steps 200 --warmup 20 > $O/bench_v${vb}_$v.json 2> $O/bench_v${vb}_$v.err || exit $?
  done
done
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
