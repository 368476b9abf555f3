# Timing-only A/B: the GENERAL tile loop without its ol_flags / hash.rss loads
# (tools/_ab/libgclassify_noside.so, wrong verdicts by design) vs the
# current build, ingress rows, fresh processes alternating.
set -o pipefail
O=gpurun_out/r02az; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in new noside; do
    cp tools/_ab/libgclassify_$v.so caladan_amd/libgclassify.so || exit 1
    timeout -k 10 240 python3 tools/ingress_run.py 10 > $O/ingress_${v}_$i.json 2> $O/ingress_${v}_$i.err || exit $?
  done
done
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo rc=0
