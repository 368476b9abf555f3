# Timing-only: the working-set row without the end-of-tile barriers
# (GCL_TUNE_ABLATE=128 on an experiment build; results race) against the
# same build with them.
set -o pipefail
O=gpurun_out/r02ak; mkdir -p $O
export TMPDIR=/tmp
cp tools/_ab/libgclassify_nb.so caladan_amd/libgclassify.so || exit 1
for a in 0 128 0 128; do
  GCL_TUNE_ABLATE=$a timeout -k 10 240 python3 tools/ingress_run.py 10 --vbytes 8 > $O/ing_a$a.json 2> $O/ing_a$a.err || exit $?
  cat $O/ing_a$a.json
done
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
