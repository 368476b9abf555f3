# GENERAL occupancy: 5 waves per SIMD (<= 96 VGPRs, some spills) with 5
# blocks per CU, against the current build at 4; ingress rows, fresh
# process each, one box.
set -o pipefail
O=gpurun_out/r02am; mkdir -p $O
export TMPDIR=/tmp
for v in new wfive new2 wfive2; do
  cp tools/_ab/libgclassify_${v%2}.so caladan_amd/libgclassify.so || exit 1
  if [ "${v%2}" = wfive ]; then export GCL_TUNE_BLOCKS_PER_CU=5; else unset GCL_TUNE_BLOCKS_PER_CU; fi
  timeout -k 10 240 python3 tools/ingress_run.py 10 > $O/ingress_$v.json 2> $O/ingress_$v.err || exit $?
done
unset GCL_TUNE_BLOCKS_PER_CU
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
