# Register-header GENERAL kernel at 4 vs 5 blocks per CU (83 VGPRs admit 5
# waves per SIMD), ingress rows, fresh processes.
set -o pipefail
O=gpurun_out/r02as; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for b in 4 5; do
    GCL_TUNE_BLOCKS_PER_CU=$b timeout -k 10 200 python3 -u tools/ingress_run.py 10 > $O/b${b}_$i.json 2> $O/b${b}_$i.err || exit $?
  done
done
echo rc=0
