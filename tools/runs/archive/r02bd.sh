# Experiment: allocation flags of the verdict ring (GCL_DEV_ALLOC_FLAGS) and
# the frame pool (GCL_PAIR_ALLOC_FLAGS): 3 = hipDeviceMallocUncached,
# 1 = fine-grained.  udp64 kernel-only bench lines, fresh processes.
set -o pipefail
O=gpurun_out/r02bd; mkdir -p $O
export TMPDIR=/tmp
run() { # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 100 > $O/$n.json 2> $O/$n.err
}
for i in 1 2; do
  run base_$i GCL_X=0 || exit $?
  run vuc_$i GCL_DEV_ALLOC_FLAGS=3 || exit $?
  run fuc_$i GCL_PAIR_ALLOC_FLAGS=3 || exit $?
  run vfg_$i GCL_DEV_ALLOC_FLAGS=1 || exit $?
done
echo rc=0
