# Experiment: cache policy of the dense frame loads (GCL_TUNE_LDAUX buffer
# loads: 2 nt, 0 plain, 16 sc1, 18 sc1 nt; unset = global_load nt, the
# default) and an agent-scope verdict store (GCL_TUNE_NT_STORE=3); udp64
# kernel-only lines, fresh processes.
set -o pipefail
O=gpurun_out/r02bh; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 100 > $O/$n.json 2> $O/$n.err; }
for i in 1 2; do
  run def_$i GCL_X=0 || exit $?
  run ld2_$i GCL_TUNE_LDAUX=2 || exit $?
  run ld0_$i GCL_TUNE_LDAUX=0 || exit $?
  run ld16_$i GCL_TUNE_LDAUX=16 || exit $?
  run ld18_$i GCL_TUNE_LDAUX=18 || exit $?
  run st3_$i GCL_TUNE_NT_STORE=3 || exit $?
done
echo rc=0
