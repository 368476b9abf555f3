# What bounds the register-header GENERAL kernel on the working-set row:
# GCL_TUNE_ABLATE variants (timing only) in fresh processes, tile kernel beside.
set -o pipefail
O=gpurun_out/r02aq; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for a in 0 2 14 15 128; do
    GCL_TUNE_ABLATE=$a timeout -k 10 200 python3 -u tools/ingress_run.py 10 --ws-only > $O/ws_a${a}_$i.json 2> $O/ws_a${a}_$i.err || exit $?
  done
  GCL_TUNE_QUAD=0 timeout -k 10 200 python3 -u tools/ingress_run.py 10 --ws-only > $O/ws_q0_$i.json 2> $O/ws_q0_$i.err || exit $?
done
echo rc=0
