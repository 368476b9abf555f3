# Ablations of the working-set ingress row (GCL_TUNE_ABLATE bits, timing
# only): 8-B verdicts so the membench body (16) stays inside the buffer.
set -o pipefail
O=gpurun_out/r02ad; mkdir -p $O
export TMPDIR=/tmp
for a in 0 16 1 2 4 8 15 64 79 0; do
  GCL_TUNE_ABLATE=$a timeout -k 10 240 python3 tools/ingress_run.py 10 --ws-only --vbytes 8 > $O/ws_a$a.json 2> $O/ws_a$a.err || exit $?
  cat $O/ws_a$a.json
done
echo done
