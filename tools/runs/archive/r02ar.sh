# Verdict store policy on the ingress rows (GCL_TUNE_NT_STORE 2 write-through,
# 0 plain, 1 non-temporal), register-header and tile kernels, fresh processes.
set -o pipefail
O=gpurun_out/r02ar; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for q in 1 0; do
    for st in 2 0 1; do
      GCL_TUNE_QUAD=$q GCL_TUNE_NT_STORE=$st timeout -k 10 200 python3 -u tools/ingress_run.py 10 > $O/q${q}_st${st}_$i.json 2> $O/q${q}_st${st}_$i.err || exit $?
    done
  done
done
echo rc=0
