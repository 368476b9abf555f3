# Verdict store encodings on udp64 (2-B verdicts): GCL_TUNE_NT_STORE 2 (sc0
# sc1, default), 3 (sc0 sc1 nt), 4 (sc1 nt), fresh processes alternating.
set -o pipefail
O=gpurun_out/r02av; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for st in 2 3 4; do
    GCL_TUNE_NT_STORE=$st timeout -k 10 300 python3 -u bench.py --no-cpu --no-secondary --no-e2e --steps 50 > $O/st${st}_$i.json 2> $O/st${st}_$i.err || exit $?
  done
done
echo rc=0
