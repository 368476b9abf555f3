# Ingress pool placed against its verdict ring (gcl_dev_alloc_paired, the
# default now) vs plain allocations (GCL_BENCH_PLACEMENT=0), fresh
# processes alternating; then the bench e2e leg once (zero-copy copy path).
set -o pipefail
O=gpurun_out/r02be; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python3 -u tools/ingress_run.py 10 > $O/placed_$i.json 2> $O/placed_$i.err || exit $?
  GCL_BENCH_PLACEMENT=0 timeout -k 10 300 python3 -u tools/ingress_run.py 10 > $O/plain_$i.json 2> $O/plain_$i.err || exit $?
done
timeout -k 10 300 python3 -u -c "
import json, torch, bench
d = torch.device('cuda', 0)
print(json.dumps(bench.ingress_pool_bench(d, bench.VERDICT_BYTES, reps=5, zerocopy=True)))" > $O/e2e.json 2> $O/e2e.err || exit $?
echo rc=0
