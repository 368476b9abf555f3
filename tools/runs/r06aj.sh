# round 6: the final kernel's per-launch time over 3000 back-to-back launches
# (~1 s) on a plain and on a placed pool, then the bench's timed loop three
# times: is the plain pool's 307 us a boost transient?
set -o pipefail
mkdir -p gpurun_out
for pl in 0 1; do
  GCL_BENCH_PLACEMENT=$pl timeout -k 10 300 python tools/drift.py 1 3000 250 > gpurun_out/r06aj_drift_pl$pl.jsonl 2> gpurun_out/r06aj_drift_pl$pl.err || { tail -5 gpurun_out/r06aj_drift_pl$pl.err; exit 1; }
  echo "placement=$pl"; python -c 'import json,sys; [print(json.dumps({k:v for k,v in json.loads(l).items() if k!="placement"})) for l in open(sys.argv[1])]' gpurun_out/r06aj_drift_pl$pl.jsonl
done
echo r06aj-done
