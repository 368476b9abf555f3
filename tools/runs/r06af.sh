# round 6: the bench's placed pair (gcl_dev_alloc_paired) against plain
# allocations for the final kernel (r06ae: 306-309 us on every plainly
# allocated pool, ~316 on the bench's placed pairs), two fresh processes each
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{}]' AB_ROUNDS=3
for i in 1 2; do
  for pl in 1 0; do
    GCL_BENCH_PLACEMENT=$pl timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06af_pl${pl}_$i.jsonl 2> gpurun_out/r06af_pl${pl}_$i.err || { tail -5 gpurun_out/r06af_pl${pl}_$i.err; exit 1; }
    python -c 'import json,sys; [print(sys.argv[1], json.loads(l)["form=0"]["kernel_us"], json.loads(l)["form=0"]["probe_us"]) for l in open(sys.argv[2]) if "round" in l]' pl=$pl gpurun_out/r06af_pl${pl}_$i.jsonl
  done
done
echo r06af-done
