# round 6: placed (gcl_dev_alloc_paired) against plain pools for the other
# dense rows: tcp1500 (deferred 2-B verdicts) and udp64 with 4-B verdicts
# (per-packet stores, what placement was built for); two processes each
set -o pipefail
mkdir -p gpurun_out
export AB_FORMS='[{}]' AB_ROUNDS=3
for i in 1 2; do
  for pl in 1 0; do
    GCL_BENCH_PLACEMENT=$pl timeout -k 10 300 python tools/tile_ab.py tcp1500 > gpurun_out/r06ag_tcp_pl${pl}_$i.jsonl 2> gpurun_out/r06ag_tcp_pl${pl}_$i.err || { tail -5 gpurun_out/r06ag_tcp_pl${pl}_$i.err; exit 1; }
    AB_VBYTES=4 GCL_BENCH_PLACEMENT=$pl timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06ag_v4_pl${pl}_$i.jsonl 2> gpurun_out/r06ag_v4_pl${pl}_$i.err || { tail -5 gpurun_out/r06ag_v4_pl${pl}_$i.err; exit 1; }
    for t in tcp v4; do
      python -c 'import json,sys; print(sys.argv[1], [json.loads(l)["form=0"]["kernel_us"] for l in open(sys.argv[2]) if "round" in l])' "$t pl=$pl" gpurun_out/r06ag_${t}_pl${pl}_$i.jsonl
    done
  done
done
echo r06ag-done
