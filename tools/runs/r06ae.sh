# round 6: how the final kernel's time spreads over frame-pool placements,
# and whether the placement probe (the minimal per-packet shape) predicts it:
# 12 pools against one verdict ring, per-packet stores and the default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/defer_place.py 12 > gpurun_out/r06ae_place.jsonl 2> gpurun_out/r06ae_place.err || { tail -5 gpurun_out/r06ae_place.err; exit 1; }
cat gpurun_out/r06ae_place.jsonl
echo r06ae-done
