# round 5: the deferred verdicts' gain against where the frame pool lands
# (12 pools in allocation order, spacers between, one verdict ring)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/defer_place.py 12 > gpurun_out/r05r_defer_place.jsonl 2> gpurun_out/r05r_defer_place.err || { tail -5 gpurun_out/r05r_defer_place.err; exit 1; }
cat gpurun_out/r05r_defer_place.jsonl
