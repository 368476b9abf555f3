# round 6: the HBM read speed of light at the header-split slab's size (8 Mi x
# 64 B = 512 MiB) and at 1 GiB (tools/read_sol)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/read_sol $((512 << 20)) 40 > gpurun_out/r06ap_read_sol_512m.jsonl 2> gpurun_out/r06ap_read_sol.err || { tail -5 gpurun_out/r06ap_read_sol.err; exit 1; }
timeout -k 10 120 ./tools/read_sol $((1 << 30)) 30 > gpurun_out/r06ap_read_sol_1g.jsonl 2>> gpurun_out/r06ap_read_sol.err || { tail -5 gpurun_out/r06ap_read_sol.err; exit 1; }
tail -1 gpurun_out/r06ap_read_sol_512m.jsonl
tail -1 gpurun_out/r06ap_read_sol_1g.jsonl
echo r06ap-done
