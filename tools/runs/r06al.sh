# round 6: the HBM read speed of light for the udp64 slab's 2 GiB (tools/read_sol)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/read_sol > gpurun_out/r06al_read_sol.jsonl 2> gpurun_out/r06al_read_sol.err || { tail -5 gpurun_out/r06al_read_sol.err; exit 1; }
timeout -k 10 120 ./tools/read_sol $((8 << 30)) 10 > gpurun_out/r06al_read_sol_8g.jsonl 2>> gpurun_out/r06al_read_sol.err || { tail -5 gpurun_out/r06al_read_sol.err; exit 1; }
sort -t: -k8 -n gpurun_out/r06al_read_sol.jsonl | tail -4
tail -1 gpurun_out/r06al_read_sol_8g.jsonl
echo r06al-done
