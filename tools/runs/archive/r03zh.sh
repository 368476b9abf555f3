# final round-3 tree: kernel-trace passes of the headline (udp64) and config-3 (tcp1500) bench
# commands, summarised by tools/prof_summary.py r03f (timed dispatches only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r03f
for wl in udp64 tcp1500; do
  D=gpurun_out/prof_r03f/${wl}_v2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${D}_trace -o run -- python3 bench.py --workload $wl --verdict-bytes 2 --no-cpu --no-secondary --no-e2e --no-group --steps 20 --warmup 5 > ${D}_bench.json 2> ${D}_trace.err || { tail ${D}_trace.err; exit 1; }
done
python3 tools/prof_summary.py r03f
