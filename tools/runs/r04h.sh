# clock probe, then the lone-burst stages and shallow rows with the poll on
# s_memrealtime (clock 0) and on s_memtime (clock 1), twice interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/clock_probe > gpurun_out/r04h_clock.jsonl || exit 1
cat gpurun_out/r04h_clock.jsonl
for rep in 1 2; do
  for clk in 0 1; do
    GCL_TUNE_LOOP_CLOCK=$clk bash tools/runs/r04c.sh r04h_clk${clk} > /dev/null || exit 1
  done
done
for clk in 0 1; do echo "clock $clk"; grep -h lone gpurun_out/r04h_clk${clk}_stages.jsonl | cut -c1-400; grep -h '"workers": 4' gpurun_out/r04h_clk${clk}_stages.jsonl | cut -c1-200; done
