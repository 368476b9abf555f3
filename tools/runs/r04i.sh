# round-4 GPU session: clock probe, full GPU suite, clock A/B of the loop, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/clock_probe > gpurun_out/r04i_clock.jsonl || exit 1
cat gpurun_out/r04i_clock.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_gputests.log 2>&1 || { tail -30 gpurun_out/r04i_gputests.log; exit 1; }
tail -2 gpurun_out/r04i_gputests.log
for clk in 0 1; do
  GCL_TUNE_LOOP_CLOCK=$clk bash tools/runs/r04c.sh r04i_clk${clk} > /dev/null || exit 1
done
for clk in 0 1; do echo "clock $clk"; grep -h lone gpurun_out/r04i_clk${clk}_stages.jsonl | cut -c1-420; grep -h '"workers": 4' gpurun_out/r04i_clk${clk}_stages.jsonl | cut -c1-160; done
