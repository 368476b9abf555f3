# round-4 final tree: full GPU suite, smoke, bench (driver's command), the
# lone-burst stages and shallow pipeline rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zm_gputests.log 2>&1 || { tail -30 gpurun_out/r04zm_gputests.log; exit 1; }
tail -2 gpurun_out/r04zm_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zm_smoke.log 2>&1 || { cat gpurun_out/r04zm_smoke.log; exit 1; }
cat gpurun_out/r04zm_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r04zm_bench.json 2> gpurun_out/r04zm_bench.err || { tail -5 gpurun_out/r04zm_bench.err; exit 1; }
bash tools/runs/r04c.sh r04zm > /dev/null || exit 1
grep -h lone gpurun_out/r04zm_stages.jsonl | cut -c1-300
