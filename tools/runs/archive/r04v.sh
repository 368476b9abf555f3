# round-4 re-entry (3rd session): full GPU suite, smoke, bench (driver's
# command, 1-B verdict headline), rocprofv3 trace + PMC passes of the udp64
# launch with 1-B verdicts, clock probe, lone-burst stages and shallow rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_gputests.log 2>&1 || { tail -30 gpurun_out/r04v_gputests.log; exit 1; }
tail -2 gpurun_out/r04v_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04v_smoke.log 2>&1 || { cat gpurun_out/r04v_smoke.log; exit 1; }
cat gpurun_out/r04v_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r04v_bench.json 2> gpurun_out/r04v_bench.err || { tail -5 gpurun_out/r04v_bench.err; exit 1; }
NO_CALIB=1 ROUND=r04 WLS="udp64" VBS="1" timeout -k 10 600 bash tools/profile.sh > gpurun_out/r04v_profile.log 2>&1 || { tail -20 gpurun_out/r04v_profile.log; exit 1; }
timeout -k 10 60 tools/clock_probe > gpurun_out/r04v_clock.jsonl || exit 1
cat gpurun_out/r04v_clock.jsonl
bash tools/runs/r04c.sh r04v > /dev/null || exit 1
grep -h lone gpurun_out/r04v_stages.jsonl | cut -c1-400
