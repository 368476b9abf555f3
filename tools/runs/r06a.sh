# round 6: the library split into translation units, gcl_tune replacing the
# GCL_TUNE_* environment: the whole GPU suite, smoke, then rocprofv3 kernel
# trace of the two dominant launches (udp64 1-B, tcp1500 2-B) to check their
# kernel times against round 5's (330.2 / 177.4 us)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06a_gputests.log 2>&1 || { tail -30 gpurun_out/r06a_gputests.log; exit 1; }
tail -1 gpurun_out/r06a_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a_smoke.log 2>&1 || { tail -5 gpurun_out/r06a_smoke.log; exit 1; }
tail -1 gpurun_out/r06a_smoke.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r06a WLS=udp64 VBS=1 NO_CALIB=1 REQ_ONLY= timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06a_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r06a_prof_udp64.log; exit 1; }
ROUND=r06a WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06a_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r06a_prof_tcp1500.log; exit 1; }
echo r06a-prof-done
# the N=2 line rehearsed on one GPU (2 gloo ranks sharing it): group_node
# (gcl_group over the line's 2 GPUs -- here 2 contexts on one, host exchange)
# and the CPU baseline from a CPU-only child, merged into rank 0's line
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 10 --warmup 2 --no-e2e --cpu-budget 10 > gpurun_out/r06a_bench_gloo2.json 2> gpurun_out/r06a_bench_gloo2.err || { tail -5 gpurun_out/r06a_bench_gloo2.err; exit 1; }
cat gpurun_out/r06a_bench_gloo2.json | head -c 600
echo r06a-gloo2-done
