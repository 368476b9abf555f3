# round 6: the rx-loop suite alone (r06a's failure: test_rxloop_fuzz_vs_oracle
# [2-8-0-2-1], device counts 12 short on one runtime with every verdict right),
# with the counts / stats / poll-counter diagnostics; then the rest of the GPU
# suite, smoke, the rocprofv3 passes, the 2-rank rehearsal and the stage A/B.
# An assertion failure in the loop suite is not a GPU fault: the rest runs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06c_rxloop.log 2>&1; rc=$?
tail -5 gpurun_out/r06c_rxloop.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread --ignore tests/test_gpu_rxloop.py > gpurun_out/r06c_rest.log 2>&1 || { tail -30 gpurun_out/r06c_rest.log; exit 1; }
tail -1 gpurun_out/r06c_rest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || { tail -5 gpurun_out/r06c_smoke.log; exit 1; }
tail -1 gpurun_out/r06c_smoke.log
for i in 1 2; do
  timeout -k 10 300 python tools/stage_ab.py udp64 tcp1500 > gpurun_out/r06c_stage_ab_$i.jsonl 2> gpurun_out/r06c_stage_ab_$i.err || { tail -5 gpurun_out/r06c_stage_ab_$i.err; exit 1; }
  grep round gpurun_out/r06c_stage_ab_$i.jsonl | tail -2
done
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --steps 10 --warmup 2 --no-e2e --cpu-budget 10 > gpurun_out/r06c_bench_gloo2.json 2> gpurun_out/r06c_bench_gloo2.err || { tail -5 gpurun_out/r06c_bench_gloo2.err; exit 1; }
head -c 300 gpurun_out/r06c_bench_gloo2.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r06c WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06c_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r06c_prof_udp64.log; exit 1; }
ROUND=r06c WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06c_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r06c_prof_tcp1500.log; exit 1; }
echo r06c-done rxloop_rc=$rc
