# round 6: wave-staged tiles (gcl_tune.stage 1) and the kernel-shape ceiling
# probe: the parity suite's dense and probe tests, then the stage A/B on the
# bench's placed buffers (three fresh processes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or probe or geometries or ctx_tune" > gpurun_out/r06b_tests.log 2>&1 || { tail -30 gpurun_out/r06b_tests.log; exit 1; }
tail -1 gpurun_out/r06b_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/stage_ab.py udp64 tcp1500 > gpurun_out/r06b_stage_ab_$i.jsonl 2> gpurun_out/r06b_stage_ab_$i.err || { tail -5 gpurun_out/r06b_stage_ab_$i.err; exit 1; }
  grep round gpurun_out/r06b_stage_ab_$i.jsonl | tail -2
done
echo r06b-done
