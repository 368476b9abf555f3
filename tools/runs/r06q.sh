# round 6: gcl_tune.vstage (the register-held deferred verdicts written 16 B
# per lane through the LDS buffer) -- the dense parity cases, then the A/B on
# the bench's placed buffers in three fresh processes (kernel and its
# kernel-shape ceiling per form)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or access_probe or ctx_tune" > gpurun_out/r06q_tests.log 2>&1 || { tail -30 gpurun_out/r06q_tests.log; exit 1; }
tail -1 gpurun_out/r06q_tests.log
for i in 1 2 3; do
  AB_KNOB=vstage timeout -k 10 300 python tools/tile_ab.py udp64 > gpurun_out/r06q_vstage_ab_$i.jsonl 2> gpurun_out/r06q_vstage_ab_$i.err || { tail -5 gpurun_out/r06q_vstage_ab_$i.err; exit 1; }
  grep -h "check\|round" gpurun_out/r06q_vstage_ab_$i.jsonl | cut -c1-400
done
echo r06q-done
