# round 5: the deferred verdicts' register extension (GCL_TUNE_DEFER=3:
# tiles past a full LDS buffer in a shift register of 10 dwords per lane, so
# udp64's whole share is written after the reads): parity, then the A/B of
# all forms on the bench's placed buffers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or verdict1 or geometr" > gpurun_out/r05g_densetests.log 2>&1 || { tail -30 gpurun_out/r05g_densetests.log; exit 1; }
tail -2 gpurun_out/r05g_densetests.log
AB_ROUNDS=5 timeout -k 10 300 python tools/defer_ab.py udp64 > gpurun_out/r05g_defer_ab.jsonl 2> gpurun_out/r05g_defer_ab.err || { tail -5 gpurun_out/r05g_defer_ab.err; exit 1; }
cat gpurun_out/r05g_defer_ab.jsonl
