# round 5: the verdict deferral moved into the tile kernel (GCL_TUNE_DEFER
# 0/1/2; the pair-kernel DENSE form lost, r05e) and the two-poller loop
# removed (lost on header records, r05e): parity for both, then the
# deferral A/B on the bench's placed buffers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or verdict1 or geometr" > gpurun_out/r05f_densetests.log 2>&1 || { tail -30 gpurun_out/r05f_densetests.log; exit 1; }
tail -2 gpurun_out/r05f_densetests.log
timeout -k 10 300 python tools/defer_ab.py > gpurun_out/r05f_defer_ab.jsonl 2> gpurun_out/r05f_defer_ab.err || { tail -5 gpurun_out/r05f_defer_ab.err; exit 1; }
cat gpurun_out/r05f_defer_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_looptests.log 2>&1 || { tail -30 gpurun_out/r05f_looptests.log; exit 1; }
tail -2 gpurun_out/r05f_looptests.log
