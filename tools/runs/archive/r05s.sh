# round 5: deferred verdicts on the pair kernel (GCL_TUNE_PAIR_DEFER=1): the
# parity file with it on, then the A/B on the ingress rows (lean waves with
# and without deferral, and the lean-off form for scale)
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_PAIR_DEFER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05s_parity_pdefer.log 2>&1 || { tail -30 gpurun_out/r05s_parity_pdefer.log; exit 1; }
tail -1 gpurun_out/r05s_parity_pdefer.log
AB_FORMS=0,1,2 timeout -k 10 400 python tools/pair_lean_ab.py 4 > gpurun_out/r05s_pair_ab.jsonl 2> gpurun_out/r05s_pair_ab.err || { tail -5 gpurun_out/r05s_pair_ab.err; exit 1; }
cat gpurun_out/r05s_pair_ab.jsonl
