# round 5: classify_pair_kernel's lean path (GCL_TUNE_PAIR_LEAN=1: waves of
# plain IPv4 packets on classify_lean): the whole parity file with it on,
# then the A/B on the integrated ingress rows
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_PAIR_LEAN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05n_parity_lean.log 2>&1 || { tail -30 gpurun_out/r05n_parity_lean.log; exit 1; }
tail -1 gpurun_out/r05n_parity_lean.log
timeout -k 10 400 python tools/pair_lean_ab.py 4 > gpurun_out/r05n_pair_lean_ab.jsonl 2> gpurun_out/r05n_pair_lean_ab.err || { tail -5 gpurun_out/r05n_pair_lean_ab.err; exit 1; }
cat gpurun_out/r05n_pair_lean_ab.jsonl
