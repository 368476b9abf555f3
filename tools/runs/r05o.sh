# round 5: the pair kernel's lean path on by default: its parity test in both
# settings, then the whole GPU suite and smoke on the tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pair_lean" > gpurun_out/r05o_pair_lean.log 2>&1 || { tail -30 gpurun_out/r05o_pair_lean.log; exit 1; }
tail -1 gpurun_out/r05o_pair_lean.log
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05o_gputests.log 2>&1 || { tail -30 gpurun_out/r05o_gputests.log; exit 1; }
tail -1 gpurun_out/r05o_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05o_smoke.log 2>&1 || { tail -5 gpurun_out/r05o_smoke.log; exit 1; }
tail -1 gpurun_out/r05o_smoke.log
