# rxloop64_kernel's lean path (classify_lean for plain-IPv4 bursts): the loop
# tests (the lean-path parity test included), then the lone-burst stages and
# shallow rows with the lean path on and off, interleaved twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zb_tests.log 2>&1 || { tail -30 gpurun_out/r04zb_tests.log; exit 1; }
tail -2 gpurun_out/r04zb_tests.log
for lean in 1 0 1 0; do
  GCL_TUNE_LOOP_LEAN=$lean bash tools/runs/r04c.sh r04zb_lean$lean > /dev/null || exit 1
done
for lean in 1 0; do echo "lean $lean"; grep -h lone gpurun_out/r04zb_lean${lean}_stages.jsonl | cut -c1-330; grep -h '"workers"' gpurun_out/r04zb_lean${lean}_stages.jsonl | cut -c1-170; done
