# rxloop64_kernel with uniform descriptors and broadcasts: loop tests, then
# lone-burst stages and shallow rows: writer wave / poller stores / general kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1 || { tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -2 gpurun_out/r04s_tests.log
for v in "1 1" "1 0" "0 1"; do
  set -- $v
  GCL_TUNE_LOOP64=$1 GCL_TUNE_LOOP_WRITER=$2 bash tools/runs/r04c.sh r04s_k$1w$2 > /dev/null || exit 1
done
for v in k1w1 k1w0 k0w1; do echo "$v"; grep -h lone gpurun_out/r04s_${v}_stages.jsonl | cut -c1-420; grep -h '"workers"' gpurun_out/r04s_${v}_stages.jsonl | cut -c1-200; done
