# round 3, first GPU call: the multi-GPU group (C ABI + RCCL), the struct
# fixture test, and a short bench with the group line
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_group.py "tests/test_gpu_parity.py::test_gpu_reference_struct_frames" \
  > gpurun_out/r03a/tests.log 2>&1 || { tail -30 gpurun_out/r03a/tests.log; exit 1; }
tail -3 gpurun_out/r03a/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-secondary --no-e2e --no-cpu \
  > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { tail -20 gpurun_out/r03a/bench.err; exit 1; }
cat gpurun_out/r03a/bench.json
