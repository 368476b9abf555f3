# rxloop64_kernel (bursts <= 64, one wave, writer wave): the loop tests,
# the soak, then the lone-burst stages and shallow rows against the general
# loop kernel (GCL_TUNE_LOOP64=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || { tail -30 gpurun_out/r04r_tests.log; exit 1; }
tail -2 gpurun_out/r04r_tests.log
for k in 1 0; do
  GCL_TUNE_LOOP64=$k bash tools/runs/r04c.sh r04r_k$k > /dev/null || exit 1
done
for k in 1 0; do echo "k64 $k"; grep -h lone gpurun_out/r04r_k${k}_stages.jsonl | cut -c1-420; grep -h '"workers"' gpurun_out/r04r_k${k}_stages.jsonl | cut -c1-230; done
