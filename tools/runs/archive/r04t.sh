# planar header records: loop tests, then lone-burst stages and shallow rows,
# rxloop64 (poller stores) against the general loop kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1 || { tail -30 gpurun_out/r04t_tests.log; exit 1; }
tail -2 gpurun_out/r04t_tests.log
for k in 1 0; do
  GCL_TUNE_LOOP64=$k bash tools/runs/r04c.sh r04t_k$k > /dev/null || exit 1
done
for k in 1 0; do echo "k64 $k"; grep -h lone gpurun_out/r04t_k${k}_stages.jsonl | cut -c1-420; grep -h '"workers"' gpurun_out/r04t_k${k}_stages.jsonl | cut -c1-200; done
