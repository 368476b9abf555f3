# rxloop64 finer stage stamps (classified, records issued) + the bench's rx
# loop leg without stamps, loop64 against the general kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1 || { tail -30 gpurun_out/r04v_tests.log; exit 1; }
tail -1 gpurun_out/r04v_tests.log
for k in 1 0; do
  GCL_TUNE_LOOP64=$k bash tools/runs/r04c.sh r04v_k$k > /dev/null || exit 1
  GCL_TUNE_LOOP64=$k timeout -k 10 300 python tools/rxloop_run.py > gpurun_out/r04v_rxloop_k$k.json || exit 1
done
for k in 1 0; do echo "k64 $k"; grep -h lone gpurun_out/r04v_k${k}_stages.jsonl | cut -c1-520; grep -h '"workers"' gpurun_out/r04v_k${k}_stages.jsonl | cut -c1-200; python3 -c "
import json; d=json.load(open('gpurun_out/r04v_rxloop_k$k.json'))
for k,v in d.items():
    if isinstance(v,dict): print(k, v.get('p50_us'), v.get('mpps'))"; done
