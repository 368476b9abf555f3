# round 3: classify_pair_kernel (GCL_TUNE_PAIR) -- parity of every GENERAL
# test with it forced on, then the working-set / random-pool A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
GCL_TUNE_PAIR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_group.py > $O/tests_pair.log 2>&1 || { tail -40 $O/tests_pair.log; exit 1; }
tail -3 $O/tests_pair.log
timeout -k 10 400 python -u tools/ws_ab.py 3 pair=GCL_TUNE_PAIR:1 pair8=GCL_TUNE_PAIR:2 pair_abl=GCL_TUNE_PAIR:1,GCL_TUNE_ABLATE:128 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
cat $O/ws_ab.jsonl
echo done
