# rx loop tests (with the soak test) and a long soak: 10 M bursts per configuration
set -o pipefail
O=gpurun_out/r03am
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rxloop.py > $O/test_rxloop.log 2>&1 || { tail -30 $O/test_rxloop.log; exit 1; }
tail -1 $O/test_rxloop.log
for cfg in "3000000 1 2 1" "10000000 4 4 4" "10000000 3 8 8" "10000000 16 16 16" "10000000 32 64 64" "10000000 64 64 64"; do
  timeout -k 10 240 ./tools/loopsoak $cfg | tee -a $O/soak.jsonl || exit 1
done
