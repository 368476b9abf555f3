# round 6: lean waves in the tile kernel (gcl_tune.tile_lean) -- the dense /
# probe / lean parity tests, the rx-loop suite (counts now ordered after the
# default stream's zeroing), then the tile_lean A/B on the bench's placed
# buffers in three fresh processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or probe or geometries or lean or ctx_tune or fuzz" > gpurun_out/r06d_tests.log 2>&1 || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -1 gpurun_out/r06d_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rxloop.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06d_rxloop.log 2>&1; rc=$?
tail -3 gpurun_out/r06d_rxloop.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3; do
  AB_KNOB=tile_lean timeout -k 10 300 python tools/tile_ab.py udp64 tcp1500 > gpurun_out/r06d_lean_ab_$i.jsonl 2> gpurun_out/r06d_lean_ab_$i.err || { tail -5 gpurun_out/r06d_lean_ab_$i.err; exit 1; }
  grep round gpurun_out/r06d_lean_ab_$i.jsonl | tail -2
done
echo r06d-done rxloop_rc=$rc
