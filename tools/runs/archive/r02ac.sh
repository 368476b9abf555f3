# A/B of kernel builds (tools/_ab/libgclassify_<variant>.so, a trailing 2
# reruns the variant; VARIANTS picks them, default new / old / new2), each running the ingress rows (random pool + working set) and the
# tcp1500 / udp64 kernel-only bench lines in a fresh process.
set -o pipefail
O=gpurun_out/r02ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
for v in ${VARIANTS:-new old new2}; do
  src=tools/_ab/libgclassify_${v%2}.so
  cp $src caladan_amd/libgclassify.so || exit 1
  timeout -k 10 240 python3 tools/ingress_run.py 10 > $O/ingress_$v.json 2> $O/ingress_$v.err || exit $?
  for wl in tcp1500 udp64; do
    timeout -k 10 240 python3 bench.py --workload $wl --no-cpu --no-secondary --no-e2e --steps 200 --warmup 20 > $O/bench_${wl}_$v.json 2> $O/bench_${wl}_$v.err || exit $?
  done
done
cp tools/_ab/libgclassify_new.so caladan_amd/libgclassify.so
echo done
