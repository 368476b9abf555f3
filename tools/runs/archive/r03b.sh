# round 3: rxloop peek tests, full-size bench-format tests, the burst-64
# pipeline rows, the CPU baseline (lazy lrpc consumers), and trace passes
# whose timed dispatches reproduce the bench line's roofline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rxloop.py "tests/test_gpu_parity.py::test_gpu_full_size_bench_format" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for cfg in "64 1 1 20000" "64 4 8 20000" "64 4 8 20000 copy" "64 8 16 40000" "64 16 32 40000" \
           "64 16 64 40000" "256 4 8 10000" "1024 8 16 4000"; do
  timeout -k 10 120 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
cat $O/rxpipe.jsonl
timeout -k 10 200 python -u -c "import bench, json; print(json.dumps(bench.cpu_baseline(12.0)))" > $O/cpu.json 2> $O/cpu.err || { tail $O/cpu.err; exit 1; }
cat $O/cpu.json
for wl in udp64 tcp1500; do
  D=gpurun_out/prof_r03/${wl}_v2
  mkdir -p gpurun_out/prof_r03
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${D}_trace -o run -- python3 bench.py --workload $wl --verdict-bytes 2 --no-cpu --no-secondary --no-e2e --no-group --steps 20 --warmup 1 > ${D}_bench.json 2> ${D}_trace.err || { tail ${D}_trace.err; exit 1; }
done
echo done
