# GCL_CFG_VERDICT1: the 1-byte queue verdict's GPU tests, then the headline
# udp64 line with 1- and 2-byte verdicts in alternating fresh processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rxloop.py -x -q --timeout 120 --timeout-method thread -k "verdict1 or fuzz_vs_oracle or post_pass or bench_format" > gpurun_out/r04y_tests.log 2>&1 || { tail -30 gpurun_out/r04y_tests.log; exit 1; }
tail -2 gpurun_out/r04y_tests.log
for rep in 1 2; do
  for vb in 1 2; do
    timeout -k 10 200 python bench.py --verdict-bytes $vb --no-secondary --no-e2e --no-cpu --no-group > gpurun_out/r04y_bench_v${vb}_$rep.json 2> gpurun_out/r04y_bench_v${vb}_$rep.err || { tail -5 gpurun_out/r04y_bench_v${vb}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r04y_bench_v${vb}_$rep.json').read().strip().splitlines()[-1]); print($vb, d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline'].get('frac_of_ceiling'), d['placement']['kernel_checks'])"
  done
done
