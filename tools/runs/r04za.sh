# A/Bs: (1) dense verdicts staged in LDS and stored as whole lines
# (GCL_TUNE_VSTAGE) against per-wave stores, write-through and plain, on the
# udp64 headline (1-B verdicts), alternating fresh processes, after parity
# tests with the knob on; (2) header records submitted by non-temporal
# stores (GCL_TUNE_LOOP_NT) in the lone-burst stages and shallow rows
set -o pipefail
mkdir -p gpurun_out
GCL_TUNE_VSTAGE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "verdict1 or fuzz_vs_oracle or bench_format or edge_sizes" > gpurun_out/r04za_tests.log 2>&1 || { tail -30 gpurun_out/r04za_tests.log; exit 1; }
tail -2 gpurun_out/r04za_tests.log
for rep in 1 2; do
  for cfg in "0 2" "1 2" "0 0" "1 0"; do
    set -- $cfg
    GCL_TUNE_VSTAGE=$1 GCL_TUNE_NT_STORE=$2 timeout -k 10 200 python bench.py --verdict-bytes 1 --no-secondary --no-e2e --no-cpu --no-group > gpurun_out/r04za_v$1_s$2_$rep.json 2> gpurun_out/r04za_v$1_s$2_$rep.err || { tail -5 gpurun_out/r04za_v$1_s$2_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r04za_v$1_s$2_$rep.json').read().strip().splitlines()[-1]); print('vstage $1 store $2', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline'].get('frac_of_ceiling'), [c['kernel_us'] for c in d['placement']['kernel_checks']])"
  done
done
for nt in 0 1 0 1; do
  GCL_TUNE_LOOP_NT=$nt bash tools/runs/r04c.sh r04za_nt$nt > /dev/null || exit 1
done
for nt in 0 1; do echo "loop nt $nt"; grep -h lone gpurun_out/r04za_nt${nt}_stages.jsonl | cut -c1-300; grep -h '"workers"' gpurun_out/r04za_nt${nt}_stages.jsonl | cut -c1-200; done
