# round 3: pair kernel specialised on the 2-byte verdict: parity (GENERAL
# tests), working-set A/B, rxpipe inline rows, and the one-rank nccl Exchange
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ws_ab.py 3 pair_abl=GCL_TUNE_ABLATE:128 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ws_ab.jsonl'):
    r=json.loads(l); d[(r['set'],r['row'])].append((r['kernel_us'], r.get('verdicts_match_default')))
for k,v in sorted(d.items()): print(k, v)
"
for cfg in "64 8 16 40000 inline" "64 16 32 40000 inline" "64 16 32 40000"; do
  timeout -k 10 120 ./tools/rxpipe $cfg >> $O/rxpipe.jsonl 2>> $O/rxpipe.err || { cat $O/rxpipe.err; exit 1; }
done
cat $O/rxpipe.jsonl
timeout -k 10 300 python -u bench.py --force-exchange --steps 20 --warmup 5 --no-secondary --no-e2e --no-cpu > $O/bench_fx.json 2> $O/bench_fx.err || { tail $O/bench_fx.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_fx.json').read().strip().splitlines()[-1])
print(d['value'], d['counts_check'], d.get('exchange'), d['config']['parallelism'], d['group'])"
echo done
