# what 1024 runtimes cost in the 1500-B shapes (slots and header split): kernel vs the
# compute-free ref, and without the histogram add / counter flush (timing-only ablations)
set -o pipefail
O=gpurun_out/r03ak
mkdir -p $O
CFGS="0:0:0:0:0:0:2 4:0:0:0:0:0:2 64:0:0:0:0:0:2 68:0:0:0:0:0:2 16:0:0:0:0:0:2"
for st in 1536 64; do
for R in 1024 16; do
  CBENCH_STRIDE=$st CBENCH_R=$R timeout -k 10 200 ./tools/cbench 1 40 $CFGS > $O/cb_${st}_${R}.jsonl 2> $O/cb_${st}_${R}.err || { cat $O/cb_${st}_${R}.err; exit 1; }
done
done
for f in $O/cb_*.jsonl; do echo $f; python3 -c "
import json,sys
for l in open('$f'.replace('\$f','')) if False else open(sys.argv[1]):
    d=json.loads(l); print('  ', d['cfg'], d.get('median_us', d.get('us')))" $f; done
