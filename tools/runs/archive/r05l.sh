# round 5: the deferred verdicts' batch writes -- the registers written
# directly or through the LDS buffer 16 B per lane, and the batch stores
# write-through (sc0 sc1), nt or plain -- parity of the variants, then the
# A/B in three fresh processes
set -o pipefail
mkdir -p gpurun_out
for v in 1 2 3 5; do
  GCL_TUNE_VFLUSH=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deferred_flushes or narrow" > gpurun_out/r05l_tests_v$v.log 2>&1 || { tail -30 gpurun_out/r05l_tests_v$v.log; exit 1; }
  tail -1 gpurun_out/r05l_tests_v$v.log
done
out=gpurun_out/r05l_vflush_ab.jsonl
: > $out
for p in 1 2 3; do
  AB_ROUNDS=3 AB_FORMS=0,1,11,12,13,14,15 timeout -k 10 300 python tools/defer_ab.py udp64 > gpurun_out/r05l_p$p.jsonl 2> gpurun_out/r05l_p$p.err || { tail -5 gpurun_out/r05l_p$p.err; exit 1; }
  sed "s/^{/{\"proc\": $p, /" gpurun_out/r05l_p$p.jsonl >> $out
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r05l_vflush_ab.jsonl"):
    r = json.loads(l)
    if "kernel_us" in r:
        d[(r["form"], r["what"])].append(r["kernel_us"])
for k, v in sorted(d.items()):
    print(k, min(v), sorted(v)[len(v) // 2], max(v))
PY
