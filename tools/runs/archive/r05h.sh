# round 5: the deferred-verdict forms in three fresh processes (r05f: forms
# 1/2 321-322 us against 328-332; r05g on another box: all forms ~333)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05h_defer_ab.jsonl
: > $out
for p in 1 2 3; do
  AB_ROUNDS=3 AB_FORMS=0,1,3 timeout -k 10 200 python tools/defer_ab.py udp64 > gpurun_out/r05h_p$p.jsonl 2> gpurun_out/r05h_p$p.err || { tail -5 gpurun_out/r05h_p$p.err; exit 1; }
  sed "s/^{/{\"proc\": $p, /" gpurun_out/r05h_p$p.jsonl >> $out
done
cat $out
