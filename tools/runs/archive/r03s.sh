set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python -u tools/zc_ab.py 3 > $O/zc_ab.jsonl 2> $O/zc_ab.err || { tail $O/zc_ab.err; exit 1; }
cat $O/zc_ab.jsonl
