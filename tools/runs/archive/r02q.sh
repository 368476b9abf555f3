set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 200 python -u tools/ingress_run.py 10 > $O/ingress.json 2> $O/ingress.err &&
timeout -k 10 200 ./tools/gather 10 > $O/gather.jsonl 2> $O/gather.err
echo rc=$?
