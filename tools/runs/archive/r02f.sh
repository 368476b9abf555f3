set -o pipefail
O=gpurun_out/r02f; mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python -u bench.py --no-secondary --no-e2e --no-cpu > $O/b$i.json 2> $O/b$i.err || exit $?
done
echo done
