set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
for a in 0 2 4 8 14 64; do
  GCL_TUNE_ABLATE=$a timeout -k 10 200 python -u tools/ingress_run.py 10 --ws-only > $O/ws_ablate$a.json 2> $O/ws_ablate$a.err || exit $?
done
echo done
