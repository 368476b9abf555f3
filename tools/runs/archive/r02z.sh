set -o pipefail
for wl in ingress_ws ingress_nic udp64; do
  WL=$wl OUT=gpurun_out/r02z timeout -k 10 600 bash tools/sqprof.sh > gpurun_out/r02z_$wl.log 2>&1 || exit $?
done
echo done
