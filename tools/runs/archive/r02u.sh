set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
export TMPDIR=/tmp
ROUND=r02 WLS="ingress_nic" VBS="2" NO_CALIB=1 timeout -k 10 900 bash tools/profile.sh > $O/profile.log 2>&1
echo rc=$?
