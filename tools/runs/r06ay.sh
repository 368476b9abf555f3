# round 6, the final tree: rocprofv3 passes (kernel trace + stats, then
# separate --pmc passes; 100 warm-up steps) of udp64, tcp1500, the ingress
# pool and its 4096-mbuf working set
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in "udp64 1" "tcp1500 2" "ingress_nic 2" "ingress_ws 2"; do
  set -- $wl
  ROUND=r06ay WLS=$1 VBS=$2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ay_prof_$1.log 2>&1 || { tail -5 gpurun_out/r06ay_prof_$1.log; exit 1; }
done
echo r06ay-done
