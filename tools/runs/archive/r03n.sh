# round 3: the rocprof set on the round-3 build -- kernel trace/stats (timed
# dispatches) and PMC passes for udp64, tcp1500 and both ingress rows
set -o pipefail
export TMPDIR=/tmp
ROUND=r03 WLS="udp64 tcp1500 ingress_nic ingress_ws" VBS="2" NO_CALIB=1 timeout -k 10 1100 bash tools/profile.sh > gpurun_out/r03n_profile.log 2>&1 || { tail -20 gpurun_out/r03n_profile.log; exit 1; }
tail -2 gpurun_out/r03n_profile.log
