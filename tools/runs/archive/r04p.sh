# round-4 rocprof evidence: kernel-trace/stats and PMC passes of the udp64,
# tcp1500 and integrated-ingress classify launches (2-B verdicts)
set -o pipefail
export TMPDIR=/tmp
NO_CALIB=1 ROUND=r04 WLS="udp64 tcp1500 ingress_nic" VBS="2" timeout -k 10 900 bash tools/profile.sh > gpurun_out/r04p_profile.log 2>&1 || { tail -20 gpurun_out/r04p_profile.log; exit 1; }
tail -3 gpurun_out/r04p_profile.log
