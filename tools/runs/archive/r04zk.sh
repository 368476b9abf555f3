# final-tree rocprofv3 evidence: kernel-trace/stats and separate PMC passes
# of the udp64 launch with 1-B verdicts (the headline) and tcp1500 with 2-B
set -o pipefail
export TMPDIR=/tmp
NO_CALIB=1 ROUND=r04z WLS="udp64" VBS="1" timeout -k 10 600 bash tools/profile.sh > gpurun_out/r04zk_profile_a.log 2>&1 || { tail -20 gpurun_out/r04zk_profile_a.log; exit 1; }
NO_CALIB=1 ROUND=r04z WLS="tcp1500" VBS="2" timeout -k 10 600 bash tools/profile.sh > gpurun_out/r04zk_profile_b.log 2>&1 || { tail -20 gpurun_out/r04zk_profile_b.log; exit 1; }
tail -1 gpurun_out/r04zk_profile_b.log
