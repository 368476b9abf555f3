# round 5, the final tree: rocprofv3 (kernel trace/stats + separate PMC
# passes) of the two dominant launches (udp64 1-B, tcp1500 2-B), as r05i
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r05 WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r05zq_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r05zq_prof_udp64.log; exit 1; }
ROUND=r05 WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r05zq_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r05zq_prof_tcp1500.log; exit 1; }
echo r05zq-done
