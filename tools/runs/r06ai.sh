# round 6: the rocprofv3 passes of the final tree with 100 warm-up steps before
# the timed window (r06ah's trace timed dispatches 5-24, inside the ramp the
# first launches of a fresh process run: 305 -> 367 -> 330 us per dispatch)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r06ai WLS=udp64 VBS=1 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ai_prof_udp64.log 2>&1 || { tail -5 gpurun_out/r06ai_prof_udp64.log; exit 1; }
ROUND=r06ai WLS=tcp1500 VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ai_prof_tcp1500.log 2>&1 || { tail -5 gpurun_out/r06ai_prof_tcp1500.log; exit 1; }
ROUND=r06ai WLS=ingress_nic VBS=2 NO_CALIB=1 timeout -k 10 400 bash tools/profile.sh > gpurun_out/r06ai_prof_ingress.log 2>&1 || { tail -5 gpurun_out/r06ai_prof_ingress.log; exit 1; }
echo r06ai-done
