# round 5: rocprofv3 of the integrated ingress row on the final tree (the
# pair kernel's lean waves): kernel trace/stats + PMC passes
set -o pipefail
mkdir -p gpurun_out
ROUND=r05 WLS=ingress_nic VBS=2 NO_CALIB=1 timeout -k 10 500 bash tools/profile.sh > gpurun_out/r05q_prof_ingress.log 2>&1 || { tail -5 gpurun_out/r05q_prof_ingress.log; exit 1; }
tail -1 gpurun_out/r05q_prof_ingress.log
