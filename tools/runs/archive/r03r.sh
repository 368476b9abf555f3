# round 3: plain-load pair kernel -- whole GPU suite, then the ingress rows'
# rocprof set (trace + PMC) on this build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ROUND=r03 WLS="ingress_nic ingress_ws" VBS="2" NO_CALIB=1 timeout -k 10 900 bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -1 $O/profile.log
