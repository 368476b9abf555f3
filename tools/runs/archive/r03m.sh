# round 3: the whole GPU suite after the quad kernel's removal (new edge tests included)
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
