# round 3: the pair kernel as the GENERAL default -- the whole GPU suite, then
# the working-set A/B and bench's GENERAL rows
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/ws_ab.py 3 pair_abl=GCL_TUNE_ABLATE:128 > $O/ws_ab.jsonl 2> $O/ws_ab.err || { tail $O/ws_ab.err; exit 1; }
timeout -k 10 600 python -u tools/general_ab.py 2 > $O/general_ab.jsonl 2> $O/general_ab.err || { tail $O/general_ab.err; exit 1; }
echo done
