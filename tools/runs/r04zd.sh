# the dense-vstage parity test; the lone-burst stages and shallow rows with
# the NIC's hash.rss (RXPIPE_HASH=nic, rx.c:83) against the GPU's JENKINS
# hash, interleaved twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "vstage" > gpurun_out/r04zd_tests.log 2>&1 || { tail -30 gpurun_out/r04zd_tests.log; exit 1; }
tail -2 gpurun_out/r04zd_tests.log
for h in nic jenkins nic jenkins; do
  RXPIPE_HASH=$h bash tools/runs/r04c.sh r04zd_$h > /dev/null || exit 1
done
for h in nic jenkins; do echo "hash $h"; grep -h lone gpurun_out/r04zd_${h}_stages.jsonl | cut -c1-250; grep -h '"workers"' gpurun_out/r04zd_${h}_stages.jsonl | cut -c1-200; done
