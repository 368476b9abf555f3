set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
export TMPDIR=/tmp
GCL_TUNE_WSLOT=16:2048:256 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fuzz or full_size or workloads or edge or ingress or scenarios" > $O/pytest_wslot.log 2>&1 &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 0 20 0:0:0:0:0:0:2:2 "0:0:0:0:0:0:2:2@16/2048/256" "0:0:0:0:0:0:2:2@16/4096/512" "0:0:0:0:0:0:2:2@8/1024/128" "0:0:0:0:0:0:2:2@16/1000000000/0" "0:0:0:0:0:0:2:0@16/2048/256" "0:0:0:0:0:0:1:2" "0:0:0:0:0:0:1:2@8/2048/256" > $O/cb_udp64_wslot.jsonl 2> $O/cb_udp64_wslot.err &&
CBENCH_PROFILE=0 CBENCH_PAIRED=1 timeout -k 10 300 ./tools/cbench 1 20 0:0:0:0:0:0:2:2 "0:0:0:0:0:0:2:2@8/2048/256" "0:0:0:0:0:0:2:2@8/4096/512" > $O/cb_tcp1500_wslot.jsonl 2> $O/cb_tcp1500_wslot.err
echo rc=$?
