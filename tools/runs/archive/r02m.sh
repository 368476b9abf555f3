set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/udp64_v2_final_trace -o run -- python3 bench.py --no-secondary --no-e2e --no-cpu --steps 20 --warmup 5 > $O/udp64_v2_final_bench.json 2> $O/udp64_v2_final_trace.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tcp1500_v2_final_trace -o run -- python3 bench.py --workload tcp1500 --no-secondary --no-e2e --no-cpu --steps 20 --warmup 5 > $O/tcp1500_v2_final_bench.json 2> $O/tcp1500_v2_final_trace.err
echo rc=$?
