# Diagnostic: udp64 step rate over ~25 s next to the DPM levels and power
# the driver exposes read-only in sysfs (tools/modes_probe.py).
set -o pipefail
O=gpurun_out/r02bf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/modes_probe.py > $O/modes.jsonl 2> $O/modes.err || exit $?
echo rc=0
