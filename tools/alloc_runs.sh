#!/bin/bash
# tools/alloc_ab experiments behind profiles/archive/r01_alloc_placement.jsonl and
# r01_alloc_sweep_tlb.jsonl: $1 = default | cfirst | xcdmap | tlb
export TMPDIR=/tmp
O=gpurun_out/r01/alloc
mkdir -p $O
case "${1:-default}" in
default) timeout -k 10 200 ./tools/alloc_ab 20 > $O/alloc_ab.jsonl 2> $O/alloc_ab.err ;;
cfirst)  timeout -k 10 200 ./tools/alloc_ab 20 cfirst > $O/alloc_cfirst.jsonl 2> $O/alloc_cfirst.err ;;
xcdmap)  timeout -k 10 300 ./tools/alloc_ab 10 sweep 16 > $O/alloc_xcdmap.jsonl 2> $O/alloc_xcdmap.err ;;
tlb)     bash tools/tlb_run.sh ;;
*)       echo "usage: $0 default|cfirst|xcdmap|tlb" >&2; exit 2 ;;
esac
