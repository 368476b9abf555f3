"""Summarise tools/sqprof.sh's SQ counter passes for one workload into
per-packet and per-wave instruction counts of the classify kernel.

    python tools/sq_summary.py gpurun_out/sq_r03 ingress_ws [kernel-substring] > profiles/...json

Counters are summed over every dispatch of the kernel in each pass (SQ_* are
already chip-wide sums per dispatch) and divided by the dispatch count, then
by the packets per launch.  SQ_WAVES counts waves launched; the per-wave
figures divide by it.  Cycle counters (SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, the
SQ_ACTIVE_INST_* and SQ_WAIT_* families) are in the units rocprofv3 reports
them for gfx950 (per-SE/agent sums), so they are given as ratios to
SQ_WAVE_CYCLES rather than as absolute times.
"""
import csv
import json
import os
import sys

PKTS = {"udp64": 32 << 20, "tcp1500": 8 << 20, "ingress_nic": 8 << 20, "ingress_ws": 8 << 20}
KNAME = {"ingress_nic": "_kernel<0,", "ingress_ws": "_kernel<0,"}  # classify_kernel or classify_pair_kernel, NIC mode


def main(base, wl, kname=None):
    kname = kname or KNAME.get(wl, "classify_kernel")
    per = {}
    for g in range(1, 10):
        path = os.path.join(base, f"{wl}_g{g}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        disp = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                if kname not in r["Kernel_Name"].replace(" ", ""):
                    continue
                disp.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for c in {k for d in disp.values() for k in d}:
            vals = [d[c] for d in disp.values() if c in d]
            per[c] = sum(vals) / len(vals)
    n = PKTS[wl]
    waves = per.get("SQ_WAVES", 0) or 1
    out = {"workload": wl, "kernel": kname, "pkts_per_launch": n, "waves_per_launch": waves,
           "per_launch": per,
           "per_pkt": {c: round(v / n, 4) for c, v in per.items() if c.startswith("SQ_INSTS")},
           "per_wave": {c: round(v / waves, 2) for c, v in per.items() if c.startswith("SQ_INSTS")}}
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        out["over_wave_cycles"] = {c: round(v / wc, 4) for c, v in per.items()
                                   if c.startswith(("SQ_ACTIVE", "SQ_WAIT", "SQ_INST_CYCLES"))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
