"""Does a placed udp64 pair stay in its class over a run?  One Workload
(bench.py, placement checked), then 300 classify launches each bracketed by
its own HIP event pair; prints the per-launch times in groups of 20 (median,
min, max), then the same for the bench's timed loop shape (50 back-to-back
launches, one event pair), three times.

    python tools/drift.py [vbytes] [launches] [group]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    vb = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nl = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    grp = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.Workload("udp64", 0, 1, dev, vbytes=vb)
    print(json.dumps({"placement": bench.placement(w)}), flush=True)
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nl)]
    for a, b in ev:
        a.record(st)
        w.step(st.cuda_stream)
        b.record(st)
    torch.cuda.synchronize()
    us = np.array([a.elapsed_time(b) * 1e3 for a, b in ev])
    for i in range(0, nl, grp):
        g = us[i:i + grp]
        print(json.dumps({"launches": [i, i + grp], "median_us": round(float(np.median(g)), 1),
                          "min_us": round(float(g.min()), 1), "max_us": round(float(g.max()), 1)}),
              flush=True)
    for k in range(3):
        el, gms = bench.run_timed(w, 50, 5, 1)
        print(json.dumps({"bench_loop": k, "gpu_us_per_step": round(gms * 1e3, 1),
                          "wall_us_per_step": round(el / 50 * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
