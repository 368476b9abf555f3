"""Does gcl_dev_alloc_paired's probe predict the classify kernel's class?

Repeats, in one process: a 4-B verdict ring, a 2 GiB udp64 frame pool placed
against it (gcl_dev_alloc_paired), the frames generated, then the classify
kernel timed over the pair (HIP events around 20 launches).  A spacer of a
varying size is held between trials so each lands somewhere else.  Prints one
JSON line per trial: the probe's verdict next to the kernel's time.

    python tools/pair_check.py [trials]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from caladan_amd import gclassify as g  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spacers = []
    for k in range(trials):
        w = bench.Workload("udp64", 0, 1, dev, vbytes=4)
        st = torch.cuda.current_stream()
        for _ in range(3):
            w.step(st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(3):
            e0.record(st)
            for _ in range(20):
                w.step(st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        print(json.dumps({"trial": k, "classify_us": round(sorted(ts)[1], 2),
                          "placement": w.frames.pair_info}), flush=True)
        del w
        torch.cuda.empty_cache()
        spacers.append(g.DeviceBuffer((1 + k % 3) << 30))


if __name__ == "__main__":
    main()
