"""bench.py's rx loop latency leg alone (e2e.rxloop): burst latency of the
persistent loop at 64..1024-packet bursts, one fresh process per call (the
staggered-poller knobs it once compared are gone from the library,
profiles/archive/r02_loop_pollers_ab.jsonl).

    python tools/rxloop_run.py [iters]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = bench.rxloop_bench(dev, bench.VERDICT_BYTES, iters=iters)
    print(json.dumps(out))
