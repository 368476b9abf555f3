"""Does the deferred verdicts' gain depend on where the frame pool lands?
One 32 Mi-entry 1-B verdict ring; K frame pools allocated one after another
(hipMalloc through gcl_dev_alloc, a growing spacer after every third, as
gcl_dev_alloc_paired steps past runs of one class); for every pool the udp64
classify kernel timed with per-packet verdict stores (gcl_tune.defer = 0) and
with the deferred batch writes (1), interleaved, plus the placement probe's
per-packet pattern over the same pair (gcl_access_probe).

    python tools/defer_place.py [pools]          one JSON line per pool
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
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl, n, stride, R, T, _ = bench.WORKLOADS["udp64"]
    vb = 1
    ring = g.DeviceBuffer(n * vb, 0)
    clfs = {}
    for f in (0, 1):
        fl, tb = bench.verdict_cfg(vb, R, T)
        # form 1: every default (deferred verdicts and the round-6 geometry)
        clfs[f] = g.Classifier(0, R, g.HASH_JENKINS, fl, thread_bits=tb, tune={"defer": 0} if f == 0 else {})
        bench.setup_tables(clfs[f], R, T)
    st = torch.cuda.current_stream().cuda_stream
    keep = []
    nsp = 0
    for i in range(k):
        if i and i % 3 == 0:
            keep.append(g.DeviceBuffer(n * stride * (2 << min(nsp, 3)), 0))
            nsp += 1
        pool = g.DeviceBuffer(n * stride, 0)
        bench.zero_fill(pool)
        g.generate(wl, n, stride, R, pool, seed=bench.SEED)
        torch.cuda.synchronize()
        row = {"pool": i, "spacers": nsp}
        for rnd in range(2):
            for f, clf in clfs.items():
                scratch = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)

                def go():
                    clf.classify(pool, n, stride, verdicts=ring, counts=scratch[:R], stats=scratch[R:], stream=st)
                _, ms = bench.timed_launches(go, 10)
                row.setdefault(f"defer{f}_us", []).append(round(ms * 1e3, 1))
        probe = bench.ceiling(clfs[1], pool, n, stride, ring, 0.33)
        row["kernel_shape_probe_us"] = round(probe.get("ceiling_ms", 0) * 1e3, 1)
        # the placement criterion (gcl_dev_alloc_paired): the minimal shape
        mp = bench.ceiling(clfs[0], pool, n, stride, ring, 0.33, minimal=True)
        row["access_probe_us"] = round(mp.get("ceiling_ms", 0) * 1e3, 1)
        print(json.dumps(row), flush=True)
        keep.append(pool)


if __name__ == "__main__":
    main()
