"""What bounds classify over the reference's ingress mbuf pool?

bench.py's `ingress_pool` line classifies 8 Mi descriptors that point at
random mbufs of the 131072-mbuf pool (9408-B elements, data at element + 344;
iokernel/defs.h:503-523), device-resident.  This runs the same kernel over the
same region with the descriptor order and the pool size varied, one process,
interleaved, so the difference between the rows is the access pattern alone:

  random     random permutations of the whole pool (the bench line)
  pool       the pool in address order, 64 times (sequential mbufs)
  sub16k     random over the first 16384 mbufs (154 MB, fits the MALL)
  sub1k      random over the first 1024 mbufs (9.6 MB, fits L2)
  *_a16      the same, frames at element + 336 (16-B aligned loads)

    python tools/ingress_ab.py > gpurun_out/ingress_ab.jsonl
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bench import SEED, WORKLOADS, classifier, g, setup_tables  # noqa: E402


def main(cycles=64, reps=10, rounds=3):
    dev = torch.device("cuda", 0)
    wl, _, _, R, T, _ = WORKLOADS["udp64"]
    P = g.IOKERNEL_NUM_MBUFS
    hdr = torch.zeros(P * 64, dtype=torch.uint8, device=dev)
    g.generate(wl, P, 64, R, hdr, seed=SEED)
    pool_offs = torch.from_numpy(g.mbuf_data_offsets(P).view(np.int64)).to(dev)
    region = torch.zeros(g.mbuf_region_bytes(P), dtype=torch.uint8, device=dev)
    region[(pool_offs[:, None] + torch.arange(64, device=dev)).view(-1)] = hdr
    # the same frames 8 bytes earlier (element + 336): 16-B aligned
    region16 = torch.zeros_like(region)
    region16[(pool_offs[:, None] - 8 + torch.arange(64, device=dev)).view(-1)] = hdr
    del hdr
    gen = torch.Generator(device="cpu").manual_seed(SEED)
    n = P * cycles
    orders = {
        "random": torch.cat([torch.randperm(P, generator=gen) for _ in range(cycles)]),
        "pool": torch.arange(P).repeat(cycles),
        "sub16k": torch.randint(0, 16384, (n,), generator=gen),
        "sub1k": torch.randint(0, 1024, (n,), generator=gen),
    }
    offs = {k: (region, pool_offs[v.to(dev)].contiguous()) for k, v in orders.items()}
    for k in ("random", "sub1k"):
        offs[k + "_a16"] = (region16, offs[k][1] - 8)
    clf = classifier(dev, R, T, 4)
    setup_tables(clf, R, T)
    cnt = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)
    dv = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {k: [] for k in offs}
    for rnd in range(rounds):
        for k, (reg, o) in offs.items():
            clf.classify(reg, n, 0, verdicts=dv, counts=cnt[:R], stats=cnt[R:], offs=o, stream=st)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                clf.classify(reg, n, 0, verdicts=dv, counts=cnt[:R], stats=cnt[R:], offs=o,
                             stream=st)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / reps)
    for k, ts in res.items():
        t = min(ts)
        print(json.dumps({"order": k, "pkts": n, "us": round(t * 1e6, 1),
                          "gpkt_s": round(n / t / 1e9, 2),
                          "all_us": [round(x * 1e6, 1) for x in ts]}), flush=True)


if __name__ == "__main__":
    bench.log = lambda *a, **k: None
    main()
