"""What bounds the GENERAL classify path on the cache-resident working-set row
(bench.py e2e.ingress_pool.integrated_nic_working_set)?

The same 8 Mi descriptors (offs + ol_flags + hash.rss, NIC mode, 2-byte
verdicts) drawn from a 4096-mbuf working set of the reference's ingress pool
geometry (9408-B elements, data at element + 344), classified by contexts
opened with different GCL_TUNE_* knobs, one process, interleaved rounds:

  default            the library default (the lane-pair kernel since round 3)
  tile               GCL_TUNE_PAIR=0: the LDS-tile classify_kernel
  loads_only         GCL_TUNE_ABLATE=16 (tile kernel): offsets, side loads,
                     header windows and LDS staging; no classification
  no_lookups         GCL_TUNE_ABLATE=2|4|8: no IP lookup, histogram, flow_tbl
  no_flush           GCL_TUNE_ABLATE=64: no counter flush at the end
  extra rows from argv as name=ENV:VAL,ENV:VAL

Timing-only rows (ablations) give wrong verdicts on purpose.

    python tools/ws_ab.py [rounds] > gpurun_out/ws_ab.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import SEED, WORKLOADS, g, setup_tables, timed_launches  # noqa: E402

ROWS = [("default", {}), ("tile", {"GCL_TUNE_PAIR": "0"}), ("loads_only", {"GCL_TUNE_ABLATE": "16"}),
        ("no_lookups", {"GCL_TUNE_ABLATE": "14"}), ("no_flush", {"GCL_TUNE_ABLATE": "64"})]


def main(rounds=3, extra=()):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl, _, _, R, T, _ = WORKLOADS["udp64"]
    P, ws, n = g.IOKERNEL_NUM_MBUFS, 4096, 8 << 20
    hdr = torch.zeros(P * 64, dtype=torch.uint8, device=dev)
    olf_p = torch.zeros(P, dtype=torch.uint8, device=dev)
    rss_p = torch.zeros(P, dtype=torch.int32, device=dev)
    g.generate(wl, P, 64, R, hdr, olflags=olf_p, rss=rss_p, seed=SEED)
    pool_offs = torch.from_numpy(g.mbuf_data_offsets(P).view(np.int64)).to(dev)
    region = torch.zeros(g.mbuf_region_bytes(P), dtype=torch.uint8, device=dev)
    region[(pool_offs[:, None] + torch.arange(64, device=dev)).view(-1)] = hdr
    gen = torch.Generator(device="cpu").manual_seed(SEED)
    sub = torch.randperm(P, generator=gen)[:ws]
    order = torch.cat([sub[torch.randperm(ws, generator=gen)] for _ in range(n // ws)]).to(dev)
    offs, olf, rss = pool_offs[order].contiguous(), olf_p[order].contiguous(), rss_p[order].contiguous()
    # the bench's random-pool row too: 64 random permutations of the whole pool
    order_r = torch.cat([torch.randperm(P, generator=gen) for _ in range(n // P)]).to(dev)
    sets = {"ws": (offs, olf, rss),
            "random": (pool_offs[order_r].contiguous(), olf_p[order_r].contiguous(),
                       rss_p[order_r].contiguous())}
    dv = torch.empty(n * 2, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    rows = list(ROWS) + [(name, dict(kv.split(":") for kv in spec.split(",")))
                         for name, spec in (e.split("=", 1) for e in extra)]
    clfs = {}
    for name, env in rows:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            clf = g.Classifier(0, R, g.HASH_NIC, g.CFG_VERDICT2, thread_bits=3)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        setup_tables(clf, R, T)
        clfs[name] = clf
    ref = None
    for rnd in range(rounds):
        for ds, (o_, f_, r_) in sets.items():
            for name, _ in rows:
                clf = clfs[name]

                def step():
                    clf.classify(region, n, 0, verdicts=dv, counts=cnt[:R], stats=cnt[R:], offs=o_,
                                 olflags=f_, rss=r_, stream=st)
                wall, gms = timed_launches(step, 10)
                rec = {"round": rnd, "set": ds, "row": name, "kernel_us": round(gms * 1e3, 2),
                       "gpkt_s": round(n / (gms * 1e-3) / 1e9, 2)}
                if "GCL_TUNE_ABLATE" not in dict(rows)[name]:
                    # every non-ablated row must write the default row's verdicts
                    torch.cuda.synchronize()
                    h = int(dv.view(torch.int16).to(torch.int64).sum().item())
                    if name == "default":
                        ref = h
                    rec["verdicts_match_default"] = h == ref
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    r = int(args.pop(0)) if args and args[0].isdigit() else 3
    main(r, args)
