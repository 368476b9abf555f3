"""A/B of a classify_pair_kernel knob (AB_KNOB, default pair_lean: waves
whose packets are all plain IPv4 take classify_lean; pair_i32: the 32-bit
form) at forms 0 and 1 on bench.py's integrated
ingress row: the reference's 131072-mbuf pool (data at element + 344) placed
in HBM against the verdict ring, 8 Mi descriptors with ol_flags and
hash.rss, NIC mode, 2-B verdicts.  One context per form over the same
buffers, launches interleaved round by round; both forms' verdicts and
counts checked equal.  Also the working-set row (4096 mbufs).

    python tools/pair_lean_ab.py [rounds]        one JSON line per (row, round, form)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from caladan_amd import gclassify as g  # noqa: E402

KNOB = os.environ.get("AB_KNOB", "pair_lean")
# AB_FORMS: a JSON list of gcl_tune dicts instead (several knobs per form)
TUNES = json.loads(os.environ["AB_FORMS"]) if os.environ.get("AB_FORMS") else [{KNOB: 0}, {KNOB: 1}]


def pool(device, vb, cycles=64, P=g.IOKERNEL_NUM_MBUFS, ws=None):
    wl, _, _, R, T, _ = bench.WORKLOADS["udp64"]
    hdr = torch.zeros(P * 64, dtype=torch.uint8, device=device)
    olf_p = torch.zeros(P, dtype=torch.uint8, device=device)
    rss_p = torch.zeros(P, dtype=torch.int32, device=device)
    g.generate(wl, P, 64, R, hdr, olflags=olf_p, rss=rss_p, seed=bench.SEED)
    pool_offs = torch.from_numpy(g.mbuf_data_offsets(P).view(np.int64)).to(device)
    region = torch.zeros(g.mbuf_region_bytes(P), dtype=torch.uint8, device=device)
    region[(pool_offs[:, None] + torch.arange(64, device=device)).view(-1)] = hdr
    del hdr
    gen = torch.Generator(device="cpu").manual_seed(bench.SEED)
    m = P if ws is None else ws
    order = torch.cat([torch.randperm(m, generator=gen) for _ in range(cycles * P // m)]).to(device)
    offs, olf, rss = pool_offs[order].contiguous(), olf_p[order].contiguous(), rss_p[order].contiguous()
    n = offs.numel()
    dv = g.DeviceBuffer(n * vb, device.index or 0)
    placed = g.DeviceBuffer(region.numel(), device.index or 0, partner=dv, vbytes=vb)
    torch.cuda.synchronize()
    bench.hip_copy(placed, region, region.numel())
    del region
    return placed, dv, offs, olf, rss, n, R, T


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    vb = bench.INGRESS_VERDICT_BYTES
    st = torch.cuda.current_stream().cuda_stream
    for row, ws in (("random_pool", None), ("working_set", 4096)):
        region, dv, offs, olf, rss, n, R, T = pool(dev, vb, ws=ws)
        clfs = {}
        for f, tn in enumerate(TUNES):
            clfs[f] = bench.classifier(dev, R, T, vb, hash_mode=g.HASH_NIC)
            clfs[f].tune(**tn)
            bench.setup_tables(clfs[f], R, T)
        ref = None
        for f, clf in clfs.items():
            cnt = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)
            clf.classify(region, n, 0, verdicts=dv, counts=cnt[:R], stats=cnt[R:], offs=offs, olflags=olf,
                         rss=rss, stream=st)
            torch.cuda.synchronize()
            v = torch.empty(n * vb, dtype=torch.uint8)
            bench.hip_copy(v, dv, n * vb)
            got = (v.clone(), cnt.cpu().clone())
            ref = ref or got
            ok = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            print(json.dumps({"row": row, "form": f, "check": "ok" if ok else "MISMATCH"}), flush=True)
        for rnd in range(rounds):
            for f, clf in clfs.items():
                scratch = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)

                def go():
                    clf.classify(region, n, 0, verdicts=dv, counts=scratch[:R], stats=scratch[R:], offs=offs,
                                 olflags=olf, rss=rss, stream=st)
                _, ms = bench.timed_launches(go, 20)
                print(json.dumps({"row": row, "round": rnd, "form": f, "tune": TUNES[f],
                                  "kernel_us": round(ms * 1e3, 2),
                                  "gpkts": round(n / (ms * 1e-3) / 1e9, 2)}), flush=True)
        del region, dv, clfs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
