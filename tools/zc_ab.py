"""Frames in pinned host memory, read zero-copy over PCIe (bench.py's e2e
udp64 and mixed-jumbo rows): the dense tile kernel (64-B windows, streaming
loads; the default for fixed-slot batches) against the GENERAL lane-pair
kernel (bytes [8, 40) per packet, plain loads; GCL_TUNE_GENERAL=1),
alternating in one process.

    python tools/zc_ab.py [rounds] > gpurun_out/zc_ab.jsonl
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import SEED, WORKLOADS, classifier, g, setup_tables  # noqa: E402


def main(rounds=3, reps=3):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name, n in (("udp64", 32 << 20), ("mixed", 256 << 10)):
        wl, _, stride, R, T, _ = WORKLOADS[name]
        dfr = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        g.generate(wl, n, stride, R, dfr, seed=SEED)
        hfr = torch.empty(n * stride, dtype=torch.uint8).pin_memory()
        hfr.copy_(dfr)
        del dfr
        hv = {v: torch.empty(n * 2, dtype=torch.uint8).pin_memory() for v in ("dense", "general")}
        clfs = {}
        for v in ("dense", "general"):
            os.environ["GCL_TUNE_GENERAL"] = "1" if v == "general" else "0"
            clfs[v] = classifier(dev, R, T, 2)
            setup_tables(clfs[v], R, T)
        os.environ.pop("GCL_TUNE_GENERAL", None)
        for rnd in range(rounds):
            for v in ("dense", "general"):
                clf = clfs[v]
                clf.classify_host(hfr, n, stride, verdicts=hv[v], mode=g.E2E_ZEROCOPY, nstreams=1)
                t0 = time.perf_counter()
                for _ in range(reps):
                    clf.classify_host(hfr, n, stride, verdicts=hv[v], mode=g.E2E_ZEROCOPY, nstreams=1)
                dt = (time.perf_counter() - t0) / reps
                print(json.dumps({"round": rnd, "set": name, "kernel": v,
                                  "zerocopy_mpps": round(n / dt / 1e6, 1),
                                  "verdicts_match": bool(torch.equal(hv["dense"], hv[v]))}), flush=True)
        del hfr, hv, clfs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
