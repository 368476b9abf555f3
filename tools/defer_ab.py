"""A/B of the dense tile kernel's verdict writes on the bench's own placed
buffers, in one process: stored per packet (gcl_tune.defer = 0) against kept
in LDS (and past a full buffer in registers) and written in at most two
batches per block (1, the default), or in as many as it takes (2).  Round
5's A/Bs also had an LDS-only form, since folded into 1
(profiles/r05_defer_ab.jsonl), and the batch writes through LDS, non-temporal
or plain (a VFLUSH knob, removed: no difference, r05_vflush_ab.jsonl).  One context per form
over the same frames and verdict ring, launches interleaved round by round;
every form's verdicts and counts are checked against form 0's.

    python tools/defer_ab.py [workload ...]     (default: udp64 tcp1500)
One JSON line per (workload, round, form).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

FORMS = {0: "per-packet stores", 1: "deferred, <= 2 writes per block", 2: "deferred always"}


def main():
    wls = sys.argv[1:] or ["udp64", "tcp1500"]
    dev = torch.device("cuda", 0)
    for name in wls:
        w = bench.Workload(name, 0, 1, dev)
        clfs = {}
        forms = [int(x) for x in os.environ.get("AB_FORMS", ",".join(map(str, FORMS))).split(",")]
        for f in forms:
            clfs[f] = bench.classifier(dev, w.R, w.T, w.vbytes)
            clfs[f].tune(defer=f)
            bench.setup_tables(clfs[f], w.R, w.T)
        st = torch.cuda.current_stream().cuda_stream
        ref = None
        for f, clf in clfs.items():  # correctness: same verdicts and counts as form 0
            cnt = torch.zeros(w.R + bench.g.NR_STATS, dtype=torch.int64, device=dev)
            w.verdicts_t = None
            clf.classify(w.frames, w.n, w.stride, verdicts=w.verdicts, counts=cnt[:w.R], stats=cnt[w.R:],
                         stream=st)
            torch.cuda.synchronize()
            v = torch.empty(w.n * w.vbytes, dtype=torch.uint8)
            bench.hip_copy(v, w.verdicts, w.n * w.vbytes)
            got = (v.clone(), cnt.cpu().clone())
            if ref is None:
                ref = got
            ok = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            print(json.dumps({"workload": name, "form": f, "check": "ok" if ok else "MISMATCH"}), flush=True)
        for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
            for f, clf in clfs.items():
                scratch = torch.zeros(w.R + bench.g.NR_STATS, dtype=torch.int64, device=dev)

                def go():
                    clf.classify(w.frames, w.n, w.stride, verdicts=w.verdicts, counts=scratch[:w.R],
                                 stats=scratch[w.R:], stream=st)
                _, ms = bench.timed_launches(go, 30)
                print(json.dumps({"workload": name, "round": rnd, "form": f, "what": FORMS[f],
                                  "kernel_us": round(ms * 1e3, 2),
                                  "frac": round(w.n * w.bytes_per_pkt / (ms * 1e-3) / 8e12, 4)}), flush=True)
        del w, clfs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
