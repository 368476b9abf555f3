"""A/B of one gcl_tune knob of the dense tile kernel on the bench's own
placed buffers, in one process: AB_KNOB (default tile_lean, the lean waves)
at each of AB_VALUES (default "0,1"), each beside its own ceiling --
gcl_access_probe in the kernel's shape (the same launch with rx_one_pkt
folded away) -- and the layout's minimal-request probe.  Contexts over the
same frames and verdict ring, launches interleaved round by round; every
form's verdicts and counts are checked against the first form's.  (Round 6's
first use, AB_KNOB=stage: block- against wave-staged tiles,
profiles/r06_stage_ab.jsonl; the wave form lost and was removed.)

    python tools/tile_ab.py [workload ...]     (default: udp64 tcp1500)
    AB_VBYTES (verdict bytes), AB_HASH (jenkins | toeplitz | nic)
One JSON line per (workload, round).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

KNOB = os.environ.get("AB_KNOB", "tile_lean")
FORMS = [int(x) for x in os.environ.get("AB_VALUES", "0,1").split(",")]
# AB_FORMS: a JSON list of gcl_tune dicts instead (several knobs per form)
TUNES = json.loads(os.environ["AB_FORMS"]) if os.environ.get("AB_FORMS") else None
if TUNES:
    KNOB = "form"
    FORMS = list(range(len(TUNES)))


def main():
    wls = sys.argv[1:] or ["udp64", "tcp1500"]
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("AB_REPS", "30"))
    for name in wls:
        vb = int(os.environ["AB_VBYTES"]) if os.environ.get("AB_VBYTES") else None
        w = bench.Workload(name, 0, 1, dev, vbytes=vb)
        hmode = {"jenkins": bench.g.HASH_JENKINS, "toeplitz": bench.g.HASH_TOEPLITZ,
                 "nic": bench.g.HASH_NIC}[os.environ.get("AB_HASH", "jenkins")]
        clfs = {}
        for f in FORMS:
            clfs[f] = bench.classifier(dev, w.R, w.T, w.vbytes, hash_mode=hmode)
            clfs[f].tune(**(TUNES[f] if TUNES else {KNOB: f}))
            bench.setup_tables(clfs[f], w.R, w.T)
        st = torch.cuda.current_stream().cuda_stream
        ref = None
        for f, clf in clfs.items():  # correctness: same verdicts and counts as form 0
            cnt = torch.zeros(w.R + bench.g.NR_STATS, dtype=torch.int64, device=dev)
            clf.classify(w.frames, w.n, w.stride, verdicts=w.verdicts, counts=cnt[:w.R], stats=cnt[w.R:],
                         stream=st)
            torch.cuda.synchronize()
            v = torch.empty(w.n * w.vbytes, dtype=torch.uint8)
            bench.hip_copy(v, w.verdicts, w.n * w.vbytes)
            got = (v.clone(), cnt.cpu().clone())
            if ref is None:
                ref = got
            ok = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            print(json.dumps({"workload": name, KNOB: f, **({"tune": TUNES[f]} if TUNES else {}),
                              "check": "ok" if ok else "MISMATCH"}), flush=True)
        out = torch.zeros(w.n * w.vbytes, dtype=torch.uint8, device=dev)
        alg = w.n * w.bytes_per_pkt
        for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
            row = {"workload": name, "round": rnd}
            for f, clf in clfs.items():
                scratch = torch.zeros(w.R + bench.g.NR_STATS, dtype=torch.int64, device=dev)

                def go():
                    clf.classify(w.frames, w.n, w.stride, verdicts=w.verdicts, counts=scratch[:w.R],
                                 stats=scratch[w.R:], stream=st)

                def probe():
                    clf.access_probe(w.frames, w.n, w.stride, out=out, stream=st)
                _, ms = bench.timed_launches(go, reps)
                _, pms = bench.timed_launches(probe, reps)
                row[f"{KNOB}={f}"] = {"kernel_us": round(ms * 1e3, 2), "frac": round(alg / (ms * 1e-3) / 8e12, 4),
                                    "probe_us": round(pms * 1e3, 2), "kernel_over_probe": round(ms / pms, 4)}
            _, mms = bench.timed_launches(
                lambda: clfs[FORMS[0]].access_probe(w.frames, w.n, w.stride, out=out, stream=st, minimal=True), reps)
            row["minimal_probe_us"] = round(mms * 1e3, 2)
            print(json.dumps(row), flush=True)
        del w, clfs, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
