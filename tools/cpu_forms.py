"""The CPU baseline's three loop forms on one pinned core, interleaved: is the
mixed stream's classify + lrpc_send faster than classify alone (VERDICT r04
Weak 9) a property of the loop, or noise?

  classify   classify_range_direct: rx_one_pkt (direct header loads) per mbuf
  lrpc       classify_range_lrpc: the same + rx_make_cmd + flow_tbl[slot]
             + lrpc_send into 4096-deep rings (rx.c:76-92)
  nosend     the lrpc loop without the ring write (ORC_BENCH_NOSEND)

    python tools/cpu_forms.py [reps]      one JSON line per (stream, mode, rep)
Test infrastructure (imports oracle/); runs on the GPU box's host cores.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from caladan_amd import gclassify as g  # noqa: E402
from oracle import orc  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    orc.build(native=True)
    cpu = bench.pick_cores(1)
    for name, (n, _) in bench.CPU_STREAMS.items():
        wl, _, stride, R, T, _ = bench.WORKLOADS[name]
        cdf = orc.zipf_cdf(bench.ZIPF_FLOWS) if wl == g.WL_TCP1500_ZIPF else None
        pkt_len = np.zeros(n, dtype=np.uint16)
        frames, olf, rss = orc.generate(wl, n, stride, R, seed=bench.SEED, native=True, cdf=cdf,
                                        pkt_len=pkt_len)
        for mname, mode in (("nic", g.HASH_NIC), ("jenkins", g.HASH_JENKINS)):
            t = orc.Tables(R, mode, 0, g.F_RSS_HASH | g.F_IP_CKSUM_GOOD, native=True)
            rng = np.random.default_rng(bench.SEED)
            for r in range(R):
                act = int(rng.integers(1, T + 1))
                idx = [int(x) for x in rng.choice(T, size=act, replace=False)]
                t.runtime_set(r, orc.runtime_ip(r), T, act, orc.steer_flows(T, idx))
            kw = dict(olflags=olf, rss=rss, pkt_len=pkt_len, direct=True, cpus=cpu)
            probe = t.bench(frames, n, stride, threads=1, passes=1, **kw)
            passes = max(1, int(0.5 / max(probe, 1e-6)))
            for rep in range(reps):
                row = {"stream": name, "mode": mname, "rep": rep, "cpu": cpu[0], "passes": passes}
                for form, extra in (("classify", {}), ("lrpc", {"lrpc": True}), ("nosend", {"nosend": True})):
                    s = t.bench(frames, n, stride, threads=1, passes=passes, **kw, **extra)
                    row[form + "_mpps"] = round(n * passes / s / 1e6, 2)
                print(json.dumps(row), flush=True)
        del frames


if __name__ == "__main__":
    main()
