"""GENERAL-path kernel A/B over bench.py's own rows that take it: the
integrated ingress pool (random pool and working set, device-resident and
PCIe zero-copy; the JENKINS offsets-only row) and the pcap trace replay
(zero-copy), with GCL_TUNE_PAIR=0 (the LDS-tile classify_kernel) and =1
(classify_pair_kernel), alternating in one process.

    python tools/general_ab.py [rounds] > gpurun_out/general_ab.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(rounds=2):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for rnd in range(rounds):
        for pair in ("0", "1"):
            os.environ["GCL_TUNE_PAIR"] = pair
            ing = bench.ingress_pool_bench(dev, 2)
            tr = bench.trace_replay(dev)
            print(json.dumps({"round": rnd, "GCL_TUNE_PAIR": int(pair), "ingress_pool": ing,
                              "trace_replay": tr}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
