"""bench.py's integrated ingress-pool leg alone (device-resident part), for
rocprofv3: 8 Mi descriptors into the reference's mbuf pool geometry with
ol_flags and hash.rss, GCL_HASH_NIC (classify_kernel<0, ...>), then the
JENKINS offsets-only row (classify_kernel<1, ...>).

    python tools/ingress_run.py [reps] [--nic-only | --ws-only] [--vbytes N]

--nic-only / --ws-only: the random-pool or the working-set NIC row alone, so
its classify_kernel<0, ...> launches are the only ones in a rocprof pass (both
rows launch the same kernel instance).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = (("nic",) if "--nic-only" in sys.argv else ("working_set",) if "--ws-only" in sys.argv
            else ("nic", "jenkins", "working_set"))
    vb = int(sys.argv[sys.argv.index("--vbytes") + 1]) if "--vbytes" in sys.argv else bench.INGRESS_VERDICT_BYTES
    print(json.dumps(bench.ingress_pool_bench(dev, vb, reps=reps, zerocopy=False,
                                              rows=rows)))
