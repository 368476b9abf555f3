"""Generate tests/golden/struct_frames_ref.npz: frames written through the
REFERENCE's own inc/net structs (struct eth_hdr / ip_hdr / udp_hdr / tcp_hdr /
arp_hdr, inc/net/ip.h:59-81 and friends, exported by oracle/ref_host.c into
oracle/_ref/libhost_ref.so) with the expected classification of each one: the
runtime owning the destination (daddr, or the ARP target IP) and the JENKINS
flow hash of the values put into the structs, computed by the reference's own
base/jenkins_hash.c (oracle/_ref/libjhash_ref.so).

The GPU test (test_gpu_reference_struct_frames) reads this fixture, so the
GPU box never loads a library built from reference sources.

Run where /root/reference exists (after `make -C oracle ref`):
    python tests/golden/make_struct_frames.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import orc  # noqa: E402
from tests.rxcases import ref_struct_batch  # noqa: E402

OUT = os.path.join(HERE, "struct_frames_ref.npz")
SEED, R, N = 17, 64, 3000


def main():
    ref, rj = orc.ref_host(), orc.ref_jhash()
    if ref is None or rj is None:
        raise SystemExit("oracle/_ref/libhost_ref.so / libjhash_ref.so not built (make -C oracle ref)")
    # the expected hashes come from the reference's jenkins_hash, not the oracle's
    refj = types.SimpleNamespace(jhash=lambda b: int(rj.jenkins_hash(b, len(b))))
    rng = np.random.default_rng(SEED)
    ips, frames, want = ref_struct_batch(ref, refj, rng, N, R)
    np.savez_compressed(
        OUT, ips=np.array(ips, dtype=np.uint32), frames=frames,
        uniqid=np.array([w[0] for w in want], dtype=np.uint16),
        hash=np.array([w[1] for w in want], dtype=np.uint32),
        hit=np.array([w[2] for w in want], dtype=bool),
        source=np.array("frames: reference inc/net structs via oracle/_ref/libhost_ref.so; "
                        "hash: reference base/jenkins_hash.c via oracle/_ref/libjhash_ref.so"))
    print(f"{N} frames -> {OUT}")


if __name__ == "__main__":
    main()
