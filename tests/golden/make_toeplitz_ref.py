"""Generate tests/golden/toeplitz_ref.json from the REFERENCE's own
do_toeplitz (runtime/net/core.c:120-139), compiled in place into
oracle/_ref/libcore_ref.so by oracle/Makefile (oracle/ref_core.c).

Run where /root/reference exists (after `make -C oracle ref`):
    python tests/golden/make_toeplitz_ref.py

Vectors: Caladan's 40-B RSS key (mlx5_init_verbs.c:90-94) and random keys,
over random 4-tuples plus the edge tuples (all-zero, all-ones, single bits).
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from caladan_amd.gclassify import CALADAN_RSS_KEY  # noqa: E402
from oracle import orc  # noqa: E402


def main():
    ref = orc.ref_toeplitz()
    if ref is None:
        raise SystemExit("oracle/_ref/libcore_ref.so not built (make -C oracle ref)")
    rnd = random.Random(0x7E0B)
    keys = [CALADAN_RSS_KEY] + [bytes(rnd.getrandbits(8) for _ in range(40)) for _ in range(7)]
    vecs = []
    for ki, key in enumerate(keys):
        tuples = [(0, 0, 0, 0), (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFF, 0xFFFF)]
        tuples += [(1 << b, 0, 0, 0) for b in (0, 7, 31)] + [(0, 1 << b, 0, 0) for b in (0, 16, 31)]
        tuples += [(0, 0, 1 << b, 0) for b in (0, 15)] + [(0, 0, 0, 1 << b) for b in (0, 15)]
        n = 400 if ki == 0 else 60
        tuples += [(rnd.getrandbits(32), rnd.getrandbits(32), rnd.getrandbits(16), rnd.getrandbits(16))
                   for _ in range(n)]
        for s, d, sp, dp in tuples:
            vecs.append({"key": ki, "saddr": s, "daddr": d, "sport": sp, "dport": dp,
                         "hash": ref(key, s, d, sp, dp)})
    out = {"source": "reference do_toeplitz (runtime/net/core.c:120-139) via oracle/_ref/libcore_ref.so",
           "keys": [k.hex() for k in keys], "vectors": vecs}
    with open(os.path.join(HERE, "toeplitz_ref.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(f"{len(vecs)} vectors")


if __name__ == "__main__":
    main()
