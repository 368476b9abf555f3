"""Generate tests/golden/trans_ref.json from the REFERENCE's own
trans_hash_5tuple / trans_hash_3tuple (runtime/net/transport.c:29-42),
compiled in place into oracle/_ref/libtrans_ref.so by oracle/Makefile
(oracle/ref_trans.c).

Run where /root/reference exists (after `make -C oracle ref`):
    python tests/golden/make_trans_ref.py

"frames": 16 runtimes (IP 10.0.0.r+1, a random trans_seed each) and IPv4
TCP/UDP packets to them: laddr = (daddr, dport), raddr = (saddr, sport), as
trans_lookup forms them for a received frame (transport.c:366-375).
"random": the hash functions over arbitrary inputs.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import orc  # noqa: E402

R = 16


def main():
    ref = orc.ref_trans()
    if ref is None:
        raise SystemExit("oracle/_ref/libtrans_ref.so not built (make -C oracle ref)")
    rnd = random.Random(0x7A45)
    seeds = [rnd.getrandbits(32) for _ in range(R)]
    ips = [0x0A000000 + r + 1 for r in range(R)]
    frames = []
    for _ in range(640):
        r = rnd.randrange(R)
        proto = rnd.choice([6, 17])
        s, sp, dp = rnd.getrandbits(32), rnd.getrandbits(16), rnd.getrandbits(16)
        h5, h3 = ref(seeds[r], proto, ips[r], dp, s, sp)
        frames.append({"runtime": r, "proto": proto, "saddr": s, "sport": sp, "dport": dp,
                       "h5": h5, "h3": h3})
    rand = []
    for _ in range(256):
        a = (rnd.getrandbits(32), rnd.getrandbits(8), rnd.getrandbits(32), rnd.getrandbits(16),
             rnd.getrandbits(32), rnd.getrandbits(16))
        h5, h3 = ref(*a)
        rand.append({"seed": a[0], "proto": a[1], "lip": a[2], "lport": a[3], "rip": a[4],
                     "rport": a[5], "h5": h5, "h3": h3})
    out = {"source": "reference trans_hash_5tuple/3tuple (runtime/net/transport.c:29-42) via "
                     "oracle/_ref/libtrans_ref.so",
           "runtime_ips": ips, "trans_seeds": seeds, "frames": frames, "random": rand}
    with open(os.path.join(HERE, "trans_ref.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(f"{len(frames)} frame vectors, {len(rand)} random")


if __name__ == "__main__":
    main()
