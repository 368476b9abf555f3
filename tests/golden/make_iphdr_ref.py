"""Generate tests/golden/iphdr_ref.json from the REFERENCE's own
ip_hdr_supported (runtime/net/core.c:203-209: which received IPv4 frames a
runtime passes to its transport demux), compiled in place into
oracle/_ref/libcore_ref.so by oracle/Makefile (oracle/ref_core.c).

Run where /root/reference exists (after `make -C oracle ref`):
    python tests/golden/make_iphdr_ref.py

Headers: every version/IHL nibble pair, the fragment-field values that
matter (MF and DF in either byte, offsets), random bytes elsewhere.
"""
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import orc  # noqa: E402


def main():
    ref = orc.ref_ip_hdr_supported()
    if ref is None:
        raise SystemExit("oracle/_ref/libcore_ref.so not built (make -C oracle ref)")
    rnd = random.Random(0x1F4D)
    frags = [0x0000, 0x4000, 0x2000, 0x6000, 0x0001, 0x1FFF, 0x0020, 0x0040, 0x8000, 0x00FF]
    out = []
    for vihl in range(256):
        for frag in frags:
            hdr = struct.pack("!BBHHHBBHII", vihl, rnd.getrandbits(8), rnd.getrandbits(16),
                              rnd.getrandbits(16), frag, rnd.getrandbits(8), rnd.choice([6, 17]),
                              rnd.getrandbits(16), rnd.getrandbits(32), rnd.getrandbits(32))
            out.append({"hdr": hdr.hex(), "supported": ref(hdr)})
    with open(os.path.join(HERE, "iphdr_ref.json"), "w") as f:
        json.dump({"source": "reference ip_hdr_supported (runtime/net/core.c:203-209) via "
                             "oracle/_ref/libcore_ref.so", "headers": out}, f, indent=0)
    print(len(out), "headers,", sum(v["supported"] for v in out), "supported")


if __name__ == "__main__":
    main()
