"""Pin the oracle's hashes (and the product's host copies) to the reference's
own outputs and to published known-answer vectors."""
import os
import socket
import struct

import pytest

from tests.rxcases import load_json


def _ip(s):
    return struct.unpack("!I", socket.inet_aton(s))[0]


def test_jhash_lookup3_kats(orc):
    # lookup3 hashlittle KATs, reproduced by base/jenkins_hash.c in the survey
    assert orc.jhash(b"") == 0xDEADBEEF
    assert orc.jhash(b"Four score and seven years ago") == 0x17770551
    assert orc.jhash(struct.pack("<I", 0xC0A80103)) == 0xE82DB31C


def test_jhash_golden_from_reference(orc):
    """tests/golden/jhash_kat.json was produced by the reference jenkins_hash.c."""
    from caladan_amd import gclassify as g
    vecs = load_json("jhash_kat.json")["vectors"]
    assert len(vecs) > 800
    for v in vecs:
        key = bytes.fromhex(v["key"])
        assert orc.jhash(key) == v["hash"], v
        assert g.jenkins_hash(key) == v["hash"], v


def test_jhash_live_reference(orc):
    """When oracle/_ref is built (reference tree mounted), compare live."""
    import ctypes
    ref = orc.ref_jhash()
    if ref is None:
        pytest.skip("oracle/_ref/libjhash_ref.so not built")
    for L in range(0, 100):
        key = os.urandom(L)
        for align in range(4):
            buf = ctypes.create_string_buffer(b"\0" * align + key + b"\0" * 16)
            assert ref.jenkins_hash(ctypes.addressof(buf) + align, L) == orc.jhash(key)


def test_toeplitz_ms_vectors(orc):
    from caladan_amd import gclassify as g
    d = load_json("toeplitz_kat.json")
    key = bytes.fromhex(d["key"])
    for v in d["vectors"]:
        s, dd = _ip(v["src"]), _ip(v["dst"])
        tup = struct.pack("!IIHH", s, dd, v["sport"], v["dport"])
        assert orc.do_toeplitz(key, s, dd, v["sport"], v["dport"]) == v["ipv4_tcp"]
        assert orc.toeplitz_bytes(key, tup) == v["ipv4_tcp"]
        assert orc.toeplitz_bytes(key, tup[:8]) == v["ipv4"]
        assert g.toeplitz(key, tup) == v["ipv4_tcp"]
        assert g.toeplitz(key, tup[:8]) == v["ipv4"]


def test_toeplitz_do_vs_bytes_random(orc):
    """do_toeplitz's word/bit formulation equals the textbook byte form."""
    import random
    from caladan_amd import gclassify as g
    rnd = random.Random(7)
    key = g.CALADAN_RSS_KEY
    for _ in range(2000):
        s, d = rnd.getrandbits(32), rnd.getrandbits(32)
        sp, dp = rnd.getrandbits(16), rnd.getrandbits(16)
        tup = struct.pack("!IIHH", s, d, sp, dp)
        h = orc.do_toeplitz(key, s, d, sp, dp)
        assert h == orc.toeplitz_bytes(key, tup)
        assert h == g.toeplitz(key, tup)


def test_toeplitz_golden_from_reference(orc):
    """tests/golden/toeplitz_ref.json was produced by the reference's own
    do_toeplitz (runtime/net/core.c:120-139, compiled in place by
    oracle/ref_core.c; tests/golden/make_toeplitz_ref.py): Caladan's RSS
    key and random keys over random and edge 4-tuples."""
    from caladan_amd import gclassify as g
    d = load_json("toeplitz_ref.json")
    keys = [bytes.fromhex(k) for k in d["keys"]]
    assert keys[0] == g.CALADAN_RSS_KEY and len(d["vectors"]) > 900
    for v in d["vectors"]:
        key = keys[v["key"]]
        s, dd, sp, dp = v["saddr"], v["daddr"], v["sport"], v["dport"]
        assert orc.do_toeplitz(key, s, dd, sp, dp) == v["hash"], v
        assert g.toeplitz(key, struct.pack("!IIHH", s, dd, sp, dp)) == v["hash"], v


def test_toeplitz_live_reference(orc):
    """When oracle/_ref is built (reference tree mounted), compare the oracle
    with the reference's do_toeplitz live on fresh random keys and tuples."""
    import random
    ref = orc.ref_toeplitz()
    if ref is None:
        pytest.skip("oracle/_ref/libcore_ref.so not built")
    rnd = random.Random(os.getpid())
    for _ in range(20):
        key = bytes(rnd.getrandbits(8) for _ in range(40))
        for _ in range(200):
            t = (rnd.getrandbits(32), rnd.getrandbits(32), rnd.getrandbits(16), rnd.getrandbits(16))
            assert orc.do_toeplitz(key, *t) == ref(key, *t), (key.hex(), t)


def test_trans_hash_golden_from_reference():
    """tests/golden/trans_ref.json was produced by the reference's own
    trans_hash_5tuple/3tuple (runtime/net/transport.c:29-42, compiled in
    place by oracle/ref_trans.c): the product's host gcl_trans_hash equals
    it on received-frame tuples and on arbitrary inputs."""
    from caladan_amd import gclassify as g
    d = load_json("trans_ref.json")
    for v in d["frames"]:
        r = v["runtime"]
        got = g.trans_hash(d["trans_seeds"][r], v["proto"], d["runtime_ips"][r], v["dport"],
                           v["saddr"], v["sport"])
        assert tuple(got) == (v["h5"], v["h3"]), v
    for v in d["random"]:
        got = g.trans_hash(v["seed"], v["proto"], v["lip"], v["lport"], v["rip"], v["rport"])
        assert tuple(got) == (v["h5"], v["h3"]), v


def test_trans_hash_live_reference(orc):
    """When oracle/_ref is built, the product's host transport hashes equal
    the reference's trans_hash_5tuple/3tuple live on fresh random inputs."""
    import random
    from caladan_amd import gclassify as g
    ref = orc.ref_trans()
    if ref is None:
        pytest.skip("oracle/_ref/libtrans_ref.so not built")
    rnd = random.Random(os.getpid())
    for _ in range(5000):
        a = (rnd.getrandbits(32), rnd.getrandbits(8), rnd.getrandbits(32), rnd.getrandbits(16),
             rnd.getrandbits(32), rnd.getrandbits(16))
        assert ref(*a) == tuple(g.trans_hash(*a)), a


def _iphdr_frames(d, ip):
    import numpy as np
    hdrs = d["headers"]
    frames = np.zeros(len(hdrs) * 64, dtype=np.uint8)
    for i, v in enumerate(hdrs):
        h = bytearray.fromhex(v["hdr"])
        h[16:20] = struct.pack("!I", ip)  # to the registered runtime; not part of the predicate
        fr = bytes(12) + b"\x08\x00" + bytes(h) + struct.pack("!HH", 1000 + i, 80)
        frames[64 * i:64 * i + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
    return frames


def test_ip_hdr_supported_golden_from_reference(orc):
    """Which delivered frames get the transport demux pre-hash follows the
    reference's own ip_hdr_supported (runtime/net/core.c:203-209, quirk
    included: IP_MF tested on the network-order field), per
    tests/golden/iphdr_ref.json (generated by core.c compiled in place): all
    256 version/IHL bytes x 10 fragment fields through the oracle."""
    import numpy as np
    from caladan_amd import gclassify as g
    d = load_json("iphdr_ref.json")
    ip = 0x0A000001
    t = orc.Tables(16, g.HASH_NIC, g.CFG_TRANS_HASH, 0x09)
    t.runtime_set(0, ip, 4, 4, [0, 1, 2, 3])
    n = len(d["headers"])
    v, _, _, _ = t.classify(_iphdr_frames(d, ip), n, 64, trans=True)
    got = (v["action"] & g.ACT_F_TRANS) != 0
    want = np.array([h["supported"] for h in d["headers"]])
    assert want.sum() == 7 and (got == want).all(), np.nonzero(got != want)[0][:5]


def test_ip_hdr_supported_live_reference(orc):
    """The same against the reference live, on random headers."""
    import random
    ref = orc.ref_ip_hdr_supported()
    if ref is None:
        pytest.skip("oracle/_ref/libcore_ref.so not built")
    d = load_json("iphdr_ref.json")
    for h in d["headers"]:
        assert ref(bytes.fromhex(h["hdr"])) == h["supported"]
    rnd = random.Random(os.getpid())
    for _ in range(2000):
        hdr = bytes(rnd.getrandbits(8) for _ in range(20))
        vihl, frag = hdr[0], hdr[6] | hdr[7] << 8
        assert ref(hdr) == (vihl == 0x45 and not (frag & 0x2000)), hdr.hex()
