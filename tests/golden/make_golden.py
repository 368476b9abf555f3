"""Generate the committed golden fixtures under tests/golden/.

Run in the survey container (where /root/reference exists):
    python tests/golden/make_golden.py

jhash_kat.json     lookup3 values computed by the REFERENCE's own
                   base/jenkins_hash.c (compiled unmodified into
                   oracle/_ref/libjhash_ref.so by oracle/Makefile), over random
                   keys of length 0..64 at every alignment, plus the 4-byte IP
                   keys and 13-byte flow keys the configs use.
toeplitz_kat.json  the Microsoft RSS verification-suite vectors (public KATs;
                   the survey ran the reference's do_toeplitz,
                   runtime/net/core.c:120-139, and got 0x51ccc178 for vector 1).
rx_scenarios.json  hand-derived expectations for rx_one_pkt
                   (iokernel/rx.c:116-233): each packet's expected verdict is
                   written out below from the reference's decision tree, not
                   computed by the oracle, so the oracle and the GPU are both
                   checked against it.  Flow hashes in the computed modes use
                   the reference jenkins_hash and the published Toeplitz KATs.
"""
import ctypes
import json
import os
import random
import socket
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libjhash_ref.so")
REF_CRC_SO = os.path.join(ROOT, "oracle", "_ref", "libcrc_ref.so")

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c"
                       "6a42b73bbeac01fa")
# (dst, dport, src, sport, ipv4-only hash, ipv4+tcp hash): the MS RSS suite
MS_VECTORS = [
    ("161.142.100.80", 1766, "66.9.149.187", 2794, 0x323e8fc2, 0x51ccc178),
    ("65.69.140.83", 4739, "199.92.111.2", 14230, 0xd718262a, 0xc626b0ea),
    ("12.22.207.184", 38024, "24.19.198.95", 12898, 0xd2d0a5de, 0x5c2b394a),
    ("209.142.163.6", 2217, "38.27.205.30", 48228, 0x82989176, 0xafc7327f),
    ("202.188.127.2", 1303, "153.39.163.191", 44251, 0x5d1809c5, 0x10e828a2),
]


def ip(s):
    return struct.unpack("!I", socket.inet_aton(s))[0]


def ref_lib():
    if not os.path.exists(REF_SO):
        sys.exit(f"{REF_SO} missing: run `make -C oracle` with /root/reference mounted")
    lib = ctypes.CDLL(REF_SO)
    lib.jenkins_hash.restype = ctypes.c_uint32
    lib.jenkins_hash.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return lib


REF = None
CRC = None


def ref_crc_lib():
    if not os.path.exists(REF_CRC_SO):
        sys.exit(f"{REF_CRC_SO} missing: run `make -C oracle` with /root/reference mounted")
    lib = ctypes.CDLL(REF_CRC_SO)
    lib.ref_crc32c_one.restype = ctypes.c_uint32
    lib.ref_crc32c_one.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    lib.ref_crc32c_two.restype = ctypes.c_uint32
    lib.ref_crc32c_two.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
    return lib


def ref_trans(seed, proto, lip, lport, rip, rport):
    """trans_hash_5tuple / _3tuple (transport.c:29-42) via the reference's
    own hash_crc32c_two / _one."""
    l = lip | lport << 32
    return (CRC.ref_crc32c_two(seed, l, rip | rport << 32 | proto << 48),
            CRC.ref_crc32c_one(seed, l | proto << 48))


def ref_jhash(key: bytes, align=0) -> int:
    buf = ctypes.create_string_buffer(b"\0" * align + key + b"\0" * 16)
    return REF.jenkins_hash(ctypes.addressof(buf) + align, len(key))


def flow_key(saddr, daddr, sport, dport, proto):
    return struct.pack("<IIHHB", saddr, daddr, dport, sport, proto)


# ---------------------------------------------------------------- frames
def eth(et, dst=b"\x02\0\0\0\0\x01", src=b"\x02\0\x11\x22\x33\x44"):
    return dst + src + struct.pack("!H", et)


def ipv4(saddr, daddr, proto, payload=b"", ihl=5, frag=0x4000, version=4, opts=None):
    optb = opts if opts is not None else b"\x01" * (4 * (ihl - 5))
    hdr = struct.pack("!BBHHHBBHII", version << 4 | ihl, 0, 20 + len(optb) + len(payload), 0x1234,
                      frag, 64, proto, 0, saddr, daddr)
    return hdr + optb + payload


def l4(sport, dport, tcp=False):
    if tcp:
        return struct.pack("!HHIIBBHHH", sport, dport, 1, 0, 0x50, 0x10, 0xFFFF, 0, 0)
    return struct.pack("!HHHH", sport, dport, 8, 0)


def arp(op, sip, tip):
    return struct.pack("!HHBBH", 1, 0x0800, 6, 4, op) + b"\x02\0\x11\x22\x33\x44" + \
        struct.pack("!I", sip) + b"\0" * 6 + struct.pack("!I", tip)


F_RSS, F_FDIR, CK_GOOD = 0x01, 0x02, 0x08
DELIVER, WAKE, DROP_ET, DROP_UNREG, BCAST, ARP_RESP = 0, 1, 2, 3, 4, 5
FDIR = 0x80

A_IP, B_IP, C_IP = ip("10.0.0.4"), ip("10.0.0.8"), ip("10.0.0.10")
# runtime A: 8 threads, active [2, 5, 7] -> sched_steer_flows (sched.c:122-147):
# identity for 2, 5, 7; slots 0,1,3,4,6 take 2,5,7,2,5 in order.
A_FLOW = [2, 5, 2, 7, 2, 5, 5, 7]
RUNTIMES = [
    {"uniqid": 3, "ip": A_IP, "thread_count": 8, "active": 3, "active_idx": [2, 5, 7],
     "flow_tbl": A_FLOW},
    {"uniqid": 7, "ip": B_IP, "thread_count": 3, "active": 3, "active_idx": [0, 1, 2],
     "flow_tbl": [0, 1, 2]},
    {"uniqid": 9, "ip": C_IP, "thread_count": 4, "active": 0, "active_idx": [],
     "flow_tbl": None},
]
TC = {3: 8, 7: 3, 9: 4}
FLOW = {3: A_FLOW, 7: [0, 1, 2]}


def steer(uniq, h):
    """rx_send_to_runtime (rx.c:55-72): the flow_tbl slot hash % thread_count
    (the verdict's `thread`), and the kthread flow_tbl[slot] the post-pass
    delivers to while the runtime has an active thread (None: wake path)."""
    slot = h % TC[uniq]
    if uniq == 9:
        return slot, None, WAKE
    return slot, FLOW[uniq][slot], DELIVER


def pkt(cite, frame, flags, rss, fdir, hash_, uniq, action, thread=None, hint=0, hint_hit=False,
        trans=None):
    """`thread` given explicitly: a runtime with an identity flow_tbl, so the
    slot is also the kthread."""
    queue = None
    if uniq is None:
        uniq, thread = 0xFFFF, 0xFF
    elif thread is None:
        thread, queue, act = steer(uniq, hash_)
        action |= act
    else:
        queue = thread
    if trans is not None:
        action |= 0x40  # GCL_ACT_F_TRANS
    return {"cite": cite, "frame": frame.hex(), "olflags": flags, "rss": rss, "fdir_hi": fdir,
            "dst_hint": hint, "hint_hit": hint_hit, "expect_trans": list(trans or (0, 0)),
            "expect": {"hash": hash_, "uniqid": uniq, "thread": thread, "action": action},
            "expect_kthread": queue}


def nic_set():
    P = []
    u = l4(1000, 2000)
    P.append(pkt("rx.c:156-163,197,213: IPv4 hit, flow_tbl[rss % 8]",
                 eth(0x0800) + ipv4(ip("1.2.3.4"), A_IP, 17, u), F_RSS | CK_GOOD, 0x12345679, 0,
                 0x12345679, 3, DELIVER))
    P.append(pkt("rx.c:160-163: no RSS flag -> RX_HASH_MISSING, still delivered",
                 eth(0x0800) + ipv4(ip("1.2.3.5"), A_IP, 17, u), 0, 10, 0, 10, 3, DELIVER))
    P.append(pkt("rx.c:198-207: unregistered IPv4 -> RX_UNREGISTERED_MAC + RX_UNHANDLED",
                 eth(0x0800) + ipv4(ip("1.2.3.6"), ip("10.9.9.9"), 17, u), F_RSS, 77, 0,
                 77, None, DROP_UNREG))
    P.append(pkt("rx.c:164-167: ARP request, tip = B -> deliver to B",
                 eth(0x0806) + arp(1, ip("10.0.0.99"), B_IP), 0, 5, 0, 5, 7, DELIVER))
    P.append(pkt("rx.c:164-167,198: ARP reply to unknown tip (non-azure) -> unregistered",
                 eth(0x0806) + arp(2, B_IP, ip("10.0.0.200")), 0, 0, 0, 0, None, DROP_UNREG))
    P.append(pkt("rx.c:191-194: IPv6 ethertype -> RX_UNHANDLED",
                 eth(0x86DD) + b"\x60" + b"\0" * 39, F_RSS, 9, 0, 9, None, DROP_ET))
    P.append(pkt("rx.c:191-194: VLAN 0x8100 is not parsed -> RX_UNHANDLED",
                 eth(0x8100) + b"\0\x05\x08\x00" + ipv4(1, A_IP, 17, u), F_RSS, 9, 0, 9, None, DROP_ET))
    P.append(pkt("rx.c:157-159: dst read at offset 30 with no version check",
                 eth(0x0800) + ipv4(ip("1.1.1.1"), A_IP, 17, u, version=6), F_RSS, 6, 0, 6, 3, DELIVER))
    P.append(pkt("rx.c:157-159: IHL=7 does not move daddr",
                 eth(0x0800) + ipv4(ip("1.1.1.2"), A_IP, 6, l4(1, 2, True), ihl=7), F_RSS, 15, 0,
                 15, 3, DELIVER))
    P.append(pkt("rx.c: fragments are classified like any IPv4 packet",
                 eth(0x0800) + ipv4(ip("1.1.1.3"), B_IP, 17, u, frag=0x2000), F_RSS, 4, 0, 4, 7, DELIVER))
    P.append(pkt("rx.c:131-146: FDIR mark of B on an IPv6 frame -> RX_FLOW_TAG_MATCH, deliver to B",
                 eth(0x86DD) + b"\x60" + b"\0" * 39, F_FDIR | F_RSS, 8, 7, 8, 7, FDIR))
    P.append(pkt("rx.c:138-146: FDIR mark of a removed proc falls through to the parse",
                 eth(0x0800) + ipv4(ip("1.1.1.4"), A_IP, 17, u), F_FDIR | F_RSS, 3, 12, 3, 3, DELIVER))
    P.append(pkt("rx.c:131-146,198: out-of-range FDIR mark, unregistered IP",
                 eth(0x0800) + ipv4(ip("1.1.1.5"), ip("172.16.0.1"), 17, u), F_FDIR | F_RSS, 3, 9999,
                 3, None, DROP_UNREG))
    P.append(pkt("rx.c:132-134: FDIR without RSS flag warns only; no RX_HASH_MISSING on this branch",
                 eth(0x0800) + ipv4(ip("1.1.1.6"), ip("1.1.1.7"), 17, u), F_FDIR, 17, 3, 17, 3, FDIR))
    P.append(pkt("rx.c:62-72: runtime with 0 active threads -> host wake path",
                 eth(0x0800) + ipv4(ip("1.1.1.8"), C_IP, 17, u), F_RSS, 21, 0, 21, 9, 0))
    P.append(pkt("rx.c:164-167: ARP reply to A (non-azure) is delivered",
                 eth(0x0806) + arp(2, B_IP, A_IP), 0, 0, 0, 0, 3, DELIVER))
    return {
        "name": "nic_mode",
        "cfg": {"max_runtimes": 16, "hash_mode": 0, "flags": 0, "default_olflags": 0,
                "rss_key": MS_KEY.hex()},
        "packets": P,
    }


def azure_set():
    P = []
    P.append(pkt("rx.c:171-190: azure ARP reply -> broadcast to every runtime",
                 eth(0x0806) + arp(2, ip("10.0.0.1"), ip("10.0.0.77")), 0, 0, 0, 0, None, BCAST))
    P.append(pkt("rx.c:200-203: azure ARP request to an unknown IP -> ARP response (host)",
                 eth(0x0806) + arp(1, ip("10.0.0.1"), ip("10.0.0.77")), 0, 0, 0, 0, None, ARP_RESP))
    P.append(pkt("rx.c:197,213: azure ARP request to B -> delivered",
                 eth(0x0806) + arp(1, ip("10.0.0.1"), B_IP), 0, 4, 0, 4, 7, DELIVER))
    P.append(pkt("rx.c:198-207: azure IPv4 miss is still unregistered",
                 eth(0x0800) + ipv4(1, ip("10.0.0.77"), 17, l4(1, 2)), F_RSS, 0, 0, 0, None, DROP_UNREG))
    return {
        "name": "azure_arp_mode",
        "cfg": {"max_runtimes": 16, "hash_mode": 0, "flags": 1, "default_olflags": 0,
                "rss_key": MS_KEY.hex()},
        "packets": P,
    }


def loopback_set():
    """Local traffic re-entering rx through rx_loopback (rx.c:235-265):
    tx_prepare_tx_mbuf sets hash.rss to the runtime's 16-bit hint and
    RSS_HASH iff TXFLAG_LOCAL_HINT (tx.c:81-83); copy_batch adds
    IP_CKSUM_GOOD (dma.c:182-185); a dst_ip hint found in ip_to_proc sets
    FDIR_ID with fdir.hi = uniqid (rx.c:250-262) and rx_one_pkt delivers on
    that mark (rx.c:131-146) whatever the frame holds."""
    P = []
    u = l4(40000, 80)
    LH = F_RSS | CK_GOOD  # TXFLAG_LOCAL_HINT set
    NH = CK_GOOD          # no local hint
    P.append(pkt("rx.c:250-262 + :131-146: hint = A -> FDIR to A, thread flow_tbl[hint16 % 8]",
                 eth(0x0800) + ipv4(A_IP - 1, A_IP, 17, u), LH, 0xBEEF, 0, 0xBEEF, 3, FDIR,
                 hint=A_IP, hint_hit=True))
    P.append(pkt("rx.c:258-260: the mark comes from the hint, not from the frame (hint B, daddr A)",
                 eth(0x0800) + ipv4(A_IP - 1, A_IP, 17, u), LH, 0x1234, 0, 0x1234, 7, FDIR,
                 hint=B_IP, hint_hit=True))
    P.append(pkt("rx.c:252-253: no hint -> parse path; no LOCAL_HINT -> RX_HASH_MISSING",
                 eth(0x0800) + ipv4(A_IP, B_IP, 17, u), NH, 0, 0, 0, 7, DELIVER))
    P.append(pkt("rx.c:258: hint miss leaves the flags -> parse path to the frame's daddr",
                 eth(0x0800) + ipv4(B_IP, A_IP, 17, u), LH, 0x55, 0, 0x55, 3, DELIVER,
                 hint=ip("10.1.1.1")))
    P.append(pkt("rx.c:62-72: hint to a runtime with no active thread -> wake",
                 eth(0x0800) + ipv4(A_IP, C_IP, 17, u), LH, 0x77, 0, 0x77, 9, FDIR,
                 hint=C_IP, hint_hit=True))
    P.append(pkt("rx.c:131-146: FDIR delivery ignores the Ethertype (hinted ARP)",
                 eth(0x0806, dst=b"\xff" * 6) + arp(1, B_IP, A_IP), LH, 0x3, 0, 0x3, 3, FDIR,
                 hint=A_IP, hint_hit=True))
    P.append(pkt("tx.c:285-289 broadcast loopback (no hint): ARP request parsed to its tip",
                 eth(0x0806, dst=b"\xff" * 6) + arp(1, A_IP, B_IP), NH, 0, 0, 0, 7, DELIVER))
    P.append(pkt("hint miss on IPv6 -> rx.c:191-194 drop",
                 eth(0x86DD) + b"\x60" + b"\0" * 39, LH, 1, 0, 1, None, DROP_ET, hint=ip("10.1.1.2")))
    P.append(pkt("rx.c:260: a hint hit overrides an mbuf's own fdir.hi",
                 eth(0x0800) + ipv4(A_IP, C_IP, 17, u), F_FDIR | LH, 0x10, 7, 0x10, 3, FDIR,
                 hint=A_IP, hint_hit=True))
    P.append(pkt("hint miss keeps an mbuf's own FDIR mark (fdir.hi = B)",
                 eth(0x0800) + ipv4(A_IP, C_IP, 17, u), F_FDIR | LH, 0x11, 7, 0x11, 7, FDIR,
                 hint=ip("10.1.1.3")))
    return {
        "name": "loopback",
        "cfg": {"max_runtimes": 16, "hash_mode": 0, "flags": 0, "default_olflags": 0,
                "rss_key": MS_KEY.hex()},
        "packets": P,
    }


SEEDS = {3: 0x12345678, 7: 0xCAFEBABE, 9: 0x0BADF00D}


def trans_set():
    """Runtime-side demux pre-hash (gclassify.h struct gcl_trans): for a packet
    delivered to runtime p, trans_hash_5tuple/_3tuple with p's trans_seed,
    when net_rx_one would pass it to net_rx_trans (core.c:203-209, :288-290)."""
    P = []
    sa, sp, dp = ip("192.168.7.9"), 51000, 443
    P.append(pkt("transport.c:29-42: UDP to A, laddr=(daddr,dport) raddr=(saddr,sport)",
                 eth(0x0800) + ipv4(sa, A_IP, 17, l4(sp, dp)), F_RSS | CK_GOOD, 0x99, 0,
                 0x99, 3, DELIVER, trans=ref_trans(SEEDS[3], 17, A_IP, dp, sa, sp)))
    P.append(pkt("TCP to B with B's seed",
                 eth(0x0800) + ipv4(sa, B_IP, 6, l4(sp, 80, True)), F_RSS, 0x5, 0, 0x5, 7, DELIVER,
                 trans=ref_trans(SEEDS[7], 6, B_IP, 80, sa, sp)))
    P.append(pkt("wake path still names the runtime: C's seed",
                 eth(0x0800) + ipv4(sa, C_IP, 17, l4(7, 9)), F_RSS, 0x6, 0, 0x6, 9, 0,
                 trans=ref_trans(SEEDS[9], 17, C_IP, 9, sa, 7)))
    P.append(pkt("core.c:207: IP options (IHL 6) are dropped by the runtime: no pre-hash",
                 eth(0x0800) + ipv4(sa, A_IP, 17, l4(sp, dp), ihl=6), F_RSS, 0x7, 0, 0x7, 3, DELIVER))
    P.append(pkt("core.c:206: version 6 in an IPv4 frame: no pre-hash",
                 eth(0x0800) + ipv4(sa, A_IP, 17, l4(sp, dp), version=6), F_RSS, 0x8, 0, 0x8, 3, DELIVER))
    P.append(pkt("core.c:208 as written: IP_MF tested on the network-order field, so a real MF "
                 "fragment (0x2000 BE) passes",
                 eth(0x0800) + ipv4(sa, A_IP, 17, l4(sp, dp), frag=0x2000), F_RSS, 0x9, 0, 0x9, 3,
                 DELIVER, trans=ref_trans(SEEDS[3], 17, A_IP, dp, sa, sp)))
    P.append(pkt("core.c:208 as written: offset 0x0020 sets the tested bit: no pre-hash",
                 eth(0x0800) + ipv4(sa, A_IP, 17, l4(sp, dp), frag=0x0020), F_RSS, 0xA, 0, 0xA, 3,
                 DELIVER))
    P.append(pkt("core.c:293-299: ICMP goes to net_rx_icmp: no pre-hash",
                 eth(0x0800) + ipv4(sa, A_IP, 1, b"\x08" + b"\0" * 7), F_RSS, 0xB, 0, 0xB, 3, DELIVER))
    P.append(pkt("unregistered IP: no runtime, no pre-hash",
                 eth(0x0800) + ipv4(sa, ip("10.9.9.9"), 17, l4(sp, dp)), F_RSS, 0xC, 0, 0xC, None,
                 DROP_UNREG))
    P.append(pkt("FDIR delivery of an ARP frame: not IPv4, no pre-hash",
                 eth(0x0806) + arp(1, sa, A_IP), F_FDIR | F_RSS, 0xD, 3, 0xD, 3, FDIR))
    return {
        "name": "trans_demux",
        "cfg": {"max_runtimes": 16, "hash_mode": 0, "flags": 8, "default_olflags": 0,
                "rss_key": MS_KEY.hex()},
        "trans_seeds": {str(k): v for k, v in SEEDS.items()},
        "packets": P,
    }


def crc_kats():
    rnd = random.Random(0xC5C)
    out = []
    for _ in range(400):
        seed, a, b = rnd.getrandbits(32), rnd.getrandbits(64), rnd.getrandbits(64)
        out.append({"seed": seed, "a": a, "b": b, "one": CRC.ref_crc32c_one(seed, a),
                    "two": CRC.ref_crc32c_two(seed, a, b)})
    return out


def jenkins_set():
    P = []
    cases = [
        ("UDP, IHL 5", 17, 5, 0x4000, 1111, 2222, ip("9.8.7.6")),
        ("TCP, IHL 6: ports at 14 + 24", 6, 6, 0x4000, 80, 51515, ip("9.8.7.5")),
        ("TCP, IHL 11: last ports inside the 64-B granule", 6, 11, 0, 443, 3333, ip("9.8.7.4")),
        ("UDP, IHL 13: ports past the 64-B granule", 17, 13, 0, 53, 5353, ip("9.8.7.3")),
    ]
    for name, proto, ihl, frag, sp, dp, sa in cases:
        h = ref_jhash(flow_key(sa, A_IP, sp, dp, proto))
        P.append(pkt(f"gclassify.h JENKINS: {name}; jenkins_hash.c value",
                     eth(0x0800) + ipv4(sa, A_IP, proto, l4(sp, dp, proto == 6), ihl=ihl, frag=frag),
                     F_RSS, 0, 0, h, 3, DELIVER))
    P.append(pkt("JENKINS: ICMP is not hashed (hash 0 -> flow_tbl[0])",
                 eth(0x0800) + ipv4(ip("9.9.9.9"), A_IP, 1, b"\x08\0\0\0\0\0\0\0"), F_RSS, 0, 0,
                 0, 3, DELIVER))
    P.append(pkt("JENKINS: fragment (MF) is not hashed",
                 eth(0x0800) + ipv4(ip("9.9.9.8"), A_IP, 17, l4(5, 6), frag=0x2000), F_RSS, 0, 0,
                 0, 3, DELIVER))
    P.append(pkt("JENKINS: non-zero fragment offset is not hashed",
                 eth(0x0800) + ipv4(ip("9.9.9.7"), B_IP, 6, l4(5, 6, True), frag=0x0010), F_RSS, 0, 0,
                 0, 7, DELIVER))
    P.append(pkt("JENKINS: IHL < 5 is not hashed",
                 eth(0x0800) + ipv4(ip("9.9.9.6"), B_IP, 6, l4(5, 6, True), ihl=4, opts=b""), F_RSS,
                 0, 0, 0, 7, DELIVER))
    P.append(pkt("JENKINS: ARP is not hashed",
                 eth(0x0806) + arp(1, 1, B_IP), 0, 0, 0, 0, 7, DELIVER))
    h = ref_jhash(flow_key(ip("7.7.7.7"), C_IP, 9, 10, 17))
    P.append(pkt("JENKINS: wake path keeps the computed hash",
                 eth(0x0800) + ipv4(ip("7.7.7.7"), C_IP, 17, l4(9, 10)), F_RSS, 0, 0, h, 9, 0))
    return {
        "name": "jenkins_mode",
        "cfg": {"max_runtimes": 16, "hash_mode": 1, "flags": 0, "default_olflags": 0,
                "rss_key": MS_KEY.hex()},
        "packets": P,
    }


def toeplitz_set(hash16):
    # register the MS vectors' destinations as extra runtimes so the expected
    # hashes are the published KAT values
    P = []
    extra = []
    for i, (d, dp, s, sp, h4, h4t) in enumerate(MS_VECTORS):
        uniq = 10 + i
        extra.append({"uniqid": uniq, "ip": ip(d), "thread_count": 5 + i, "active": 5 + i,
                      "active_idx": list(range(5 + i)), "flow_tbl": list(range(5 + i))})
        h = h4t & 0xFFFF if hash16 else h4t
        P.append(pkt(f"runtime/net/core.c:120-139 Toeplitz, MS RSS vector {i + 1} (TCP)",
                     eth(0x0800) + ipv4(ip(s), ip(d), 6, l4(sp, dp, True)), F_RSS, 0, 0,
                     h, uniq, DELIVER, thread=h % (5 + i)))
    d, dp, s, sp, h4, h4t = MS_VECTORS[0]
    h = h4t & 0xFFFF if hash16 else h4t
    P.append(pkt("Toeplitz over UDP uses the same tuple (rss_hf NONFRAG_IPV4_UDP, dpdk.c:79)",
                 eth(0x0800) + ipv4(ip(s), ip(d), 17, l4(sp, dp)), F_RSS, 0, 0, h, 10, DELIVER,
                 thread=h % 5))
    return {
        "name": "toeplitz16_mode" if hash16 else "toeplitz_mode",
        "cfg": {"max_runtimes": 16, "hash_mode": 2, "flags": 2 if hash16 else 0,
                "default_olflags": 0, "rss_key": MS_KEY.hex()},
        "extra_runtimes": extra,
        "packets": P,
    }


def expected_stats(s):
    st = [0] * 8
    fl_set = s["cfg"]["flags"]
    for p in s["packets"]:
        e = p["expect"]
        act = e["action"] & 0x3F
        fl = p["olflags"]
        st[6] += 1  # RX_PULLED
        if fl & F_FDIR or p.get("hint_hit"):
            st[3] += 1  # RX_FLOW_TAG_MATCH
        et = int(p["frame"][24:28], 16)
        if not (e["action"] & FDIR) and et == 0x0800 and not (fl & F_RSS):
            st[5] += 1  # RX_HASH_MISSING (parse path only)
        if act == DROP_UNREG:
            st[0] += 1
            st[4] += 1
        elif act == DROP_ET:
            st[4] += 1
        _ = fl_set
    return st


def expected_counts(s):
    counts = [0] * s["cfg"]["max_runtimes"]
    for p in s["packets"]:
        e = p["expect"]
        if e["action"] & 0x3F in (DELIVER, WAKE):
            counts[e["uniqid"]] += 1
    return counts


def jhash_kats():
    rnd = random.Random(0xCA1ADA4)
    out = []
    for L in list(range(0, 65)) * 12:
        key = bytes(rnd.getrandbits(8) for _ in range(L))
        align = rnd.randrange(4)
        out.append({"key": key.hex(), "align": align, "hash": ref_jhash(key, align)})
    for r in range(32):
        k = struct.pack("<I", 0x0A000000 + r + 1)
        out.append({"key": k.hex(), "align": 0, "hash": ref_jhash(k), "what": "ip_to_proc key"})
    for i in range(64):
        k = flow_key(rnd.getrandbits(32), 0x0A000000 + i + 1, rnd.getrandbits(16),
                     rnd.getrandbits(16), rnd.choice([6, 17]))
        out.append({"key": k.hex(), "align": 0, "hash": ref_jhash(k), "what": "13-B flow key"})
    out.append({"key": b"Four score and seven years ago".hex(), "align": 0,
                "hash": ref_jhash(b"Four score and seven years ago"), "what": "lookup3 KAT"})
    return out


def main():
    global REF, CRC
    REF = ref_lib()
    CRC = ref_crc_lib()
    with open(os.path.join(HERE, "crc32c_kat.json"), "w") as f:
        json.dump({"source": "reference hash_crc32c_one/two (inc/base/hash.h) via oracle/_ref/libcrc_ref.so",
                   "vectors": crc_kats()}, f, indent=0)
    assert ref_jhash(b"") == 0xdeadbeef
    assert ref_jhash(b"Four score and seven years ago") == 0x17770551
    with open(os.path.join(HERE, "jhash_kat.json"), "w") as f:
        json.dump({"source": "reference base/jenkins_hash.c (oracle/_ref/libjhash_ref.so)",
                   "vectors": jhash_kats()}, f, indent=0)
    with open(os.path.join(HERE, "toeplitz_kat.json"), "w") as f:
        json.dump({"source": "Microsoft RSS verification suite (public KAT)", "key": MS_KEY.hex(),
                   "vectors": [{"dst": d, "dport": dp, "src": s, "sport": sp, "ipv4": h4,
                                "ipv4_tcp": h4t} for d, dp, s, sp, h4, h4t in MS_VECTORS]},
                  f, indent=1)
    sets = [nic_set(), azure_set(), loopback_set(), trans_set(), jenkins_set(),
            toeplitz_set(False), toeplitz_set(True)]
    for s in sets:
        s["runtimes"] = RUNTIMES + s.pop("extra_runtimes", [])
        s["expect_stats"] = expected_stats(s)
        s["expect_counts"] = expected_counts(s)
    with open(os.path.join(HERE, "rx_scenarios.json"), "w") as f:
        json.dump({"source": "hand-derived from iokernel/rx.c:116-233 (see make_golden.py); expect.thread is the "
                           "flow_tbl slot hash % thread_count, expect_kthread the flow_tbl entry the "
                           "host post-pass delivers to (rx.c:55-59), null on the wake path",
                   "slot": 128, "sets": sets}, f, indent=1)
    print("wrote", [s["name"] + f"({len(s['packets'])})" for s in sets])


if __name__ == "__main__":
    main()
