"""Test-side builders: golden scenario loader and a seeded edge-case packet
generator that exercises every branch of rx_one_pkt (iokernel/rx.c:116-233)."""
import json
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

F_RSS, F_FDIR = 0x01, 0x02


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def scenario_sets():
    return load_json("rx_scenarios.json")["sets"]


def scenario_batch(s, slot=128):
    """Frames of a scenario set in `slot`-byte slots plus per-packet arrays."""
    pk = s["packets"]
    n = len(pk)
    frames = np.zeros(n * slot, dtype=np.uint8)
    for i, p in enumerate(pk):
        b = bytes.fromhex(p["frame"])
        assert len(b) <= slot
        frames[i * slot:i * slot + len(b)] = np.frombuffer(b, dtype=np.uint8)
    olflags = np.array([p["olflags"] for p in pk], dtype=np.uint8)
    rss = np.array([p["rss"] for p in pk], dtype=np.uint32)
    fdir = np.array([p["fdir_hi"] for p in pk], dtype=np.uint32)
    hint = np.array([p.get("dst_hint", 0) for p in pk], dtype=np.uint32)
    exp = np.zeros(n, dtype=[("hash", "<u4"), ("uniqid", "<u2"), ("thread", "u1"), ("action", "u1")])
    for i, p in enumerate(pk):
        e = p["expect"]
        exp[i] = (e["hash"], e["uniqid"], e["thread"], e["action"])
    return frames, olflags, rss, fdir, exp, (hint if hint.any() else None)


def scenario_trans(s):
    """Expected (h5, h3) per packet of a set, or None if the set has no seeds."""
    if "trans_seeds" not in s:
        return None
    t = np.zeros(len(s["packets"]), dtype=[("h5", "<u4"), ("h3", "<u4")])
    for i, p in enumerate(s["packets"]):
        t[i] = tuple(p["expect_trans"])
    return t


def apply_seeds(target, s):
    for u, seed in s.get("trans_seeds", {}).items():
        assert target.set_trans_seed(int(u), seed) in (0, None)


def apply_runtimes(target, runtimes):
    """target: oracle Tables or gclassify.Classifier (same runtime_set API)."""
    for r in runtimes:
        ret = target.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"])
        assert ret == 0, (r, ret)


# ---------------------------------------------------------------- fuzz
def _csum(hdr):
    s = sum(struct.unpack("!%dH" % (len(hdr) // 2), hdr))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def random_runtimes(rng, max_runtimes, count, max_threads=16):
    """Runtimes with random IPs, thread counts (incl. non-powers of two) and
    active sets (incl. zero active threads); flow tables by sched_steer_flows."""
    from oracle import orc
    uniqs = rng.choice(max_runtimes, size=count, replace=False)
    ips = set()
    out = []
    for u in uniqs:
        while True:
            ip = int(rng.integers(1, 2**32 - 1))
            if ip not in ips:
                ips.add(ip)
                break
        tc = int(rng.integers(1, max_threads + 1))
        active = int(rng.integers(0, tc + 1)) if rng.random() < 0.85 else 0
        act_idx = [int(x) for x in rng.choice(tc, size=active, replace=False)]
        flow = orc.steer_flows(tc, act_idx) if active else None
        out.append({"uniqid": int(u), "ip": ip, "thread_count": tc, "active": active,
                    "active_idx": act_idx, "flow_tbl": flow})
    return out


def fuzz_batch(rng, n, runtimes, max_runtimes, slot=128, tail_runts=True, misalign=None):
    """Random frames hitting every branch; 16-B aligned shuffled offsets, the
    last frames straddling the end of the buffer (reads past it see 0).
    misalign: None, "mbuf" (every frame at +8, like mbuf data in the
    reference's ingress pool), "mixed" (shifts of 0..15 bytes) or "lineend"
    (shifts of up to 92 bytes, most putting a 128-B line end 40-56 bytes
    into the frame; needs slot >= 256)."""
    ips = [r["ip"] for r in runtimes] or [0x0A000001]
    buf_slots = n + 8
    frames = np.zeros(buf_slots * slot, dtype=np.uint8)
    order = rng.permutation(buf_slots)[:n]
    offs = (order.astype(np.uint64) * slot)
    if misalign == "mbuf":
        offs += np.uint64(8)
    elif misalign == "mixed":
        offs += rng.choice([0, 8, 8, 4, 12, 1, 2, 3, 5, 15], size=n).astype(np.uint64)
    elif misalign == "lineend":
        # first 128-B line ends 40, 48 or 56 bytes into the frame (staged
        # header cut at the line, the rest read on demand), or later
        offs += rng.choice([88, 80, 72, 88, 80, 72, 8, 40, 84, 92], size=n).astype(np.uint64)
    olflags = rng.integers(0, 16, size=n, dtype=np.uint8)
    rss = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    fdir = np.where(rng.random(n) < 0.7,
                    rng.choice([r["uniqid"] for r in runtimes] or [0], size=n),
                    rng.integers(0, max_runtimes + 64, size=n)).astype(np.uint32)
    for i in range(n):
        kind = rng.random()
        dst = int(rng.choice(ips)) if rng.random() < 0.75 else int(rng.integers(0, 2**32))
        src = int(rng.integers(0, 2**32))
        eth = bytes(rng.integers(0, 256, size=12, dtype=np.uint8))
        if kind < 0.55:
            ihl = 5 if rng.random() < 0.6 else int(rng.integers(0, 16))
            ver = 4 if rng.random() < 0.95 else int(rng.integers(0, 16))
            proto = int(rng.choice([6, 17, 6, 17, 1, 47, 132]))
            frag = int(rng.choice([0, 0x4000, 0x4000, 0x2000, 0x0001, 0x1FFF, 0x8000]))
            optlen = max(0, 4 * ihl - 20)
            hdr = struct.pack("!BBHHHBBHII", ver << 4 | ihl, 0, 100, 7, frag, 64, proto, 0, src, dst)
            hdr = hdr[:10] + struct.pack("!H", _csum(hdr)) + hdr[12:]
            opts = bytes(rng.integers(0, 256, size=optlen, dtype=np.uint8))
            l4 = struct.pack("!HH", int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
            fr = eth + b"\x08\x00" + hdr + opts + l4 + bytes(8)
        elif kind < 0.72:
            op = int(rng.choice([1, 2, 3]))
            fr = eth + b"\x08\x06" + struct.pack("!HHBBH", 1, 0x0800, 6, 4, op) + bytes(6) + \
                struct.pack("!I", src) + bytes(6) + struct.pack("!I", dst)
        elif kind < 0.80:
            fr = eth + b"\x86\xdd" + bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
        elif kind < 0.86:
            fr = eth + b"\x81\x00\x00\x05\x08\x00" + bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
        else:
            fr = bytes(rng.integers(0, 256, size=int(rng.integers(14, slot)), dtype=np.uint8))
        fr = fr[:slot - (96 if misalign == "lineend" else 16 if misalign else 0)]
        o = int(offs[i])
        frames[o:o + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
    # loopback hints (tx_pktmbuf_priv.dst_ip): none, a registered IP, or a miss
    u = rng.random(n)
    hint = np.where(u < 0.5, 0, np.where(u < 0.85, rng.choice(ips, size=n),
                                         rng.integers(1, 2**32, size=n))).astype(np.uint32)
    frames_len = frames.nbytes
    if tail_runts and n >= 4:
        # put 3 packets at the very end so their headers straddle frames_len
        last = (buf_slots - 1) * slot
        for j, cut in enumerate((20, 36, 60)):
            offs[n - 1 - j] = last + 16 * j
        frames_len = last + 16 * 2 + 40
        if misalign == "lineend":
            # the line-end cut (8 bytes at last + 120) straddling frames_len
            offs[n - 3] = last + 88
            frames_len = last + 124
    return frames, frames_len, offs, olflags, rss, fdir, hint


def plain_batch(rng, n, runtimes, slot=128):
    """Plain IPv4 frames (Ethertype IPv4, IHL 5: the burst-of-64 loop's lean
    path) with every field that path still decides on varied: UDP/TCP/other
    protocols, fragment fields, any version nibble, registered and unknown
    destinations, ol_flags with and without RSS_HASH (never FDIR), hash.rss.
    Shuffled 16-B aligned offsets; fdir all 0."""
    ips = [r["ip"] for r in runtimes] or [0x0A000001]
    order = rng.permutation(n + 8)[:n]
    offs = order.astype(np.uint64) * np.uint64(slot)
    frames = np.zeros((n + 8) * slot, dtype=np.uint8)
    for i in range(n):
        dst = int(rng.choice(ips)) if rng.random() < 0.8 else int(rng.integers(0, 2**32))
        src = int(rng.integers(0, 2**32))
        ver = 4 if rng.random() < 0.9 else int(rng.integers(0, 16))
        proto = int(rng.choice([6, 17, 6, 17, 1, 47]))
        frag = int(rng.choice([0, 0x4000, 0x4000, 0x2000, 0x0001, 0x8000]))
        hdr = struct.pack("!BBHHHBBHII", ver << 4 | 5, int(rng.integers(0, 256)), 100, 7, frag, 64,
                          proto, 0, src, dst)
        hdr = hdr[:10] + struct.pack("!H", _csum(hdr)) + hdr[12:]
        l4 = struct.pack("!HH", int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
        fr = bytes(rng.integers(0, 256, size=12, dtype=np.uint8)) + b"\x08\x00" + hdr + l4 + bytes(8)
        frames[int(offs[i]):int(offs[i]) + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
    olflags = (rng.integers(0, 16, size=n, dtype=np.uint8) & np.uint8(0xFD))
    rss = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    fdir = np.zeros(n, dtype=np.uint32)
    return frames, offs, olflags, rss, fdir


def to_verdict4(v, thread_count=None):
    """8-B verdicts -> the GCL_CFG_VERDICT4 form: drop the hash.  Every
    DELIVER and WAKE verdict, in either width, carries the flow_tbl slot
    hash % thread_count (rx.c:57, :68); thread_count is not needed since
    the 8-B verdicts already carry it (kept for callers)."""
    from caladan_amd.gclassify import VERDICT4_DTYPE
    out = np.zeros(len(v), dtype=VERDICT4_DTYPE)
    out["uniqid"], out["thread"], out["action"] = v["uniqid"], v["thread"], v["action"]
    return out


def to_verdict2(v, thread_count, thread_bits):
    """8-B verdicts -> the GCL_CFG_VERDICT2 form (include/gclassify.h): u16
    q = uniqid << thread_bits | slot for DELIVER (slot = the flow_tbl slot),
    0x4000 | q for WAKE, 0xC000 | action otherwise."""
    v4 = to_verdict4(v, thread_count)
    act = v4["action"].astype(np.uint32) & 0x3F
    q = v4["uniqid"].astype(np.uint32) << thread_bits | v4["thread"].astype(np.uint32)
    out = np.where(act == 0, q, np.where(act == 1, 0x4000 | q, 0xC000 | act))
    return out.astype(np.uint16)


def to_verdict1(v, thread_count, thread_bits):
    """8-B verdicts -> the GCL_CFG_VERDICT1 form (include/gclassify.h): u8
    q = uniqid << thread_bits | slot for DELIVER and WAKE alike (no wake
    mark), 0x80 | action otherwise."""
    v4 = to_verdict4(v, thread_count)
    act = v4["action"].astype(np.uint32) & 0x3F
    q = v4["uniqid"].astype(np.uint32) << thread_bits | v4["thread"].astype(np.uint32)
    out = np.where((act == 0) | (act == 1), q, 0x80 | act)
    return out.astype(np.uint8)


def load_struct_frames():
    """tests/golden/struct_frames_ref.npz (make_struct_frames.py): (ips,
    frames[n, 64], uniqid, hash, hit), frames written by the reference's
    inc/net structs, hashes by the reference's jenkins_hash."""
    with np.load(os.path.join(GOLDEN, "struct_frames_ref.npz"), allow_pickle=False) as z:
        return z["ips"], z["frames"], z["uniqid"], z["hash"], z["hit"]


def ref_struct_batch(ref, orc, rng, n, R):
    """@n 64-B frames written by the reference's own inc/net structs
    (oracle/ref_host.c ref_build_frame): IPv4 UDP/TCP with IHL 5..11 and
    fragment fields, and ARP requests/replies; 80% to one of @R runtime IPs.
    Returns (ips, frames[n, 64], want) with want[i] = (uniqid or 0xFFFF,
    JENKINS hash of the values put into the structs, hit)."""
    import struct
    ips = [int(x) for x in rng.choice(1 << 31, size=R, replace=False) + (1 << 30)]
    frames = np.zeros((n, 64), dtype=np.uint8)
    want = []
    for i in range(n):
        kind = int(rng.integers(0, 3))
        u = int(rng.integers(0, R))
        hit = rng.random() < 0.8
        dst = ips[u] if hit else int(rng.integers(1, 1 << 30))
        src = int(rng.integers(0, 1 << 32))
        sp, dp = int(rng.integers(0, 1 << 16)), int(rng.integers(0, 1 << 16))
        ihl = int(rng.choice([5, 5, 5, 6, 8, 11]))
        off = int(rng.choice([0, 0, 0, 0x2000, 0x0010, 0x4000]))  # MF, offset, DF
        op = int(rng.choice([1, 2]))
        assert ref.ref_build_frame(frames[i].ctypes.data, kind, src, dst, sp, dp, ihl, off, op) == 0
        if kind == 2 or off & 0x3FFF:
            h = 0
        else:
            h = orc.jhash(struct.pack("<IIHHB", src, dst, dp, sp, 17 if kind == 0 else 6))
        want.append((u if hit else 0xFFFF, h, hit))
    return ips, frames, want
