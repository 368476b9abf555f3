"""Trace ingest: pcap write/load round trips, foreign pcap
variants, errors, and that a replayed trace classifies like the original
batch (CPU oracle)."""
import os
import struct

import numpy as np
import pytest


@pytest.fixture(scope="module")
def g():
    from caladan_amd import gclassify
    return gclassify


def _mixed(orc, n, stride=9216, R=16):
    pl = np.zeros(n, dtype=np.uint16)
    frames, olf, rss = orc.generate(2, n, stride, R, pkt_len=pl)
    return frames, olf, rss, pl


def test_pcap_round_trip(g, orc, tmp_path):
    n, stride = 3000, 9216
    frames, _, _, pl = _mixed(orc, n, stride)
    assert pl.min() >= 60 and pl.max() <= 9014
    ts = np.arange(n, dtype=np.uint64) * 12345 + 7
    path = str(tmp_path / "mixed.pcap")
    g.pcap_write(path, frames, pl, stride=stride, ts_ns=ts)
    assert os.path.getsize(path) == 24 + n * 16 + int(pl.sum())
    t = g.Trace(path)
    assert t.n == n
    assert (t.pkt_len == pl).all() and (t.orig_len == pl).all() and (t.ts_ns == ts).all()
    assert (t.offs % 16 == 0).all() and t.frames.ctypes.data % (1 << 21) == 0
    for i in range(0, n, 97):
        o, L = int(t.offs[i]), int(pl[i])
        assert (t.frames[o:o + L] == frames[i * stride:i * stride + L]).all()
    assert t.frames_len >= int(t.offs[-1]) + int(pl[-1]) + 64
    t2 = g.Trace(path, max_pkts=100)
    assert t2.n == 100 and (t2.offs == t.offs[:100]).all()


def test_pcap_snaplen_cuts_captures(g, orc, tmp_path):
    frames, _, _, pl = _mixed(orc, 200)
    path = str(tmp_path / "snap.pcap")
    g.pcap_write(path, frames, pl, stride=9216, snaplen=128)
    t = g.Trace(path)
    assert (t.pkt_len == np.minimum(pl, 128)).all() and (t.orig_len == pl).all()


def test_pcap_foreign_byte_order_and_usec(g, tmp_path):
    """A big-endian, microsecond pcap as other tools write it."""
    path = str(tmp_path / "be.pcap")
    frames = [bytes(range(60)), bytes(range(100, 180)) + b"\x01\x02"]
    with open(path, "wb") as f:
        f.write(struct.pack(">IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack(">IIII", 100 + i, 250000, len(fr), len(fr)))
            f.write(fr)
    t = g.Trace(path)
    assert t.n == 2 and list(t.pkt_len) == [60, 82]
    assert list(t.ts_ns) == [100 * 10**9 + 250000 * 1000, 101 * 10**9 + 250000 * 1000]
    for i, fr in enumerate(frames):
        o = int(t.offs[i])
        assert bytes(t.frames[o:o + len(fr)]) == fr


def test_pcap_skips_oversized_records(g, tmp_path):
    """Records longer than 65535 bytes (a capture on lo, or GRO/TSO
    super-frames with snaplen 262144) are skipped and counted, the rest of
    the trace loads."""
    path = tmp_path / "lo.pcap"
    small = [bytes(range(64)), bytes(range(64, 164))]
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B23C4D, 2, 4, 0, 0, 262144, 1))
        for i, fr in enumerate([small[0], b"\x07" * 65536, b"\x08" * 200000, small[1]]):
            f.write(struct.pack("<IIII", i, 0, len(fr), len(fr)) + fr)
    t = g.Trace(str(path))
    assert t.n == 2 and t.skipped == 2
    assert list(t.pkt_len) == [64, 100] and list(t.ts_ns) == [0, 3 * 10**9]
    for i, fr in enumerate(small):
        o = int(t.offs[i])
        assert bytes(t.frames[o:o + len(fr)]) == fr
    t1 = g.Trace(str(path), max_pkts=1)
    assert t1.n == 1 and t1.skipped == 0


def test_pcap_errors(g, tmp_path):
    with pytest.raises(OSError) as e:
        g.Trace(str(tmp_path / "missing.pcap"))
    assert e.value.errno == 2
    bad = tmp_path / "bad.pcap"
    bad.write_bytes(b"not a pcap file at all, definitely")
    with pytest.raises(OSError) as e:
        g.Trace(str(bad))
    assert e.value.errno == 71  # EPROTO
    raw = tmp_path / "raw.pcap"   # LINKTYPE_RAW (101) is not Ethernet
    raw.write_bytes(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 101))
    with pytest.raises(OSError):
        g.Trace(str(raw))


def test_replayed_trace_classifies_like_the_batch(g, orc, tmp_path):
    n, R, T = 4000, 16, 8
    frames, olf, rss, pl = _mixed(orc, n, 9216, R)
    path = str(tmp_path / "replay.pcap")
    g.pcap_write(path, frames, pl, stride=9216)
    tr = g.Trace(path)
    t = orc.Tables(R, 1, 0, 0x09)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, orc.steer_flows(T, list(range(r % T + 1))))
    v1, c1, s1 = t.classify(frames, n, 9216, olflags=olf)
    v2, c2, s2 = t.classify(tr.frames, n, 0, offs=tr.offs, olflags=olf, frames_len=tr.frames_len)
    assert (v1 == v2).all() and (c1 == c2).all() and (s1 == s2).all()
