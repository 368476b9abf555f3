"""The host C of the rx path (caladan_amd/csrc/gcl_host.c) against the
reference's own code, compiled unmodified into oracle/_ref/libhost_ref.so
(base/lrpc.c plus the header-only lrpc_send / lrpc_recv, union rxq_cmd and
loopback hint helpers, exported by oracle/ref_host.c):

* the lrpc ring: the same bytes, parities and full-ring refusals as the
  reference's lrpc_send / __lrpc_send (inc/base/lrpc.h:48-63,
  base/lrpc.c:10-27) over random send/drain interleavings, and rings filled
  by gcl_host_deliver4 read back by the reference's lrpc_recv;
* the layouts of struct lrpc_msg / lrpc_chan_out, which the boundary shares;
* rx_make_cmd's union rxq_cmd encoding (rx.c:24-38, queue.h:10-65);
* the loopback hint payload (queue.h:120-134) and TXFLAG_LOCAL_HINT;
* NCPU.

Skipped where the reference tree was not mounted at build time."""
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def ref(orc):
    r = orc.ref_host()
    if r is None:
        pytest.skip("oracle/_ref/libhost_ref.so not built (reference tree absent)")
    return r


@pytest.fixture(scope="module")
def g():
    from caladan_amd import gclassify
    return gclassify


class ChanIn(ctypes.Structure):
    """struct lrpc_chan_in (inc/base/lrpc.h:112-117)"""
    _fields_ = [("tbl", ctypes.c_void_p), ("recv_head_wb", ctypes.c_void_p),
                ("recv_head", ctypes.c_uint32), ("size", ctypes.c_uint32)]


def test_lrpc_layouts(g, ref):
    out = (ctypes.c_uint64 * 10)()
    ref.ref_lrpc_layout(out)
    M, C = g.GclLrpcMsg, g.GclLrpcChanOut
    assert list(out) == [ctypes.sizeof(M), M.cmd.offset, M.payload.offset, ctypes.sizeof(C),
                         C.send_head.offset, C.send_tail.offset, C.tbl.offset,
                         C.recv_head_wb.offset, C.size.offset, C.pad.offset]


class Ring:
    """One producer channel over its own table, with the reference's
    consumer (lrpc_init_in + lrpc_recv) draining it."""

    def __init__(self, g, ref, size, ours):
        self.tbl = (g.GclLrpcMsg * size)()
        self.wb = ctypes.c_uint32(0)
        self.out = g.GclLrpcChanOut()
        self.inn = ChanIn()
        init = g.lib.gcl_lrpc_init_out if ours else ref.lrpc_init_out
        assert init(ctypes.byref(self.out), self.tbl, size, ctypes.byref(self.wb)) == 0
        assert ref.lrpc_init_in(ctypes.byref(self.inn), self.tbl, size, ctypes.byref(self.wb)) == 0
        self.send = (lambda c, p: bool(g.lib.gcl_lrpc_send(ctypes.byref(self.out), c, p))) if ours \
            else (lambda c, p: bool(ref.ref_lrpc_send(ctypes.byref(self.out), c, p)))
        self.ref = ref

    def drain(self, k):
        got = []
        cmd, pay = ctypes.c_uint64(), ctypes.c_ulong()
        for _ in range(k):
            if not self.ref.ref_lrpc_recv(ctypes.byref(self.inn), ctypes.byref(cmd), ctypes.byref(pay)):
                break
            got.append((cmd.value, pay.value))
        return got

    def raw(self):
        return bytes(self.tbl)


@pytest.mark.parametrize("size", [1, 4, 64])
def test_lrpc_send_matches_reference(g, ref, size):
    rng = np.random.default_rng(size)
    a, b = Ring(g, ref, size, ours=True), Ring(g, ref, size, ours=False)
    sent = full = 0
    for step in range(4000):
        if rng.random() < 0.75:
            cmd = int(rng.integers(0, 1 << 63))
            pay = int(rng.integers(0, 1 << 63))
            ra, rb = a.send(cmd, pay), b.send(cmd, pay)
            assert ra == rb, step
            sent += ra
            full += not ra
        else:
            k = int(rng.integers(0, 3)) if rng.random() < 0.9 else size + 1
            assert a.drain(k) == b.drain(k), step
        assert a.raw() == b.raw(), step
        assert (a.out.send_head, a.out.send_tail) == (b.out.send_head, b.out.send_tail), step
    assert sent > 500 and full > 10


def test_lrpc_rejects_non_power_of_two(g, ref):
    for size in (0, 3, 6, 100):
        t = (g.GclLrpcMsg * 128)()
        wb = ctypes.c_uint32()
        ca, cb = g.GclLrpcChanOut(), g.GclLrpcChanOut()
        ra = g.lib.gcl_lrpc_init_out(ctypes.byref(ca), t, size, ctypes.byref(wb))
        rb = ref.lrpc_init_out(ctypes.byref(cb), t, size, ctypes.byref(wb))
        assert ra == rb, size


def test_rxq_cmd_matches_reference(g, ref):
    rng = np.random.default_rng(5)
    for _ in range(2000):
        n = int(rng.integers(0, 1 << 16))
        fl = int(rng.integers(0, 256))
        good = (fl & g.F_IP_CKSUM_MASK) == g.F_IP_CKSUM_GOOD
        assert g.lib.gcl_rx_make_cmd(n, fl) == ref.ref_rxq_cmd(n, int(good))


def test_loopback_hint_matches_reference(g, ref):
    rng = np.random.default_rng(6)
    for _ in range(2000):
        ptr = int(rng.integers(0, 1 << 48))
        rss = int(rng.integers(0, 1 << 16))
        p = ref.ref_txpkt_to_payload(ptr, rss)
        assert g.lib.gcl_txpkt_rss(p) == ref.ref_rss_from_txpkt_payload(p) == rss
    hint = ref.ref_txflag_local_hint()
    assert g.lib.gcl_loopback_olflags(hint) & g.F_RSS_HASH
    assert not g.lib.gcl_loopback_olflags(0xFF & ~hint) & g.F_RSS_HASH
    assert g.GCL_NCPU == ref.ref_ncpu()


def test_deliver_rings_read_by_reference_consumer(g, ref, orc):
    """Rings filled by gcl_host_deliver4 (its DELIVER fast path and the
    generic replay) read back through the reference's lrpc_recv: every
    message is the reference's rxq_cmd for that packet with its shmptr."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict4
    rng = np.random.default_rng(15)
    R = 32
    rts = random_runtimes(rng, R, 20, max_threads=8)
    n = 2000
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0, 0x09)
    for r in rts:
        assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
    v, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    v4 = to_verdict4(v, {r["uniqid"]: r["thread_count"] for r in rts})
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)
    shm = offs.astype(np.uint64)
    procs, rings, keep = {}, {}, []
    for rt in rts:
        p = g.GclHostProc()
        p.uniqid, p.thread_count, p.active_thread_count = rt["uniqid"], rt["thread_count"], rt["active"]
        p.idle_top = 0 if rt["active"] == 0 else -1
        for i, x in enumerate(rt["flow_tbl"] or []):
            p.flow_tbl[i] = x
        for th in range(rt["thread_count"]):
            ring = Ring(g, ref, 4096, ours=True)
            rings[(rt["uniqid"], th)] = ring
            p.rxq[th] = ctypes.pointer(ring.out)
        procs[rt["uniqid"]] = p
        keep.append(p)
    by_id = (ctypes.c_void_p * R)()
    for u, p in procs.items():
        by_id[u] = ctypes.addressof(p)
    clients = (ctypes.c_void_p * len(procs))(*[ctypes.addressof(p) for p in procs.values()])
    stats = np.zeros(8, dtype=np.uint64)
    d = g.lib.gcl_host_deliver4(by_id, R, clients, len(procs), v4.ctypes.data, None,
                                pkt_len.ctypes.data, olf.ctypes.data, 0x09, shm.ctypes.data, n,
                                None, stats.ctypes.data)
    # expected: DELIVER to flow_tbl[slot], WAKE (no sched_add_core here) to
    # the idle thread, in packet order per ring
    want = {k: [] for k in rings}
    for i in range(n):
        a = int(v4["action"][i]) & 0x3F
        if a not in (g.ACT_DELIVER, g.ACT_WAKE):
            continue
        u = int(v4["uniqid"][i])
        th = procs[u].flow_tbl[int(v4["thread"][i])] if a == g.ACT_DELIVER else procs[u].idle_top
        good = (int(olf[i]) & g.F_IP_CKSUM_MASK) == g.F_IP_CKSUM_GOOD
        want[(u, th)].append((ref.ref_rxq_cmd(int(pkt_len[i]), int(good)), int(shm[i])))
    assert d == sum(len(x) for x in want.values()) > n // 3
    for k, ring in rings.items():
        assert ring.drain(5000) == want[k], k


def test_protocol_constants_match_reference(ref):
    """The kernel's ethertype / ARP opcode constants (include/gclassify.h)
    are the reference's (ethernet.h:88,94,300, arp.h:42-43)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "gclassify.h")).read()
    d = {m.group(1): int(m.group(2), 0)
         for m in re.finditer(r"#define\s+GCL_(ETHTYPE_\w+|ARP_OP_\w+)\s+(0x[0-9A-Fa-f]+|\d+)", src)}
    c = (ctypes.c_uint32 * 6)()
    ref.ref_net_consts(c)
    assert [d["ETHTYPE_IP"], d["ETHTYPE_ARP"], d["ETHTYPE_IPV6"], d["ARP_OP_REQUEST"],
            d["ARP_OP_REPLY"]] == list(c)[:5]
    assert c[5] == 0x3FFF  # IP_MF | IP_OFFMASK: what "is a fragment" tests


def test_parse_offsets_match_reference_structs(g, ref, orc):
    """Frames written through the reference's own struct eth_hdr / ip_hdr /
    udp_hdr / tcp_hdr / arp_hdr(_ethip) classify as the values put into the
    structs say: the destination (daddr, or the ARP target) picks the
    runtime, and the JENKINS flow hash is lookup3 over {saddr, daddr, dport,
    sport, proto} as set, 0 for fragments and ARP.  The GPU is bit-exact
    with the oracle (tests/test_gpu_parity.py), so this pins both."""
    from tests.rxcases import ref_struct_batch
    rng = np.random.default_rng(16)
    R, n = 64, 3000
    ips, frames, want = ref_struct_batch(ref, orc, rng, n, R)
    t = orc.Tables(R, 1, 0, 0x09)
    for u, ip in enumerate(ips):
        assert t.runtime_set(u, ip, 4, 4, [0, 1, 2, 3]) == 0
    v, _, _ = t.classify(frames.reshape(-1), n, 64)
    for i, (u, h, hit) in enumerate(want):
        assert int(v["uniqid"][i]) == u, i
        if hit:
            assert int(v["action"][i]) & 0x3F == g.ACT_DELIVER, i
            assert int(v["hash"][i]) == h, i
            assert int(v["thread"][i]) == h % 4, i
        else:
            assert int(v["action"][i]) & 0x3F == g.ACT_DROP_UNREG, i


def test_struct_frames_fixture_matches_oracle(g, orc):
    """The committed struct-frame fixture (tests/golden/struct_frames_ref.npz,
    frames from the reference's inc/net structs, hashes from its
    jenkins_hash) classifies on the oracle as it records: what the GPU test
    checks without loading anything built from reference sources."""
    from tests.rxcases import load_struct_frames
    ips, frames, uniq, hashes, hit = load_struct_frames()
    R, n = 64, len(frames)
    t = orc.Tables(R, 1, 0, 0x09)
    for u, ip in enumerate(ips):
        assert t.runtime_set(u, int(ip), 4, 4, [0, 1, 2, 3]) == 0
    v, _, _ = t.classify(frames.reshape(-1), n, 64)
    assert (v["uniqid"] == uniq).all()
    assert (v["hash"][hit] == hashes[hit]).all()
    assert (v["thread"][hit] == hashes[hit] % 4).all()
    assert ((v["action"][~hit] & 0x3F) == g.ACT_DROP_UNREG).all()


def test_struct_frames_fixture_regenerates(ref, orc):
    """With the reference mounted, make_struct_frames.py's recipe reproduces
    the committed fixture exactly."""
    import types
    from tests.rxcases import load_struct_frames, ref_struct_batch
    rj = orc.ref_jhash()
    if rj is None:
        pytest.skip("oracle/_ref/libjhash_ref.so not built")
    refj = types.SimpleNamespace(jhash=lambda b: int(rj.jenkins_hash(b, len(b))))
    ips, frames, want = ref_struct_batch(ref, refj, np.random.default_rng(17), 3000, 64)
    f_ips, f_frames, f_uniq, f_hash, f_hit = load_struct_frames()
    assert (np.array(ips, dtype=np.uint32) == f_ips).all()
    assert (frames == f_frames).all()
    assert [w[0] for w in want] == f_uniq.tolist()
    assert [w[1] for w in want] == f_hash.tolist()
