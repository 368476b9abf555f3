"""C-ABI surface checks that need no GPU: every declared symbol is exported,
the host-side C (steer_flows, lrpc, rx_make_cmd, the verdict post-pass) behaves
like the reference functions it replaces."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    from caladan_amd import gclassify
    return gclassify


def declared_functions():
    names = set()
    for h in ("gclassify.h", "gcl_host.h", "gcl_pcap.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(gcl_\w+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol(g):
    names = declared_functions()
    assert len(names) >= 18, names
    lib = ctypes.CDLL(g.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_integration_guide_calls_declared_functions():
    """Every gcl_* function INTEGRATION.md's C calls, and every GCL_* name it
    uses, is declared in include/ (gcl_group.h too), so the guide a
    maintainer copies from cannot drift from the ABI."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = "\n".join(re.findall(r"```c\n(.*?)```", doc, flags=re.S))
    assert code, "no C blocks in INTEGRATION.md"
    hdr = "".join(open(os.path.join(ROOT, "include", h)).read()
                  for h in ("gclassify.h", "gcl_host.h", "gcl_pcap.h", "gcl_group.h"))
    own = set(re.findall(r"#define\s+(GCL_\w+)", code))  # the guide's own macros
    calls = set(re.findall(r"\b(gcl_\w+)\s*\(", code))
    names = set(re.findall(r"\b(GCL_[A-Z0-9_]+)\b", code)) - own
    assert len(calls) >= 10, calls
    missing = sorted(n for n in calls | names if not re.search(r"\b" + n + r"\b", hdr))
    assert not missing, missing


def test_struct_layouts(g):
    assert ctypes.sizeof(g.GclCfg) == 56
    assert ctypes.sizeof(g.GclBatch) == 80
    assert ctypes.sizeof(g.GclVerdict) == 8
    assert ctypes.sizeof(g.GclLrpcMsg) == 16
    assert ctypes.sizeof(g.GclLrpcChanOut) == 32  # struct lrpc_chan_out, lrpc.h:28-35


def test_open_without_gpu_is_enodev(g):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(OSError) as e:
        g.Classifier(0, 16)
    assert e.value.errno in (19, 22)


def test_open_rejects_bad_cfg(g):
    cfg = g.GclCfg(max_runtimes=0)
    ctx = ctypes.c_void_p()
    assert g.lib.gcl_open(0, ctypes.byref(cfg), ctypes.byref(ctx)) == -22
    cfg = g.GclCfg(max_runtimes=4097)
    assert g.lib.gcl_open(0, ctypes.byref(cfg), ctypes.byref(ctx)) == -22
    cfg = g.GclCfg(max_runtimes=16, hash_mode=3)
    assert g.lib.gcl_open(0, ctypes.byref(cfg), ctypes.byref(ctx)) == -22


def test_steer_flows_matches_oracle(g, orc):
    rng = np.random.default_rng(3)
    for _ in range(500):
        tc = int(rng.integers(1, 257))
        act = int(rng.integers(1, tc + 1))
        idx = [int(x) for x in rng.choice(tc, size=act, replace=False)]
        assert g.steer_flows(tc, idx) == orc.steer_flows(tc, idx)
    # sched.c:128-129: no active thread leaves the table untouched
    out = (ctypes.c_uint16 * 4)(7, 7, 7, 7)
    assert g.lib.gcl_steer_flows(4, None, 0, out) == 0 and list(out) == [7, 7, 7, 7]
    # hand example: 8 threads, active [2, 5, 7]
    assert g.steer_flows(8, [2, 5, 7]) == [2, 5, 2, 7, 2, 5, 5, 7]
    with pytest.raises(OSError):
        g.steer_flows(4, [4])
    with pytest.raises(OSError):
        g.steer_flows(300, [1])


def test_loopback_helpers(g):
    # tx.c:81: RSS_HASH iff TXFLAG_LOCAL_HINT (BIT(6), queue.h:42); dma.c:184 csum good
    assert g.lib.gcl_loopback_olflags(1 << 6) == g.F_RSS_HASH | g.F_IP_CKSUM_GOOD
    assert g.lib.gcl_loopback_olflags(1 << 4) == g.F_IP_CKSUM_GOOD
    # queue.h:120-134: the 16-bit hint rides in bits 48..63 of the payload
    assert g.lib.gcl_txpkt_rss((0xBEEF << 48) | 0x123456789A) == 0xBEEF


def test_rx_make_cmd(g):
    # rx.c:24-38: RX_NET_RECV | len << 16 | csum_type << 48
    assert g.lib.gcl_rx_make_cmd(1514, g.F_IP_CKSUM_GOOD) == (1514 << 16) | (1 << 48)
    for f in (g.F_IP_CKSUM_UNKNOWN, g.F_IP_CKSUM_BAD, g.F_IP_CKSUM_NONE):
        assert g.lib.gcl_rx_make_cmd(60, f | g.F_RSS_HASH) == 60 << 16


class Ring:
    def __init__(self, g, size):
        self.tbl = (g.GclLrpcMsg * size)()
        self.wb = ctypes.c_uint32(0)
        self.chan = g.GclLrpcChanOut()
        assert g.lib.gcl_lrpc_init_out(ctypes.byref(self.chan), self.tbl, size, ctypes.byref(self.wb)) == 0
        self.size = size
        self.read = 0

    def drain(self):
        """Consumer: lrpc_recv on the parity bit (lrpc.h:102-127)."""
        out = []
        while True:
            m = self.tbl[self.read & (self.size - 1)]
            parity = 0 if (self.read & self.size) else 1
            if (m.cmd >> 63) != parity:
                break
            out.append((m.cmd & ~(1 << 63), m.payload))
            self.read += 1
        self.wb.value = self.read
        return out


def test_lrpc_ring_semantics(g):
    tbl = (g.GclLrpcMsg * 3)()
    ch = g.GclLrpcChanOut()
    assert g.lib.gcl_lrpc_init_out(ctypes.byref(ch), tbl, 3, None) == -22
    r = Ring(g, 4)
    for i in range(4):
        assert g.lib.gcl_lrpc_send(ctypes.byref(r.chan), i, 100 + i)
    assert not g.lib.gcl_lrpc_send(ctypes.byref(r.chan), 9, 9)  # full
    assert r.drain() == [(i, 100 + i) for i in range(4)]
    for i in range(4):  # second lap flips the parity bit
        assert g.lib.gcl_lrpc_send(ctypes.byref(r.chan), 10 + i, i)
    assert r.drain() == [(10 + i, i) for i in range(4)]


def _host_procs(g, runtimes, ring_size):
    procs, rings, keep = {}, {}, []
    for rt in runtimes:
        p = g.GclHostProc()
        p.uniqid = rt["uniqid"]
        p.thread_count = rt["thread_count"]
        p.active_thread_count = rt["active"]
        p.idle_top = -1 if rt["active"] == rt["thread_count"] else \
            min(set(range(rt["thread_count"])) - set(rt["active_idx"]))
        if rt["flow_tbl"]:
            for i, v in enumerate(rt["flow_tbl"]):
                p.flow_tbl[i] = v
        for th in range(rt["thread_count"]):
            ring = Ring(g, ring_size)
            rings[(rt["uniqid"], th)] = ring
            p.rxq[th] = ctypes.pointer(ring.chan)
        procs[rt["uniqid"]] = p
        keep.append(p)
    return procs, rings, keep


def test_host_deliver_matches_reference_model(g, orc):
    """gcl_host_deliver vs a direct model of rx_send_pkt_to_runtime /
    rx_send_to_runtime (rx.c:50-92) with sched_add_core activating a thread."""
    from tests.rxcases import fuzz_batch, random_runtimes
    rng = np.random.default_rng(11)
    R = 64
    rts = random_runtimes(rng, R, 24, max_threads=6)
    n = 3000
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0, 0x09)
    for r in rts:
        assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
    v, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)

    ring_size = 16
    procs, rings, keep = _host_procs(g, rts, ring_size)
    by_id = (ctypes.c_void_p * R)()
    for u, p in procs.items():
        by_id[u] = ctypes.addressof(p)
    clients = (ctypes.c_void_p * len(procs))(*[ctypes.addressof(p) for p in procs.values()])

    woke = []

    @g.SCHED_ADD_CORE_FN
    def add_core(arg, pp):
        p = pp.contents
        if p.active_thread_count == 0:  # activate thread 0: sched_steer_flows
            p.active_thread_count = 1
            for i in range(p.thread_count):
                p.flow_tbl[i] = 0
            woke.append(p.uniqid)

    freed = []

    @g.FREE_PKT_FN
    def free_pkt(arg, i):
        freed.append(i)

    ops = g.GclHostOps()
    ops.sched_add_core = add_core
    ops.free_pkt = free_pkt
    stats = np.zeros(8, dtype=np.uint64)
    shm = offs.astype(np.uint64)
    delivered = g.lib.gcl_host_deliver(by_id, R, clients, len(procs), v.ctypes.data, pkt_len.ctypes.data,
                                       olf.ctypes.data, 0x09, shm.ctypes.data, n, ctypes.byref(ops),
                                       stats.ctypes.data)

    # model
    active = {r["uniqid"]: r["active"] for r in rts}
    flow = {r["uniqid"]: list(r["flow_tbl"]) if r["flow_tbl"] else [0] * r["thread_count"] for r in rts}
    tc = {r["uniqid"]: r["thread_count"] for r in rts}
    fill = {k: 0 for k in rings}
    expect_msgs = {k: [] for k in rings}
    exp_fail = exp_unh = exp_deliv = 0
    exp_freed = []
    for i in range(n):
        act = v[i]["action"] & 0x3F
        if act in (0, 1):
            u = int(v[i]["uniqid"])
            assert int(v[i]["thread"]) == int(v[i]["hash"]) % tc[u]  # the flow_tbl slot
            if act == 0:
                th = flow[u][int(v[i]["thread"])]
            else:
                if active[u] == 0:
                    active[u] = 1
                    flow[u] = [0] * tc[u]
                th = flow[u][int(v[i]["hash"]) % tc[u]]
            cmd = (int(pkt_len[i]) << 16) | (((int(olf[i]) & 0x0C) == 0x08) << 48)
            if fill[(u, th)] < ring_size:
                fill[(u, th)] += 1
                expect_msgs[(u, th)].append((cmd, int(shm[i])))
                exp_deliv += 1
            else:
                exp_fail += 1
                exp_unh += 1
                exp_freed.append(i)
        else:
            exp_freed.append(i)
    assert delivered == exp_deliv
    assert stats[1] == exp_fail and stats[4] == exp_unh
    assert freed == exp_freed
    for k, ring in rings.items():
        assert ring.drain() == expect_msgs[k], k
    assert len(woke) == len(set(woke))


def test_host_deliver_broadcast_and_arp(g):
    procs, rings, keep = _host_procs(g, [
        {"uniqid": 1, "thread_count": 2, "active": 2, "active_idx": [0, 1], "flow_tbl": [0, 1]},
        {"uniqid": 2, "thread_count": 1, "active": 0, "active_idx": [], "flow_tbl": None},
    ], 4)
    procs[2].idle_top = 0
    by_id = (ctypes.c_void_p * 4)(None, ctypes.addressof(procs[1]), ctypes.addressof(procs[2]), None)
    clients = (ctypes.c_void_p * 2)(ctypes.addressof(procs[1]), ctypes.addressof(procs[2]))
    v = np.zeros(3, dtype=g.VERDICT_DTYPE)
    v[0] = (5, 0xFFFF, 0xFF, g.ACT_BROADCAST)
    v[1] = (0, 0xFFFF, 0xFF, g.ACT_ARP_RESPOND)
    v[2] = (0, 0xFFFF, 0xFF, g.ACT_ARP_RESPOND)
    calls = []

    @g.ARP_RESPOND_FN
    def arp(arg, i):
        calls.append(i)
        return i == 1

    refc = []

    @g.REFCNT_FN
    def refcnt(arg, i, d):
        refc.append((i, d))

    ops = g.GclHostOps()
    ops.arp_respond = arp
    ops.refcnt_update = refcnt
    stats = np.zeros(8, dtype=np.uint64)
    n = g.lib.gcl_host_deliver(by_id, 4, clients, 2, v.ctypes.data, None, None, 0, None, 3,
                               ctypes.byref(ops), stats.ctypes.data)
    assert n == 1
    # rx.c:171-190: one copy to every runtime (the idle one to its idle thread)
    assert rings[(1, 5 % 2)].drain() == [(0, 0)]
    assert rings[(2, 0)].drain() == [(0, 0)]
    assert refc == [(0, 1)]
    # rx.c:200-207: a failed ARP response counts as unregistered + unhandled
    assert calls == [1, 2]
    assert stats[0] == 1 and stats[4] == 1


@pytest.mark.parametrize("R,nrt,forms", [(64, 24, (4, 2, "recs4", "recs2", "recs8")),
                                         (16, 12, (1, "recs1"))])
def test_host_deliver4_matches_deliver(g, orc, R, nrt, forms):
    """Compact verdicts (4, 2 and 1 bytes) replay exactly like 8-B ones: same rings, counters and
    callbacks in the same order with the same packet indices (polls, ownership
    records, frees, ARP responses), including wakes that change the flow_tbl
    mid-batch and broadcasts fanned out with the caller's hashes.  The 1-byte
    form (16 runtimes x 8 queues) carries no WAKE mark: the wakes come from
    the live active count alone."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict1, to_verdict2, to_verdict4
    rng = np.random.default_rng(12)
    rts = random_runtimes(rng, R, nrt, max_threads=6)
    n = 3000
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0x1, 0x09)  # NIC hash, Azure ARP: broadcasts too
    for r in rts:
        assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
    v, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    assert ((v["action"] & 0x3F) == g.ACT_WAKE).any() and ((v["action"] & 0x3F) == g.ACT_BROADCAST).any()
    v4 = to_verdict4(v, {r["uniqid"]: r["thread_count"] for r in rts})
    v2 = to_verdict2(v, {r["uniqid"]: r["thread_count"] for r in rts}, 3)
    v1 = to_verdict1(v, {r["uniqid"]: r["thread_count"] for r in rts}, 3) if R << 3 <= 128 else None
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)
    shm = offs.astype(np.uint64)
    bhash = rss.astype(np.uint32)  # NIC mode: the hash is hash.rss whatever the flags

    def recs(vb):
        """the rx loop's 16-B records (struct gcl_loop_rec) of these verdicts"""
        r = np.zeros(n, dtype=g.LOOP_REC_DTYPE)
        r["ticket"] = 7
        if vb == 8:
            r["hash"], r["verdict"] = v.view(np.uint64) & 0xFFFFFFFF, v.view(np.uint64) >> 32
        else:
            r["hash"] = 0xDEADBEEF  # unused in the compact forms
            r["verdict"] = v4.view(np.uint32) if vb == 4 else v2.astype(np.uint32) if vb == 2 \
                else v1.astype(np.uint32)
        return r

    def run(compact):
        procs, rings, keep = _host_procs(g, rts, 8)
        by_id = (ctypes.c_void_p * R)()
        for u, p in procs.items():
            by_id[u] = ctypes.addressof(p)
        clients = (ctypes.c_void_p * len(procs))(*[ctypes.addressof(p) for p in procs.values()])
        events = []

        @g.SCHED_ADD_CORE_FN
        def add_core(arg, pp):
            p = pp.contents
            if p.active_thread_count == 0:
                p.active_thread_count = 1
                for i in range(p.thread_count):
                    p.flow_tbl[i] = p.thread_count - 1
                events.append(("wake", p.uniqid))

        @g.FREE_PKT_FN
        def free_pkt(arg, i):
            events.append(("free", i))

        @g.REFCNT_FN
        def refcnt(arg, i, d):
            events.append(("ref", i, d))

        @g.OWNED_FN
        def owned(arg, pp, i):
            events.append(("own", pp.contents.uniqid, i))

        @g.ENABLE_POLL_FN
        def poll(arg, pp, th):
            events.append(("poll", pp.contents.uniqid, th))

        @g.ARP_RESPOND_FN
        def arp(arg, i):
            events.append(("arp", i))
            return i % 2 == 0

        ops = g.GclHostOps()
        ops.sched_add_core, ops.free_pkt, ops.refcnt_update = add_core, free_pkt, refcnt
        ops.owned, ops.enable_poll, ops.arp_respond = owned, poll, arp
        stats = np.zeros(8, dtype=np.uint64)
        if isinstance(compact, str):  # "recs<vb>": the records read in place
            vb = int(compact[4:])
            rr = recs(vb)
            d = g.lib.gcl_host_deliver_recs(by_id, R, clients, len(procs), rr.ctypes.data, vb, 3,
                                            bhash.ctypes.data if vb != 8 else None,
                                            pkt_len.ctypes.data, olf.ctypes.data, 0x09,
                                            shm.ctypes.data, n, ctypes.byref(ops), stats.ctypes.data)
        elif compact == 2:
            d = g.lib.gcl_host_deliver2(by_id, R, clients, len(procs), v2.ctypes.data, 3,
                                        bhash.ctypes.data, pkt_len.ctypes.data, olf.ctypes.data,
                                        0x09, shm.ctypes.data, n, ctypes.byref(ops),
                                        stats.ctypes.data)
        elif compact == 1:
            d = g.lib.gcl_host_deliver1(by_id, R, clients, len(procs), v1.ctypes.data, 3,
                                        bhash.ctypes.data, pkt_len.ctypes.data, olf.ctypes.data,
                                        0x09, shm.ctypes.data, n, ctypes.byref(ops),
                                        stats.ctypes.data)
        elif compact == 4:
            d = g.lib.gcl_host_deliver4(by_id, R, clients, len(procs), v4.ctypes.data,
                                        bhash.ctypes.data, pkt_len.ctypes.data, olf.ctypes.data,
                                        0x09, shm.ctypes.data, n, ctypes.byref(ops),
                                        stats.ctypes.data)
        else:
            d = g.lib.gcl_host_deliver(by_id, R, clients, len(procs), v.ctypes.data,
                                       pkt_len.ctypes.data, olf.ctypes.data, 0x09,
                                       shm.ctypes.data, n, ctypes.byref(ops), stats.ctypes.data)
        return d, list(stats), events, {k: r.drain() for k, r in rings.items()}

    full = run(False)
    kinds = {e[0] for e in full[2]}
    assert full[0] > 0 and {"wake", "own", "poll", "free", "ref", "arp"} <= kinds, kinds
    for f in forms:
        assert full == run(f), f


def _live_batch(orc, seed, n=3000, R=64, nrt=24):
    """A NIC-hash, Azure-ARP batch over @nrt random runtimes (some with no
    active thread) classified by the oracle: verdicts in all three widths."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict2, to_verdict4
    rng = np.random.default_rng(seed)
    rts = random_runtimes(rng, R, nrt, max_threads=6)
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0x1, 0x09)
    for r in rts:
        assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
    v, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    tc = {r["uniqid"]: r["thread_count"] for r in rts}
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)
    return rts, v, to_verdict4(v), to_verdict2(v, tc, 3), pkt_len, olf, offs.astype(np.uint64), \
        rss.astype(np.uint32)


@pytest.mark.parametrize("form", [8, 4, 2, "recs8", "recs4", "recs2"])
def test_host_deliver_live_flow_tbl(g, orc, form):
    """The post-pass steers every DELIVER / WAKE verdict through the runtime's
    flow_tbl and active count as they stand when the packet is delivered,
    like rx.c:55-72, not as the device saw them: the sched_add_core of one
    runtime's wake reaches __sched_run's pending branch (sched.c:208-216) and
    disables a kthread of ANOTHER runtime (re-steering it, sched.c:174-192,
    sometimes taking its last core), so that runtime's later packets in the
    same batch follow the new table or take the wake path.  Ring contents,
    counters and every callback equal the serial per-packet model."""
    from tests.schedmodel import Sched, loop_records, make_cprocs, rx_model, run_post_pass
    R, ring = 64, 32
    rts, v, v4, v2, pkt_len, olf, shm, bh = _live_batch(orc, 21)
    order = [r["uniqid"] for r in rts]
    arp_ok = lambda i: i % 2 == 0  # noqa: E731

    S_model = Sched(rts, 5, np.random.default_rng(5))
    want = rx_model(S_model, v, order, ring, pkt_len, olf, shm, bh, arp_ok)
    dis = [e for e in want[2] if e[0] == "disable"]
    # the model really exercises the cross-runtime side effect, to zero too
    assert len(dis) > 20 and any(e[3] == 0 for e in dis), dis[:5]
    assert any(e[1] != w[1] for e, w in zip(want[2], want[2][1:]) if e[0] == "disable")

    S = Sched(rts, 5, np.random.default_rng(5))
    cprocs, rings = make_cprocs(g, S, ring, Ring)
    if isinstance(form, str):
        verd = loop_records(g, v, v4, v2, int(form[4:]))
    else:
        verd = {8: v, 4: v4, 2: v2}[form]
    got = run_post_pass(g, S, cprocs, rings, form, verd, R, order, pkt_len, olf, shm, bh, arp_ok,
                        thread_bits=3)
    assert got[0] == want[0] and got[1] == want[1]
    assert got[2] == want[2]
    assert got[3] == want[3]


def test_host_deliver_snapshot_thread_would_differ(g, orc):
    """The batch of test_host_deliver_live_flow_tbl is one where steering
    from the device's snapshot (flow_tbl as of classification) puts packets
    in different rings: the live read above is observable."""
    from tests.schedmodel import Sched, rx_model
    R, ring = 64, 32
    rts, v, v4, v2, pkt_len, olf, shm, bh = _live_batch(orc, 21)
    order = [r["uniqid"] for r in rts]
    S = Sched(rts, 5, np.random.default_rng(5))
    snap = {u: list(p.flow) for u, p in S.procs.items()}
    snap_active = {u: len(p.active) for u, p in S.procs.items()}
    live = rx_model(S, v, order, ring, pkt_len, olf, shm, bh, lambda i: i % 2 == 0)[3]
    moved = 0
    for i in range(len(v)):
        u = int(v["uniqid"][i])
        if (v["action"][i] & 0x3F) == 0 and snap_active[u]:
            th = snap[u][int(v["thread"][i])]
            msg = (int(pkt_len[i]) << 16 | ((int(olf[i]) & 0x0C) == 0x08) << 48, int(shm[i]))
            moved += msg not in live[(u, th)]
    assert moved > 0


def test_host_deliver_golden_kthreads(g):
    """The hand-derived golden verdicts (tests/golden/rx_scenarios.json, each
    from its rx.c line) through gcl_host_deliver: every DELIVER packet lands
    in the ring of expect_kthread, flow_tbl[hash % thread_count] (rx.c:57),
    and the wake verdicts (no sched_add_core here) in the idle thread's."""
    from tests.rxcases import scenario_batch, scenario_sets
    for s in scenario_sets():
        rts = s["runtimes"]
        R = s["cfg"]["max_runtimes"]
        procs, rings, keep = _host_procs(g, rts, 64)
        by_id = (ctypes.c_void_p * R)()
        for u, p in procs.items():
            by_id[u] = ctypes.addressof(p)
        clients = (ctypes.c_void_p * len(procs))(*[ctypes.addressof(p) for p in procs.values()])
        _, _, _, _, exp, _ = scenario_batch(s)
        n = len(exp)
        shm = np.arange(n, dtype=np.uint64) + 1000
        stats = np.zeros(8, dtype=np.uint64)
        g.lib.gcl_host_deliver(by_id, R, clients, len(procs), exp.ctypes.data, None, None, 0,
                               shm.ctypes.data, n, None, stats.ctypes.data)
        seen = {}
        for (u, th), ring in rings.items():
            for _, pay in ring.drain():
                seen[int(pay) - 1000] = (u, th)
        for i, pk in enumerate(s["packets"]):
            a = pk["expect"]["action"] & 0x3F
            if a == g.ACT_DELIVER:
                assert seen[i] == (pk["expect"]["uniqid"], pk["expect_kthread"]), (s["name"], pk["cite"])
            elif a == g.ACT_WAKE:
                u = pk["expect"]["uniqid"]
                assert seen[i] == (u, procs[u].idle_top), (s["name"], pk["cite"])


@pytest.mark.parametrize("meta", ["all", "no_olflags", "none"])
def test_host_deliver4_fast_path(g, orc, meta):
    """With no callbacks gcl_host_deliver4 takes its DELIVER fast path; it must
    fill the same rings in the same order as the generic replay of the 8-B
    verdicts, with the full rings (8 deep here) and the non-DELIVER verdicts
    handed back to the generic code packet by packet."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict4
    rng = np.random.default_rng(13)
    R = 64
    rts = random_runtimes(rng, R, 24, max_threads=6)
    n = 3000
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0x1, 0x09)
    for r in rts:
        assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
    v, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    v4 = to_verdict4(v, {r["uniqid"]: r["thread_count"] for r in rts})
    assert ((v4["action"] & 0x3F) == g.ACT_DELIVER).sum() > n // 3
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)
    shm = offs.astype(np.uint64)
    bhash = rss.astype(np.uint32)
    pl = None if meta == "none" else pkt_len.ctypes.data
    of = olf.ctypes.data if meta == "all" else None
    sp = None if meta == "none" else shm.ctypes.data

    def run(compact):
        procs, rings, keep = _host_procs(g, rts, 8)
        for p in procs.values():
            if p.active_thread_count == 0 and p.thread_count > 1:
                p.idle_top = 1
        by_id = (ctypes.c_void_p * R)()
        for u, p in procs.items():
            by_id[u] = ctypes.addressof(p)
        clients = (ctypes.c_void_p * len(procs))(*[ctypes.addressof(p) for p in procs.values()])
        stats = np.zeros(8, dtype=np.uint64)
        if compact == "recs":  # the fast path over 16-B loop records, in place
            # (after the wait-time hint on the rings, which changes nothing)
            g.lib.gcl_host_prefetch_rxq(clients, len(procs))
            rr = np.zeros(n, dtype=g.LOOP_REC_DTYPE)
            rr["verdict"] = v4.view(np.uint32)
            d = g.lib.gcl_host_deliver_recs(by_id, R, clients, len(procs), rr.ctypes.data, 4, 0,
                                            bhash.ctypes.data, pl, of, 0x09, sp, n, None,
                                            stats.ctypes.data)
        elif compact == 4:
            d = g.lib.gcl_host_deliver4(by_id, R, clients, len(procs), v4.ctypes.data,
                                        bhash.ctypes.data, pl, of, 0x09, sp, n, None,
                                        stats.ctypes.data)
        else:
            d = g.lib.gcl_host_deliver(by_id, R, clients, len(procs), v.ctypes.data, pl, of, 0x09,
                                       sp, n, None, stats.ctypes.data)
        return d, list(stats), {k: r.drain() for k, r in rings.items()}

    full, compact = run(False), run(True)
    assert full[0] > 0 and full[1][1] > 0  # deliveries and ring-full failures both happen
    assert full == compact
    assert full == run("recs")


def test_dev_alloc_paired_rejects_bad_args(g):
    """Argument checks come before any HIP call (no GPU needed)."""
    out = ctypes.c_void_p()
    f = g.lib.gcl_dev_alloc_paired
    assert f(0, 1 << 20, None, 1 << 20, g.PAIR_NEW_READS, ctypes.byref(out), None) == -22
    assert f(0, 0, 4096, 1 << 20, g.PAIR_NEW_READS, ctypes.byref(out), None) == -22
    assert f(0, 1 << 20, 4096, 1 << 20, 0, ctypes.byref(out), None) == -22
    assert f(0, 1 << 20, 4096, 1 << 20, 3, ctypes.byref(out), None) == -22
    assert f(0, 1 << 20, 4096, 1 << 20, g.PAIR_NEW_READS, None, None) == -22
    # the read side must hold one 256-packet tile of 64-B granules
    assert f(0, 1 << 13, 4096, 1 << 20, g.PAIR_NEW_READS, ctypes.byref(out), None) == -22


def test_rxloop_rejects_bad_args(g):
    """The persistent-loop entry points validate before touching the GPU."""
    out = ctypes.c_void_p()
    cfg = g.GclRxloopCfg(slots=64, max_burst=64, workers=1, lifetime_ms=1000, region=4096,
                         region_len=1 << 20)
    assert g.lib.gcl_rxloop_start(None, ctypes.byref(cfg), ctypes.byref(out)) == -22
    assert g.lib.gcl_rxloop_submit(None, 1, 4096, None, None, None, None) == -22
    assert g.lib.gcl_rxloop_wait(None, 1, None, 0) == -22
    assert g.lib.gcl_rxloop_stop(None) == -22
    assert g.lib.gcl_rxloop_drive(None, 1, 4096, 1, 1, None, None) == -22
    cnt = np.zeros(3, dtype=np.uint64)
    assert g.lib.gcl_rxloop_poll_stats(None, cnt.ctypes.data) == -22
    assert g.lib.gcl_rxloop_lean_bursts(None, cnt.ctypes.data) == -22
    assert ctypes.sizeof(g.GclRxloopCfg) == 56


def test_verdict2_widening(g, orc):
    """gcl_verdict2_to4 inverts the 2-byte encoding: every oracle verdict of a
    fuzz batch, narrowed to u16 and widened again, is its gcl_verdict4 minus
    the GCL_ACT_F_FDIR / F_TRANS flags."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict2, to_verdict4
    rng = np.random.default_rng(14)
    for R, tb in [(64, 4), (1024, 4), (16, 0), (16, 8)]:
        rts = random_runtimes(rng, R, min(R, 40), max_threads=1 << tb)
        frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, 2000, rts, R)
        t = orc.Tables(R, 0, 0x1, 0x09)
        for r in rts:
            assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
        v, _, _ = t.classify(frames, 2000, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                             frames_len=flen, dst_hint=hint)
        tc = {r["uniqid"]: r["thread_count"] for r in rts}
        v4, v2 = to_verdict4(v, tc), to_verdict2(v, tc, tb)
        assert len(set((v4["action"] & 0x3F).tolist())) >= 4
        w = np.array([g.lib.gcl_verdict2_to4(int(x), tb) for x in v2], dtype=np.uint32)
        assert (w & 0xFFFF == v4["uniqid"]).all()
        assert (w >> 16 & 0xFF == v4["thread"]).all()
        assert (w >> 24 == v4["action"] & 0x3F).all()


@pytest.mark.parametrize("form", [1, "recs1"])
def test_host_deliver1_live_flow_tbl(g, orc, form):
    """test_host_deliver_live_flow_tbl for the 1-byte verdicts (16 runtimes
    x 8 queues): no WAKE mark in the verdict, the wakes and the re-steered
    runtimes come from the live flow_tbl and active count alone, and every
    ring, counter and callback equals the serial per-packet model."""
    from tests.rxcases import to_verdict1
    from tests.schedmodel import Sched, loop_records, make_cprocs, rx_model, run_post_pass
    R, ring = 16, 32
    rts, v, v4, v2, pkt_len, olf, shm, bh = _live_batch(orc, 23, R=R, nrt=12)
    v1 = to_verdict1(v, {r["uniqid"]: r["thread_count"] for r in rts}, 3)
    order = [r["uniqid"] for r in rts]
    arp_ok = lambda i: i % 2 == 0  # noqa: E731
    want = rx_model(Sched(rts, 5, np.random.default_rng(5)), v, order, ring, pkt_len, olf, shm, bh, arp_ok)
    assert any(e[0] == "disable" for e in want[2])
    assert ((v["action"] & 0x3F) == g.ACT_WAKE).any()
    S = Sched(rts, 5, np.random.default_rng(5))
    cprocs, rings = make_cprocs(g, S, ring, Ring)
    verd = loop_records(g, v, v4, v2, 1, v1) if isinstance(form, str) else v1
    got = run_post_pass(g, S, cprocs, rings, form, verd, R, order, pkt_len, olf, shm, bh, arp_ok,
                        thread_bits=3)
    assert got == want


def test_verdict1_roundtrip(g, orc):
    """gcl_verdict1_to4 inverts the 1-byte encoding: every oracle verdict of a
    fuzz batch, narrowed to u8 and widened again, is its gcl_verdict4 with
    WAKE read as DELIVER (the post-pass decides the wake) and the FDIR /
    TRANS flags dropped."""
    from tests.rxcases import fuzz_batch, random_runtimes, to_verdict1, to_verdict4
    rng = np.random.default_rng(15)
    for R, tb in [(16, 3), (32, 2), (128, 0), (1, 7)]:
        rts = random_runtimes(rng, R, min(R, 40), max_threads=1 << tb)
        frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, 2000, rts, R)
        t = orc.Tables(R, 0, 0x1, 0x09)
        for r in rts:
            assert t.runtime_set(r["uniqid"], r["ip"], r["thread_count"], r["active"], r["flow_tbl"]) == 0
        v, _, _ = t.classify(frames, 2000, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                             frames_len=flen, dst_hint=hint)
        tc = {r["uniqid"]: r["thread_count"] for r in rts}
        v4, v1 = to_verdict4(v, tc), to_verdict1(v, tc, tb)
        w = np.array([g.lib.gcl_verdict1_to4(int(x), tb) for x in v1], dtype=np.uint32)
        act = v4["action"] & 0x3F
        assert (w & 0xFFFF == v4["uniqid"]).all()
        assert (w >> 16 & 0xFF == v4["thread"]).all()
        assert (w >> 24 == np.where(act == g.ACT_WAKE, g.ACT_DELIVER, act)).all()


def test_open_rejects_bad_verdict1_cfg(g):
    """Checked before the device: past 128 queues, thread_bits > 7, or
    combined with VERDICT2 / VERDICT4 / TRANS_HASH."""
    ctx = ctypes.c_void_p()
    for flags, R, tb in [(g.CFG_VERDICT1, 32, 3), (g.CFG_VERDICT1, 1, 8), (g.CFG_VERDICT1, 129, 0),
                         (g.CFG_VERDICT1 | g.CFG_VERDICT2, 16, 3),
                         (g.CFG_VERDICT1 | g.CFG_VERDICT4, 16, 3),
                         (g.CFG_VERDICT1 | g.CFG_TRANS_HASH, 16, 3)]:
        cfg = g.GclCfg(max_runtimes=R, hash_mode=1, flags=flags, thread_bits=tb)
        assert g.lib.gcl_open(0, ctypes.byref(cfg), ctypes.byref(ctx)) == -22, (flags, R, tb)


def test_open_rejects_bad_verdict2_cfg(g):
    """Checked before the device: past 16 Ki queues, thread_bits > 8, or
    combined with VERDICT4 / TRANS_HASH."""
    ctx = ctypes.c_void_p()
    for flags, R, tb in [(g.CFG_VERDICT2, 4096, 3), (g.CFG_VERDICT2, 16, 9),
                         (g.CFG_VERDICT2, 2048, 4),
                         (g.CFG_VERDICT2 | g.CFG_VERDICT4, 16, 2),
                         (g.CFG_VERDICT2 | g.CFG_TRANS_HASH, 16, 2)]:
        cfg = g.GclCfg(max_runtimes=R, hash_mode=1, flags=flags, thread_bits=tb)
        assert g.lib.gcl_open(0, ctypes.byref(cfg), ctypes.byref(ctx)) == -22, (flags, R, tb)
    assert g.thread_bits_for(16, 8) == 3 and g.thread_bits_for(1024, 4) == 2
    assert g.thread_bits_for(1024, 16) == 4 and g.thread_bits_for(1024, 17) is None
    assert g.thread_bits_for(16, 1) == 0 and g.thread_bits_for(16, 256) == 8


def test_python_constants_match_header_defines(g):
    """Every integer #define GCL_<NAME> in include/*.h that the ctypes
    binding mirrors as gclassify.<NAME> (flags, modes, counters, loop and
    group options) has the same value, so a flag added on one side only
    cannot drift."""
    defs = {}
    for h in ("gclassify.h", "gcl_host.h", "gcl_pcap.h", "gcl_group.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        for m in re.finditer(r"^#define\s+GCL_(\w+)\s+\(?(0x[0-9A-Fa-f]+|\d+)u?\)?\s*(?:/\*.*)?$", src, re.M):
            defs[m.group(1)] = int(m.group(2), 0)
    mirrored = {k: v for k, v in defs.items() if hasattr(g, k)}
    assert len(mirrored) >= 25 and "LOOP_HDR_RECORDS" in mirrored, sorted(mirrored)
    bad = {k: (v, getattr(g, k)) for k, v in mirrored.items() if getattr(g, k) != v}
    assert not bad, bad


def test_tune_struct_and_defaults(g):
    """struct gcl_tune (the tests' and tools' overrides since the library
    stopped reading GCL_TUNE_* from the environment): the layout the header
    declares, every field GCL_TUNE_AUTO after gcl_tune_init, and
    gcl_ctx_tune refusing a NULL context."""
    assert ctypes.sizeof(g.GclTune) == 96
    t = g.make_tune()
    assert t.size == 96 and t.loop_t0 == 0 and t.debug == 0
    for name, _ in g.GclTune._fields_:
        if name not in ("size", "loop_t0", "debug", "pad"):
            assert getattr(t, name) == g.TUNE_AUTO, name
    t = g.make_tune(defer=2, threads=512, loop_phase=(120, 8, 1))
    assert (t.defer, t.threads, t.loop_phase_max, t.loop_phase_up, t.loop_phase_down) == (2, 512, 120, 8, 1)
    with pytest.raises(AttributeError):
        g.make_tune(no_such_knob=1)
    assert g.lib.gcl_ctx_tune(None, ctypes.byref(t)) == -22
    assert g.lib.gcl_abi_version() == 6


def test_library_reads_no_environment(g):
    """No getenv anywhere in the product's sources, and neither library
    imports one: production behaviour cannot be changed from the
    environment; overrides go through gcl_ctx_tune."""
    import subprocess
    csrc = os.path.join(ROOT, "caladan_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(csrc, f)).read(), flags=re.S)
        assert "getenv" not in src, f
    for so in (g.LIB_PATH, g.GROUP_LIB_PATH):
        if not os.path.exists(so):
            continue
        und = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True).stdout
        assert not re.search(r"\b(secure_)?getenv\b", und), so
