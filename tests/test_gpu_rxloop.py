"""GPU parity of the persistent rx loop (gcl_rxloop_*): bursts of <= 64
mbufs (IOKERNEL_RX_BURST_SIZE, iokernel/defs.h:75) classified by a persistent
kernel straight from a registered host region, bit-exact against the oracle
run over the same packets, including table changes between bursts, recycled
mbufs (the same addresses rewritten by the CPU), several workers and a full
ring."""
import time

import numpy as np
import pytest

from tests.rxcases import (apply_runtimes, fuzz_batch, plain_batch, random_runtimes, to_verdict1,
                           to_verdict2, to_verdict4)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def g():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from caladan_amd import gclassify
    return gclassify


def bursts(n, size=64):
    return [(s, min(n, s + size)) for s in range(0, n, size)]


def want(ve, tc, vb, tb=4):
    return to_verdict1(ve, tc, tb) if vb == 1 else to_verdict2(ve, tc, tb) if vb == 2 \
        else to_verdict4(ve, tc) if vb == 4 else ve


LOOP_FLAGS = (lambda g: 0, lambda g: g.LOOP_INLINE_HDRS, lambda g: g.LOOP_HDR_RECORDS)


def tc_map(rts, max_rt):
    tc = np.ones(max_rt, dtype=np.int64)
    for r in rts:
        tc[r["uniqid"]] = r["thread_count"]
    return tc


def poll_stats_settled(loop, nb, timeout_s=2.0):
    """The loop's poll counters once all @nb bursts are in them: the writer
    wave posts them after the bursts' verdict records (gclassify.h), so they
    may lag the last wait by a few microseconds."""
    deadline = time.monotonic() + timeout_s
    ps = loop.poll_stats()
    while sum(ps.values()) < nb and time.monotonic() < deadline:
        time.sleep(0.001)
        ps = loop.poll_stats()
    return ps


LOOP_CASES = [(m, vb, 0, 0) for m in (0, 1, 2) for vb in (8, 4, 2)] + \
    [(m, 8, fl, 0) for m in (0, 1, 2) for fl in (1, 2)] + \
    [(0, 8, 1, 1), (1, 4, 0, 1), (2, 8, 2, 1), (1, 2, 1, 1)] + \
    [(m, vb, 0, 2) for m in (0, 1, 2) for vb in (8, 4, 2)] + [(0, 8, 1, 2), (2, 8, 2, 2)] + \
    [(m, 1, 0, i) for m in (0, 2) for i in (0, 1, 2)] + [(0, 1, 1, 2), (2, 1, 2, 0)]


# Python takes longer than the loop's default speculative window (4 us, 1 ms
# with <= 2 workers) between bursts: tests that want every burst of <= 64
# taken with its poll (offsets or header records current at the first poll,
# or re-read after a stale one) open it to 1 s (gcl_tune.loop_spec, 10-ns
# ticks), so that a burst is never "late" however Python paces the submits
SPEC_WIDE = 100_000_000


@pytest.mark.parametrize("k64", [1, 0])
@pytest.mark.parametrize("mode,vb,flags,inline", LOOP_CASES)
def test_rxloop_fuzz_vs_oracle(g, orc, mode, vb, flags, inline, k64):
    """k64: bursts of <= 64 through rxloop64_kernel (the default for
    max_burst <= 64), or through the general loop kernel (gcl_tune.loop64 = 0);
    vb: verdict bytes (8 gcl_verdict, 4 VERDICT4, 2 VERDICT2, 1 VERDICT1 with
    16 runtimes x up to 8 kthreads);
    flags: 0 plain, 1 Azure ARP mode (GCL_CFG_AZURE_ARP), 2 16-bit hash;
    inline: 1 header granules copied into the ring slot (GCL_LOOP_INLINE_HDRS),
    2 stamped header records (GCL_LOOP_HDR_RECORDS), including the frames that
    straddle the end of the region and IPv4 options past byte 43."""
    rng = np.random.default_rng(7000 + 10 * mode + vb + 100 * flags + 1000 * inline)
    max_rt = 1024 if mode == 1 and vb != 1 else 16
    rts = random_runtimes(rng, max_rt, 300 if max_rt == 1024 else 12, max_threads=8 if vb == 1 else 16)
    tb = 3 if vb == 1 else 4
    n = 3000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    cflags = {8: 0, 4: g.CFG_VERDICT4, 2: g.CFG_VERDICT2, 1: g.CFG_VERDICT1}[vb] | flags
    t = orc.Tables(max_rt, mode, flags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, cflags, 0x09, key, thread_bits=tb)
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    g.host_register(frames)
    cnt = torch.zeros(max_rt, dtype=torch.int64, device="cuda")
    st = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    # the zero fills run on torch's stream, the loop on a stream of its own:
    # done before the loop adds to them (gcl_rxloop_start also orders the
    # default stream's work first)
    torch.cuda.synchronize()
    # header records, and the offsets of the NIC-mode cases, taken with the
    # poll (see the ragged-burst test); the other cases read after the word
    early = inline == 2 or (inline == 0 and mode == 0)
    # header records: the submitting core's header prefetch distance
    # (gcl_tune.rec_prefetch) none, one, the whole burst and the default
    pf = {"rec_prefetch": {8: 0, 4: 1, 2: 64}.get(vb, g.TUNE_AUTO)} if inline == 2 else {}
    # and the next slot taken for writing during a wait (gcl_tune.slot_prefetch)
    pf["slot_prefetch"] = {8: 1, 2: 1, 4: 0}.get(vb, g.TUNE_AUTO)
    clf.tune(loop64=k64, **({"loop_spec": SPEC_WIDE} if early else {}), **pf)
    loop = clf.rxloop(frames, slots=8, counts=cnt, stats=st, region_len=flen,
                      flags=LOOP_FLAGS[inline](g))
    try:
        got = []
        for k, (a, b) in enumerate(bursts(n)):
            tk = loop.submit(offs[a:b], olf[a:b], rss[a:b], fdir[a:b], hint[a:b])
            assert tk > 0
            if k % 2 == 0:
                got.append(loop.wait(tk, b - a))
                continue
            # every other burst read in place (gcl_rxloop_peek) and released
            rec = loop.peek(tk)
            assert len(rec) == b - a and (rec["ticket"] == tk).all()
            if vb == 8:
                x = (rec["verdict"].astype(np.uint64) << np.uint64(32)) | rec["hash"].astype(np.uint64)
                got.append(x.view(g.VERDICT_DTYPE))
            elif vb == 4:
                got.append(rec["verdict"].copy().view(g.VERDICT4_DTYPE))
            elif vb == 2:
                got.append(rec["verdict"].astype(np.uint16))
            else:
                got.append(rec["verdict"].astype(np.uint8))
            loop.release(tk)
        got = np.concatenate(got)
        ps = poll_stats_settled(loop, len(bursts(n)))
        assert sum(ps.values()) == len(bursts(n)), ps  # the writer wave took every burst
        if early:  # every burst taken with its poll (early, or re-read if stale)
            assert ps["late"] == 0, ps
    finally:
        loop.stop()
        g.host_unregister(frames)
    w = want(ve, tc_map(rts, max_rt), vb, tb)
    bad = np.nonzero(got != w)[0]
    assert not len(bad), f"{len(bad)} differ, first {bad[0]}: {got[bad[0]]} vs {w[bad[0]]}"
    torch.cuda.synchronize()
    c, s_ = cnt.cpu().numpy().astype(np.uint64), st.cpu().numpy().astype(np.uint64)
    diff = {int(i): (int(c[i]), int(ce[i])) for i in np.nonzero(c != ce)[0]}
    assert not diff and (s_ == se).all(), (f"counts (got, want) {diff}; stats {s_.tolist()} vs {se.tolist()}; "
                                           f"polls {ps}")


LEAN_CASES = [(m, vb, fl, lf) for m in (0, 1, 2) for vb in (8, 4, 2, 1) for fl, lf in ((0, 2), (2, 0))]


@pytest.mark.parametrize("mode,vb,flags,lflag", LEAN_CASES)
def test_rxloop_lean_path(g, orc, mode, vb, flags, lflag):
    """rxloop64_kernel's lean path (classify_lean) against the oracle: bursts
    of plain IPv4 (every packet Ethertype IPv4, IHL 5, no FDIR mark) take it,
    bursts with one FDIR-marked packet, or with dst_ip hints, take
    classify_core; both give the oracle's verdicts and counters, and
    gcl_rxloop_lean_bursts counts exactly the plain bursts.  Modes NIC /
    JENKINS / TOEPLITZ, every verdict width, the 16-bit hash, records or
    offsets; misses, runtimes with no active kthread (WAKE), fragments and
    non-TCP/UDP protocols (hash 0), ol_flags without RSS_HASH."""
    rng = np.random.default_rng(9100 + 10 * mode + vb + 100 * flags + 1000 * lflag)
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12, max_threads=8 if vb == 1 else 16)
    tb = 3 if vb == 1 else 4
    n = 64 * 24 + 17
    frames, offs, olf, rss, fdir = plain_batch(rng, n, rts)
    hint = np.zeros(n, dtype=np.uint32)
    spans = bursts(n)
    # every 4th burst general: one FDIR-marked packet, or (every 8th) dst_ip hints
    fdir_b = {k for k in range(len(spans)) if k % 8 == 3}
    hint_b = {k for k in range(len(spans)) if k % 8 == 7}
    for k in fdir_b:
        a, _ = spans[k]
        olf[a + 5] |= np.uint8(0x02)  # GCL_F_FDIR_ID
        fdir[a + 5] = np.uint32(rts[0]["uniqid"])
    for k in hint_b:
        a, b = spans[k]
        hint[a:b:3] = np.uint32(rts[1]["ip"])
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    cflags = {8: 0, 4: g.CFG_VERDICT4, 2: g.CFG_VERDICT2, 1: g.CFG_VERDICT1}[vb] | flags
    t = orc.Tables(max_rt, mode, flags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, cflags, 0x09, key, thread_bits=tb)
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=frames.nbytes, dst_hint=hint)
    g.host_register(frames)
    cnt = torch.zeros(max_rt, dtype=torch.int64, device="cuda")
    st = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    # the zero fills run on torch's stream, the loop on a stream of its own:
    # done before the loop adds to them (gcl_rxloop_start also orders the
    # default stream's work first)
    torch.cuda.synchronize()
    clf.tune(loop_spec=SPEC_WIDE)
    loop = clf.rxloop(frames, slots=8, counts=cnt, stats=st, flags=LOOP_FLAGS[lflag](g))
    try:
        got = []
        for k, (a, b) in enumerate(spans):
            tk = loop.submit(offs[a:b], olf[a:b], rss[a:b], fdir[a:b],
                             hint[a:b] if k in hint_b else None)
            assert tk > 0
            got.append(loop.wait(tk, b - a))
        got = np.concatenate(got)
        # the writer wave posts the lean counter after the burst's records
        # (the host can see a burst complete before its count): poll for it
        expect = len(spans) - len(fdir_b) - len(hint_b)
        deadline = time.monotonic() + 1.0
        lean = loop.lean_bursts()
        while lean < expect and time.monotonic() < deadline:
            time.sleep(0.001)
            lean = loop.lean_bursts()
    finally:
        loop.stop()
        g.host_unregister(frames)
    w = want(ve, tc_map(rts, max_rt), vb, tb)
    bad = np.nonzero(got != w)[0]
    assert not len(bad), f"{len(bad)} differ, first {bad[0]}: {got[bad[0]]} vs {w[bad[0]]}"
    assert lean == expect, lean
    torch.cuda.synchronize()
    assert (cnt.cpu().numpy().astype(np.uint64) == ce).all()
    assert (st.cpu().numpy().astype(np.uint64) == se).all()


@pytest.mark.parametrize("lflag", [0, 2])
def test_rxloop_tables_and_recycled_mbufs(g, orc, lflag):
    """Table changes apply from the next burst on; frames rewritten in place
    by the CPU between bursts are read fresh (system-scope loads, or the
    submitting core's header records)."""
    rng = np.random.default_rng(7100 + lflag)
    max_rt = 64
    rts = random_runtimes(rng, max_rt, 20)
    n = 64
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt, tail_runts=False)
    t = orc.Tables(max_rt, 1, 0, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, 1, 0, 0x09)
    apply_runtimes(clf, rts)
    g.host_register(frames)
    loop = clf.rxloop(frames, slots=4, flags=LOOP_FLAGS[lflag](g))
    try:
        for rnd in range(6):
            tk = loop.submit(offs, olf, None, fdir, None)
            got = loop.wait(tk, n)
            ve, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, fdir_hi=fdir)
            assert (got == ve).all(), f"round {rnd}"
            # tables: drop two runtimes, add a new one at a fresh uniqid
            for r in rts[:2]:
                assert t.runtime_del(r["uniqid"]) == 0
                clf.runtime_del(r["uniqid"])
            rts = rts[2:]
            fresh = random_runtimes(rng, max_rt, 40)
            used = {r["uniqid"] for r in rts} | {r["ip"] for r in rts}
            add = [r for r in fresh if r["uniqid"] not in used and r["ip"] not in used][:1]
            apply_runtimes(t, add)
            apply_runtimes(clf, add)
            rts += add
            # recycled mbufs: new packets at the same addresses
            nf, _, _, olf, _, fdir, _ = fuzz_batch(rng, n, rts, max_rt, tail_runts=False)
            assert nf.shape == frames.shape
            frames[:] = nf
    finally:
        loop.stop()
        g.host_unregister(frames)


def test_rxloop_workers_pipelined_and_full_ring(g, orc):
    rng = np.random.default_rng(7200)
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12)
    n = 64 * 40
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    t = orc.Tables(max_rt, 1, g.CFG_VERDICT4, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, 1, g.CFG_VERDICT4, 0x09)
    apply_runtimes(clf, rts)
    ve, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, frames_len=flen)
    w = to_verdict4(ve, tc_map(rts, max_rt))
    g.host_register(frames)
    loop = clf.rxloop(frames, slots=8, workers=4, region_len=flen)
    try:
        bs = bursts(n)
        # a full ring refuses the next burst until the oldest one is retired
        tks = [loop.submit(offs[a:b], olf[a:b]) for a, b in bs[:8]]
        assert all(x > 0 for x in tks)
        assert loop.submit(offs[:64], olf[:64]) == -11  # -EAGAIN
        # a peeked burst holds its slot until released
        rec = loop.peek(tks[0])
        assert (rec["verdict"].copy().view(g.VERDICT4_DTYPE) == w[:64]).all()
        assert loop.submit(offs[:64], olf[:64]) == -11
        assert g.lib.gcl_rxloop_release(loop._h, tks[-1] + 5) == -22
        got = [loop.wait(tk, 64) for tk in tks]
        for a, b in bs[8:]:
            tk = loop.submit(offs[a:b], olf[a:b])
            assert tk > 0
            tks.append(tk)
            if len(tks) - len(got) == 8:
                got.append(loop.wait(tks[len(got)], 64))
        while len(got) < len(tks):
            got.append(loop.wait(tks[len(got)], 64))
        got = np.concatenate(got)
        assert (got == w).all()
        lat, el = loop.drive(offs[:64], 200, depth=4)
        assert (lat > 0).all() and el > 0
    finally:
        loop.stop()
        g.host_unregister(frames)


@pytest.mark.parametrize("max_burst,workers,lflag", [(64, 1, 0), (64, 3, 0), (256, 2, 0),
                                                     (64, 1, 2), (64, 3, 2), (256, 2, 2),
                                                     (1024, 2, 0), (1024, 2, 2)])
def test_rxloop_stamped_offsets_ragged_bursts(g, orc, max_burst, workers, lflag):
    """Offsets ride in the slot stamped with the slot's use count, and a
    worker polling a burst of <= 64 takes them with the poll when every stamp
    is current (lflag 2: whole header records, GCL_LOOP_HDR_RECORDS, each
    16-B chunk stamped).  Two slots reused ~700 times each (past the periodic
    rewrite of the entries beyond a burst's n), burst sizes drawn from
    1..max_burst so stale entries of longer bursts sit behind shorter ones,
    and offsets at and past 2^40 (the stamp's bit) that read as frames past
    the region."""
    rng = np.random.default_rng(7300 + max_burst + workers + 17 * lflag)
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12)
    n = 4096
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    far = np.array([1 << 40, (1 << 40) - 1, (1 << 41) + 77, 1 << 50], dtype=np.uint64)
    offs = np.concatenate([offs, far])
    olf = np.concatenate([olf, np.full(len(far), 0x09, dtype=np.uint8)])
    rss = np.concatenate([rss, rng.integers(0, 2**32, size=len(far), dtype=np.uint64).astype(np.uint32)])
    t = orc.Tables(max_rt, 1, 0, 0x09)
    apply_runtimes(t, rts)
    ve, _, _ = t.classify(frames, len(offs), 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    assert (ve[n:]["action"] == ve[n]["action"]).all()  # zero frames: one drop verdict
    clf = g.Classifier(0, max_rt, 1, 0, 0x09)
    apply_runtimes(clf, rts)
    g.host_register(frames)
    # every burst of <= 64 taken with its poll (SPEC_WIDE), as bursts from a C
    # dataplane loop are
    clf.tune(loop_spec=SPEC_WIDE)
    loop = clf.rxloop(frames, slots=2, workers=workers, max_burst=max_burst, region_len=flen,
                      flags=LOOP_FLAGS[lflag](g))
    try:
        nb = 1400
        sizes = np.where(rng.random(nb) < 0.3, max_burst, rng.integers(1, max_burst + 1, size=nb))
        for k, m in enumerate(sizes):
            idx = rng.integers(0, len(offs), size=int(m))
            if k % 50 == 0:
                idx[-1] = n + k // 50 % len(far)  # an offset past 2^40
            tk = loop.submit(offs[idx], olf[idx], rss[idx])
            assert tk > 0
            got = loop.wait(tk, int(m))
            bad = np.nonzero(got != ve[idx])[0]
            assert not len(bad), f"burst {k} (n {m}): packet {bad[0]} {got[bad[0]]} vs {ve[idx][bad[0]]}"
        ps = poll_stats_settled(loop, nb)
        assert sum(ps.values()) == nb, ps
        # How many bursts were current at their first poll (early) rather
        # than re-read after it (stale) depends on how the host paces its
        # stores against the polls: a measurement (reported), not a gate.
        # What does not depend on pacing: bursts of <= 64 are all taken with
        # the poll, longer ones never.
        print(f"poll stats max_burst={max_burst} workers={workers} lflag={lflag}: {ps}")
        if max_burst <= 64:
            assert ps["late"] == 0, ps
        else:
            assert ps["early"] == 0 and ps["stale"] == 0, ps
    finally:
        loop.stop()
        g.host_unregister(frames)


@pytest.mark.parametrize("cfg", [("200000", "1", "2", "1"), ("400000", "4", "4", "4"), ("400000", "32", "64", "64"),
                                 ("200000", "1", "2", "1", "records"), ("400000", "4", "4", "4", "records"),
                                 ("400000", "32", "64", "64", "records")])
def test_rxloop_soak_stamped_offsets(g, cfg):
    """tools/loopsoak: random 1..64-packet bursts at random offsets into a
    mixed-traffic region, few slots, a tight host loop with random pauses
    racing the workers' polls; every verdict equal to the batch kernel's for
    the same packet (exit 2 on a mismatch)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "loopsoak")
    if not os.access(exe, os.X_OK):
        pytest.fail("tools/loopsoak not built (python -c 'import __graft_entry__ as g; g.build()')")
    r = subprocess.run([exe, *cfg], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, (r.stdout[-300:], r.stderr[-300:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["packets_checked"] > int(cfg[0]) * 30


def test_rxloop_lifetime_and_errors(g):
    frames = np.zeros(1 << 16, dtype=np.uint8)
    clf = g.Classifier(0, 16, 1)
    with pytest.raises(OSError):  # region not registered
        clf.rxloop(frames)
    g.host_register(frames)
    try:
        loop = clf.rxloop(frames, slots=4, lifetime_ms=300)
        with pytest.raises(OSError):  # one loop per context
            clf.rxloop(frames)
        offs = np.arange(4, dtype=np.uint64) * 64
        tk = loop.submit(offs)
        assert (loop.wait(tk, 4)["action"] == 2).all()  # zero frames: bad Ethertype
        assert loop.submit(np.zeros(65, dtype=np.uint64)) == -22  # > max_burst
        time.sleep(0.8)
        assert loop.submit(offs) == -108  # -ESHUTDOWN: the kernel left on its own
        loop.stop()
        with pytest.raises(OSError):  # inline granules and header records exclude each other
            clf.rxloop(frames, flags=g.LOOP_INLINE_HDRS | g.LOOP_HDR_RECORDS)
        with pytest.raises(OSError):  # unknown flag (0x4 is GCL_LOOP_STAMPS)
            clf.rxloop(frames, flags=0x8)
        lp2 = clf.rxloop(frames, slots=4)
        tk = lp2.submit(offs)
        lp2.wait(tk, 4)
        with pytest.raises(OSError):  # no transport hashes in this context
            lp2.trans(tk, 4)
        lp2.stop()
    finally:
        g.host_unregister(frames)


@pytest.mark.parametrize("mode,vb,lflag", [(1, 8, 0), (0, 4, 0), (2, 8, 2), (1, 4, 2)])
def test_rxloop_transport_hashes(g, orc, mode, vb, lflag):
    """GCL_CFG_TRANS_HASH through the loop: each delivered IPv4 TCP/UDP
    packet's trans_hash_5tuple / _3tuple with its runtime's seed
    (runtime/net/transport.c:29-42, as gcl_classify_ex computes them) come
    back beside the verdicts (gcl_rxloop_trans), equal to the oracle's, with
    the offsets or header records taken with the poll half the time."""
    rng = np.random.default_rng(7500 + 10 * mode + vb + lflag)
    max_rt = 64
    rts = random_runtimes(rng, max_rt, 40)
    n = 2500
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    cflags = g.CFG_TRANS_HASH | (g.CFG_VERDICT4 if vb == 4 else 0)
    t = orc.Tables(max_rt, mode, cflags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, cflags, 0x09, key)
    apply_runtimes(clf, rts)
    for r in rts:
        seed = int(rng.integers(0, 2**32))
        t.set_trans_seed(r["uniqid"], seed)
        clf.set_trans_seed(r["uniqid"], seed)
    ve, _, _, te = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                              frames_len=flen, dst_hint=hint, trans=True)
    assert (te["h5"] != 0).sum() > n // 10
    g.host_register(frames)
    if lflag == 2:
        clf.tune(loop_spec=SPEC_WIDE)
    loop = clf.rxloop(frames, slots=8, region_len=flen, flags=LOOP_FLAGS[lflag](g))
    try:
        got, gt = [], []
        for k, (a, b) in enumerate(bursts(n)):
            tk = loop.submit(offs[a:b], olf[a:b], rss[a:b], fdir[a:b], hint[a:b])
            assert tk > 0
            if k % 2:
                rec = loop.peek(tk)
                gt.append(loop.trans(tk, b - a))
                v = rec["verdict"].copy()
                got.append(((v.astype(np.uint64) << np.uint64(32)) | rec["hash"].astype(np.uint64))
                           .view(g.VERDICT_DTYPE) if vb == 8 else v.view(g.VERDICT4_DTYPE))
                loop.release(tk)
            else:
                got.append(loop.wait(tk, b - a))
                gt.append(loop.trans(tk, b - a))
        got, gt = np.concatenate(got), np.concatenate(gt)
    finally:
        loop.stop()
        g.host_unregister(frames)
    w = want(ve, tc_map(rts, max_rt), vb)
    assert (got == w).all()
    bad = np.nonzero(gt != te)[0]
    assert not len(bad), f"{len(bad)} transport hashes differ, first {bad[0]}: {gt[bad[0]]} vs {te[bad[0]]}"


@pytest.mark.parametrize("lflag,spec,use0", [(0, 0, (1 << 23) - 150), (0, SPEC_WIDE, (1 << 23) - 150),
                                             (2, SPEC_WIDE, (1 << 31) - 150), (2, 0, (1 << 31) - 150)])
def test_rxloop_stamp_wrap(g, orc, lflag, spec, use0):
    """The slots' use count crossing the stamps' wrap (2^23 for stamped
    offsets, 2^31 for header records) with the loop started near it
    (gcl_tune.loop_t0): stamps are never 0, so a zeroed or never-loaded
    entry never passes for a current one, with the speculative window closed
    (spec 0: every burst read after its word) or wide open (every burst with
    the poll).  Every verdict equals the oracle's."""
    rng = np.random.default_rng(7700 + lflag + len(str(spec)))
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12)
    n = 2048
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    t = orc.Tables(max_rt, 1, 0, 0x09)
    apply_runtimes(t, rts)
    ve, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    clf = g.Classifier(0, max_rt, 1, 0, 0x09)
    apply_runtimes(clf, rts)
    g.host_register(frames)
    slots = 2
    clf.tune(loop_spec=spec, loop_t0=slots * use0)
    loop = clf.rxloop(frames, slots=slots, workers=1, region_len=flen, flags=LOOP_FLAGS[lflag](g))
    try:
        nb = 600  # 300 uses of each slot: across the wrap
        for k in range(nb):
            m = int(rng.integers(1, 65))
            idx = rng.integers(0, n, size=m)
            tk = loop.submit(offs[idx], olf[idx], rss[idx])
            assert tk == slots * use0 + k + 1
            got = loop.wait(tk, m)
            bad = np.nonzero(got != ve[idx])[0]
            assert not len(bad), f"burst {k} (use {use0 + k // slots + 1}): {got[bad[0]]} vs {ve[idx][bad[0]]}"
        ps = poll_stats_settled(loop, nb)
        if spec == 0:
            assert ps["early"] == 0 and ps["stale"] == 0, ps
        else:
            assert ps["late"] == 0, ps
    finally:
        loop.stop()
        g.host_unregister(frames)


@pytest.mark.parametrize("phase", [None, (0, 16, 1), (1000, 1000, 0), (1, 1, 1)])
@pytest.mark.parametrize("workers,lflag", [(1, 2), (2, 2), (1, 0), (1, 1)])
def test_rxloop_phase_delay(g, orc, phase, workers, lflag):
    """The poll-phase delay (gcl_tune.loop_phase_* (max, up, down); None: the
    default, on for loops of 1-2 workers) only moves when a ticket's first
    poll is issued: bursts submitted in a closed loop (each after the last
    one's verdicts), with host-side gaps now and then, come back equal to the
    oracle's whatever the delay does -- off, pinned at 10 us after the first
    late find ((1000, 1000, 0)), or one tick."""
    rng = np.random.default_rng(7900 + workers + 10 * lflag + (len(",".join(map(str, phase))) if phase else 0))
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12)
    n = 2048
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    t = orc.Tables(max_rt, 1, 0, 0x09)
    apply_runtimes(t, rts)
    ve, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    clf = g.Classifier(0, max_rt, 1, 0, 0x09)
    apply_runtimes(clf, rts)
    g.host_register(frames)
    if phase is not None:
        clf.tune(loop_phase=phase)
    loop = clf.rxloop(frames, slots=8, workers=workers, region_len=flen, flags=LOOP_FLAGS[lflag](g))
    try:
        for k in range(300):
            m = int(rng.integers(1, 65))
            idx = rng.integers(0, n, size=m)
            tk = loop.submit(offs[idx], olf[idx], rss[idx])
            got = loop.wait(tk, m)
            bad = np.nonzero(got != ve[idx])[0]
            assert not len(bad), f"burst {k}: {got[bad[0]]} vs {ve[idx][bad[0]]}"
            if k % 50 == 49:
                time.sleep(0.001)  # sparse now and then: the delay must not stall
    finally:
        loop.stop()
        g.host_unregister(frames)


@pytest.mark.parametrize("prefetch", [None, 0, 1])
@pytest.mark.parametrize("lflag", [0, 2])
@pytest.mark.parametrize("slots,workers", [(16, 4), (4, 4), (2, 4)])
def test_rxloop_prefetch(g, orc, prefetch, lflag, slots, workers):
    """The next ticket's poll issued before a burst is classified
    (gcl_tune.loop_prefetch; None: the default, on for stamped offsets with
    more than two workers): bursts kept 12 deep across 4 workers, so that
    polls find them queued, and drained now and then, so that they catch up;
    every verdict equal to the oracle's."""
    rng = np.random.default_rng(7950 + lflag + (3 if prefetch is None else prefetch) + 10 * slots)
    max_rt = 16
    rts = random_runtimes(rng, max_rt, 12)
    n = 2048
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    t = orc.Tables(max_rt, 1, 0, 0x09)
    apply_runtimes(t, rts)
    ve, _, _ = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    clf = g.Classifier(0, max_rt, 1, 0, 0x09)
    apply_runtimes(clf, rts)
    g.host_register(frames)
    if prefetch is not None:
        clf.tune(loop_prefetch=prefetch)
    loop = clf.rxloop(frames, slots=slots, workers=workers, region_len=flen, flags=LOOP_FLAGS[lflag](g))
    deep = min(12, slots)  # in flight at most: the ring's slots
    try:
        inflight = []
        for k in range(600):
            m = int(rng.integers(1, 65))
            idx = rng.integers(0, n, size=m)
            tk = loop.submit(offs[idx], olf[idx], rss[idx])
            assert tk > 0, tk
            inflight.append((tk, m, idx))
            if len(inflight) >= deep or k % 97 == 96:
                while inflight:  # every 97th burst: drain, so the workers catch up
                    tk, mm, ii = inflight.pop(0)
                    got = loop.wait(tk, mm)
                    bad = np.nonzero(got != ve[ii])[0]
                    assert not len(bad), f"ticket {tk}: {got[bad[0]]} vs {ve[ii][bad[0]]}"
                    if len(inflight) < deep * 2 // 3 and k % 97 != 96:
                        break
        for tk, mm, ii in inflight:
            got = loop.wait(tk, mm)
            assert (got == ve[ii]).all(), tk
    finally:
        loop.stop()
        g.host_unregister(frames)


def test_rxloop_release_incomplete(g):
    """gcl_rxloop_release refuses (-EAGAIN) a burst the GPU has not completed,
    so its slot is never handed to the next submit while still being written."""
    frames = np.zeros(1 << 16, dtype=np.uint8)
    clf = g.Classifier(0, 16, 1)
    g.host_register(frames)
    try:
        loop = clf.rxloop(frames, slots=2, lifetime_ms=2000)
        offs = np.arange(64, dtype=np.uint64) * 64
        tk = loop.submit(offs)
        r = g.lib.gcl_rxloop_release(loop._h, tk)
        assert r in (0, -11)  # -EAGAIN unless the GPU was already done
        loop.wait(tk, 64)
        assert g.lib.gcl_rxloop_release(loop._h, tk) == 0
        loop.stop()
    finally:
        g.host_unregister(frames)
