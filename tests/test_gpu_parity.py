"""GPU parity: the HIP classifier through the C ABI vs the CPU oracle and the
golden fixtures.  Bit-exact on every verdict, count and counter."""
import ctypes

import numpy as np
import pytest

from tests.rxcases import (apply_runtimes, apply_seeds, fuzz_batch, random_runtimes, scenario_batch,
                           to_verdict1, to_verdict2, to_verdict4,
                           scenario_sets, scenario_trans)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def g():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from caladan_amd import gclassify
    return gclassify


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda() if a is not None else None


def gpu_run(g, clf, frames, n, stride=0, offs=None, olflags=None, rss=None, fdir=None,
            frames_len=None, counts=None, stats=None, hint=None, trans=False):
    f = dev(frames.view(np.uint8))
    v = torch.zeros(n * clf.vbytes, dtype=torch.uint8, device="cuda")
    c = counts if counts is not None else torch.zeros(clf.max_runtimes, dtype=torch.int64, device="cuda")
    s = stats if stats is not None else torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    o = dev(offs.astype(np.int64)) if offs is not None else None
    tr = torch.zeros(n * 8, dtype=torch.uint8, device="cuda") if trans else None
    clf.classify(f, n, stride, verdicts=v, counts=c, stats=s, offs=o, olflags=dev(olflags), trans=tr,
                 rss=dev(rss.view(np.int32)) if rss is not None else None,
                 fdir_hi=dev(fdir.astype(np.int32)) if fdir is not None else None,
                 frames_len=frames_len,
                 dst_hint=dev(hint.view(np.int32)) if hint is not None else None)
    torch.cuda.synchronize()
    res = (v.cpu().numpy().view(g.verdict_dtype(clf.vbytes)), c.cpu().numpy().astype(np.uint64),
           s.cpu().numpy().astype(np.uint64))
    if trans:
        res += (tr.cpu().numpy().view(g.TRANS_DTYPE),)
    return res


def assert_same(v, ve, what=""):
    if not (v == ve).all():
        bad = np.nonzero(v != ve)[0]
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} verdicts differ, first at {i}: gpu={v[i]} want={ve[i]}")


SETS = scenario_sets()


@pytest.mark.parametrize("s", SETS, ids=[s["name"] for s in SETS])
def test_gpu_scenarios(g, s):
    cfg = s["cfg"]
    clf = g.Classifier(0, cfg["max_runtimes"], cfg["hash_mode"], cfg["flags"], cfg["default_olflags"],
                       bytes.fromhex(cfg["rss_key"]))
    apply_runtimes(clf, s["runtimes"])
    apply_seeds(clf, s)
    frames, olflags, rss, fdir, exp, hint = scenario_batch(s)
    want_tr = scenario_trans(s)
    out = gpu_run(g, clf, frames, len(exp), 128, olflags=olflags, rss=rss, fdir=fdir,
                  hint=hint, trans=want_tr is not None)
    v, c, st = out[:3]
    if want_tr is not None:
        assert (out[3] == want_tr).all(), (out[3], want_tr)
    for i in range(len(exp)):
        assert tuple(v[i]) == tuple(exp[i]), (s["packets"][i]["cite"], v[i], exp[i])
    assert list(st) == s["expect_stats"]
    assert list(c) == s["expect_counts"]


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("flags", [0, 1, 2])
@pytest.mark.parametrize("max_rt", [16, 1024, 4096])
@pytest.mark.parametrize("i32", [1, 0])
def test_gpu_fuzz_vs_oracle(g, orc, mode, flags, max_rt, i32):
    """i32: the pair kernel's 32-bit form (the default for batches within
    2 GiB) or its 64-bit form (gcl_tune.pair_i32 = 0, what larger batches run)."""
    rng = np.random.default_rng(1000 * mode + 10 * flags + max_rt)
    rts = random_runtimes(rng, max_rt, min(max_rt, 40 if max_rt == 16 else 300))
    n = 5000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    if flags == 2:
        hint = None  # keep one arm without the loopback feed
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    cflags = flags | (g.CFG_TRANS_HASH if flags != 1 else 0)
    t = orc.Tables(max_rt, mode, cflags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, cflags, 0x09, key, tune={"pair_i32": i32})
    apply_runtimes(clf, rts)
    want_tr = cflags & g.CFG_TRANS_HASH
    if want_tr:
        for r in rts:
            seed = int(rng.integers(0, 2**32))
            t.set_trans_seed(r["uniqid"], seed)
            clf.set_trans_seed(r["uniqid"], seed)
    oe = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen,
                    dst_hint=hint, trans=bool(want_tr))
    og = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir, frames_len=flen,
                 hint=hint, trans=bool(want_tr))
    ve, ce, se = oe[:3]
    v, c, st = og[:3]
    if want_tr:
        assert (og[3] == oe[3]).all(), "trans hashes differ"
    assert_same(v, ve, f"mode={mode} flags={flags} R={max_rt}")
    assert (c == ce).all()
    assert (st == se).all(), (st, se)


@pytest.mark.parametrize("misalign", ["mbuf", "mixed", "lineend"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("i32", [1, 0])
def test_gpu_fuzz_misaligned_offsets(g, orc, misalign, mode, i32):
    """Frame offsets that are not 16-B aligned: 8-B aligned like mbuf data in
    the reference's ingress pool (element + 344, iokernel/defs.h:503-506),
    arbitrary byte shifts, and frames whose first 128-B line ends 40-56 bytes
    in (header staged up to the line end; ARP's target IP and IPv4 options
    read past it)."""
    rng = np.random.default_rng(9100 + 10 * mode + (misalign == "mixed") + 2 * (misalign == "lineend"))
    rts = random_runtimes(rng, 1024, 300)
    n = 5000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(
        rng, n, rts, 1024, slot=256 if misalign == "lineend" else 128, misalign=misalign)
    t = orc.Tables(1024, mode, g.CFG_TRANS_HASH, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, 1024, mode, g.CFG_TRANS_HASH, 0x09, tune={"pair_i32": i32})
    apply_runtimes(clf, rts)
    ve, ce, se, tre = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                                 frames_len=flen, dst_hint=hint, trans=True)
    v, c, st, tr = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                           frames_len=flen, hint=hint, trans=True)
    assert_same(v, ve, f"misalign={misalign} mode={mode} i32={i32}")
    assert (tr == tre).all() and (c == ce).all() and (st == se).all()


@pytest.mark.parametrize("tables", ["lds", "global"])
@pytest.mark.parametrize("misalign", ["mbuf", "mixed", "lineend"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gpu_general_kernels_fuzz(g, orc, misalign, mode, tables):
    """The GENERAL kernel (classify_pair_kernel) on the misaligned-offset
    fuzz: frames at every 16-B phase, frames that are not 4-B aligned
    (bytewise), headers cut at a line end, frames straddling frames_len,
    IHL > 5 ports and ARP target IPs read from the frame, loopback hints,
    FDIR marks and the transport pre-hash, in all three hash modes, an odd
    packet count, with the tables in LDS and forced to global memory
    (gcl_tune.tables = 1)."""
    kernel = "pair"
    rng = np.random.default_rng(9300 + 10 * mode + {"mbuf": 0, "mixed": 1, "lineend": 2}[misalign]
                                + 100 * (tables == "global") + 1000 * 2)
    rts = random_runtimes(rng, 1024, 300)
    n = 7001
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(
        rng, n, rts, 1024, slot=256 if misalign == "lineend" else 128, misalign=misalign)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    t = orc.Tables(1024, mode, g.CFG_TRANS_HASH, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, 1024, mode, g.CFG_TRANS_HASH, 0x09, key,
                       tune={"tables": 1} if tables == "global" else None)
    apply_runtimes(clf, rts)
    ve, ce, se, tre = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                                 frames_len=flen, dst_hint=hint, trans=True)
    v, c, st, tr = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                           frames_len=flen, hint=hint, trans=True)
    assert_same(v, ve, f"{kernel} misalign={misalign} mode={mode}")
    assert (tr == tre).all() and (c == ce).all() and (st == se).all()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("flags", [1, 2])
@pytest.mark.parametrize("max_rt", [16, 1024])
def test_gpu_fuzz_verdict4(g, orc, mode, flags, max_rt):
    """GCL_CFG_VERDICT4: the same verdicts without the hash, WAKE carrying
    its flow_tbl slot (hash % thread_count)."""
    rng = np.random.default_rng(7000 + 1000 * mode + 10 * flags + max_rt)
    rts = random_runtimes(rng, max_rt, min(max_rt, 40 if max_rt == 16 else 300))
    n = 5000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    t = orc.Tables(max_rt, mode, flags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, flags | g.CFG_VERDICT4, 0x09, key)
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                       frames_len=flen, hint=hint)
    assert ((ve["action"] & 0x3F) == g.ACT_WAKE).any()
    exp = to_verdict4(ve, {r["uniqid"]: r["thread_count"] for r in rts})
    assert_same(v, exp, f"verdict4 mode={mode} flags={flags} R={max_rt}")
    assert (c == ce).all() and (st == se).all()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("flags", [1, 2])
@pytest.mark.parametrize("max_rt", [16, 1024])
def test_gpu_fuzz_verdict2(g, orc, mode, flags, max_rt):
    """GCL_CFG_VERDICT2: one u16 kthread-queue index per packet (WAKE with
    its flow_tbl slot), up to the full 16 Ki queues at R=1024, 16 threads."""
    rng = np.random.default_rng(7100 + 1000 * mode + 10 * flags + max_rt)
    rts = random_runtimes(rng, max_rt, min(max_rt, 40 if max_rt == 16 else 300))
    for r in rts[:2]:  # WAKE verdicts in every case
        r.update(active=0, active_idx=[], flow_tbl=None)
    n = 5000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    tb = g.thread_bits_for(max_rt, 16)
    assert tb == 4
    t = orc.Tables(max_rt, mode, flags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, flags | g.CFG_VERDICT2, 0x09, key, thread_bits=tb)
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                       frames_len=flen, hint=hint)
    assert ((ve["action"] & 0x3F) == g.ACT_WAKE).any()
    exp = to_verdict2(ve, {r["uniqid"]: r["thread_count"] for r in rts}, tb)
    assert_same(v, exp, f"verdict2 mode={mode} flags={flags} R={max_rt}")
    assert (c == ce).all() and (st == se).all()


def test_gpu_verdict2_limits(g):
    """Runtimes with more kthreads than 1 << thread_bits are refused; a
    configuration past 16 Ki queues, or combined with VERDICT4 or TRANS_HASH,
    does not open."""
    clf = g.Classifier(0, 64, 1, g.CFG_VERDICT2, thread_bits=3)
    assert clf.runtime_set(5, 0x0A000001, 8, 8, list(range(8))) == 0
    with pytest.raises(OSError):
        clf.runtime_set(6, 0x0A000002, 9, 0, None)
    for flags, R, tb in [(g.CFG_VERDICT2, 4096, 3), (g.CFG_VERDICT2, 16, 9),
                         (g.CFG_VERDICT2 | g.CFG_VERDICT4, 16, 2),
                         (g.CFG_VERDICT2 | g.CFG_TRANS_HASH, 16, 2)]:
        with pytest.raises(OSError):
            g.Classifier(0, R, 1, flags, thread_bits=tb)
    g.Classifier(0, 4096, 1, g.CFG_VERDICT2, thread_bits=2).close()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("flags", [1, 2])
@pytest.mark.parametrize("max_rt,max_th", [(16, 8), (32, 4), (128, 1)])
def test_gpu_fuzz_verdict1(g, orc, mode, flags, max_rt, max_th):
    """GCL_CFG_VERDICT1: one u8 kthread-queue index per packet, up to all 128
    queues (16 x 8, 32 x 4, 128 x 1), WAKE unmarked; per-packet offsets and
    side arrays (the GENERAL kernel)."""
    rng = np.random.default_rng(7150 + 1000 * mode + 10 * flags + max_rt)
    rts = random_runtimes(rng, max_rt, min(max_rt, 40), max_threads=max_th)
    for r in rts[:2]:  # runtimes with no active kthread: WAKE in the 4-B form
        r.update(active=0, active_idx=[], flow_tbl=None)
    n = 5000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, max_rt)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    tb = max(0, (max_th - 1).bit_length())
    assert max_rt << tb <= g.V1_QUEUES
    t = orc.Tables(max_rt, mode, flags, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, max_rt, mode, flags | g.CFG_VERDICT1, 0x09, key, thread_bits=tb)
    assert clf.vbytes == 1
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                       frames_len=flen, hint=hint)
    assert ((ve["action"] & 0x3F) == g.ACT_WAKE).any()
    exp = to_verdict1(ve, {r["uniqid"]: r["thread_count"] for r in rts}, tb)
    assert_same(v, exp, f"verdict1 mode={mode} flags={flags} R={max_rt}")
    assert (c == ce).all() and (st == se).all()
    # every queue verdict decodes (gcl_verdict1_to4) to the 4-B form's runtime
    # and slot, WAKE read back as DELIVER
    w4 = to_verdict4(ve, {r["uniqid"]: r["thread_count"] for r in rts})
    dec = np.array([g.lib.gcl_verdict1_to4(int(x), tb) for x in v], dtype=np.uint32).view(g.VERDICT4_DTYPE)
    act = w4["action"] & 0x3F
    assert (dec["uniqid"] == w4["uniqid"]).all() and (dec["thread"] == w4["thread"]).all()
    assert (dec["action"] == np.where(act == g.ACT_WAKE, g.ACT_DELIVER, act)).all()


@pytest.mark.parametrize("wl,R,T", [(0, 16, 8), (2, 16, 8)])
def test_gpu_dense_verdict1(g, orc, wl, R, T):
    """GCL_CFG_VERDICT1 on the dense path (fixed slots, no side arrays: the
    bench's udp64 format) and on the mixed stream's 9216-B slots."""
    stride = {0: 64, 2: 9216}[wl]
    n = 40000 if wl == 0 else 6000
    df = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    g.generate(wl, n, stride, R, df, seed=11)
    frames = df.cpu().numpy()
    del df
    tb = 3
    clf = g.Classifier(0, R, g.HASH_JENKINS, g.CFG_VERDICT1, thread_bits=tb)
    t = orc.Tables(R, g.HASH_JENKINS, 0, g.F_RSS_HASH | g.F_IP_CKSUM_GOOD)
    for r in range(R):
        act = r % T  # runtimes 0 and 8: no active kthread (WAKE in the 4-B form)
        fl = g.steer_flows(T, list(range(act))) if act else None
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
    v, c, st = gpu_run(g, clf, frames, n, stride)
    ve, ce, se = t.classify(frames, n, stride)
    assert_same(v, to_verdict1(ve, [T] * R, tb), f"dense verdict1 wl={wl}")
    assert (c == ce).all() and (st == se).all()


DEFER_FORMS = {0: "per-packet stores", 1: "deferred (<= 2 writes per block, the default)", 2: "deferred always"}


@pytest.mark.parametrize("lean", [1, 0])
@pytest.mark.parametrize("defer", sorted(DEFER_FORMS))
@pytest.mark.parametrize("wl,R,T,vb", [(0, 16, 8, 1), (0, 16, 8, 2), (1, 1024, 4, 2)])
def test_gpu_dense_narrow_verdicts(g, orc, wl, R, T, vb, defer, lean):
    """Dense slots' 1- and 2-B verdicts in every form (gcl_tune.defer): the
    tile kernel's write-through byte and short stores per packet, or kept in
    LDS and written 16 B per lane in batches; the partial last tile
    included; 256- (udp64) and 512-lane (1024-runtime tcp1500) blocks."""
    stride = {0: 64, 1: 1536}[wl]
    n = 40000 + 77
    df = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    cdf = orc.zipf_cdf(1 << 16) if wl == 1 else None
    g.generate(wl, n, stride, R, df, seed=13, zipf_cdf_dev=dev(cdf.view(np.int64)) if cdf is not None else None,
               nflows=0 if cdf is None else len(cdf))
    frames = df.cpu().numpy()
    del df
    tb = 3 if vb == 1 else 4
    clf = g.Classifier(0, R, g.HASH_JENKINS, g.CFG_VERDICT1 if vb == 1 else g.CFG_VERDICT2, thread_bits=tb,
                       tune={"defer": defer, "tile_lean": lean})
    t = orc.Tables(R, g.HASH_JENKINS, 0, g.F_RSS_HASH | g.F_IP_CKSUM_GOOD)
    for r in range(R):
        act = r % T
        fl = g.steer_flows(T, list(range(act))) if act else None
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
    v, c, st = gpu_run(g, clf, frames, n, stride)
    ve, ce, se = t.classify(frames, n, stride)
    w = to_verdict1(ve, [T] * R, tb) if vb == 1 else to_verdict2(ve, [T] * R, tb)
    assert_same(v, w, f"narrow verdicts wl={wl} vb={vb} {DEFER_FORMS[defer]} lean={lean}")
    assert (c == ce).all() and (st == se).all()


@pytest.mark.parametrize("defer,env", [
    (1, {}), (2, {"grid": 3}), (2, {"grid": 5, "depth": 1}),
    (1, {"blocks_per_cu": 1, "grid": 301}),
    (2, {"threads": 512, "grid": 7}), (2, {"threads": 1024, "grid": 7}),
    (1, {"grid": 20}), (1, {"grid": 40}), (1, {"grid": 70}),
    (1, {"grid": 20, "depth": 1}), (1, {"threads": 512, "grid": 12}),
    (1, {"tables": 1, "grid": 40}), (2, {"tables": 1, "grid": 9}),
    # every wave on classify_core (the lean waves off)
    (1, {"tile_lean": 0}), (2, {"tile_lean": 0, "grid": 3}), (1, {"tile_lean": 0, "grid": 20}),
    (2, {"tile_lean": 0, "threads": 512, "grid": 7}), (1, {"tile_lean": 0, "grid": 5, "depth": 1}),
    # the last register flush staged through the LDS buffer (gcl_tune.vstage)
    (1, {"vstage": 1}), (1, {"vstage": 1, "grid": 40}), (1, {"vstage": 1, "grid": 20}),
    (1, {"vstage": 1, "grid": 40, "depth": 1}), (2, {"vstage": 1, "threads": 512, "grid": 7}),
    (1, {"vstage": 0, "grid": 40}),
    # one contiguous run of tiles per block (gcl_tune.tile_order): the buffer
    # and register flushes land on the block's own run; grid 301 leaves the
    # last blocks without a tile; defer 0 stores every verdict as it goes
    (1, {"tile_order": 1}), (2, {"tile_order": 1, "grid": 3}), (1, {"tile_order": 1, "grid": 40}),
    (1, {"tile_order": 1, "grid": 20, "depth": 1}), (2, {"tile_order": 1, "threads": 512, "grid": 7}),
    (1, {"tile_order": 1, "blocks_per_cu": 1, "grid": 301}), (0, {"tile_order": 1, "grid": 20}),
    (1, {"tile_order": 0})])
@pytest.mark.parametrize("vb", [1, 2])
def test_gpu_dense_deferred_flushes(g, orc, vb, defer, env):
    """The tile kernel's LDS verdict buffer when a block walks more tiles
    than it holds (few blocks: gcl_tune.grid, gcl_tune.defer = 2): full
    buffers written inside the loop, a partial one at the end, the batch's
    ragged last tile cut at n; the registers past a full buffer partly
    filled (grid 40), full and written out inside the loop (grid 20 / 12),
    or unused (grid 70 at 1-B verdicts); DEPTH 1 and 2; 256-, 512- and
    1024-lane tiles; tables in LDS and in HBM -- against the oracle on a
    1 Mi + 77-packet udp64 batch, with its counts and counters."""
    R, T, stride = 16, 8, 64
    n = (1 << 20) + 77
    df = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    g.generate(0, n, stride, R, df, seed=29)
    frames = df.cpu().numpy()
    tb = 3 if vb == 1 else 4
    clf = g.Classifier(0, R, g.HASH_JENKINS, g.CFG_VERDICT1 if vb == 1 else g.CFG_VERDICT2, thread_bits=tb,
                       tune={"defer": defer, **env})
    t = orc.Tables(R, g.HASH_JENKINS, 0, g.F_RSS_HASH | g.F_IP_CKSUM_GOOD)
    for r in range(R):
        act = (r * 3) % (T + 1)
        fl = g.steer_flows(T, list(range(act))) if act else None
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
    v = torch.full((n * vb + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    st = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    clf.classify(df, n, stride, verdicts=v, counts=c, stats=st)
    torch.cuda.synchronize()
    got = v.cpu().numpy()
    assert (got[n * vb:] == 0xEE).all(), "a verdict store past n"
    got = got[:n * vb].view(np.uint8 if vb == 1 else np.uint16)
    ve, ce, se = t.classify(frames, n, stride)
    w = to_verdict1(ve, [T] * R, tb) if vb == 1 else to_verdict2(ve, [T] * R, tb)
    assert_same(got, w, f"deferred flushes vb={vb} defer={defer} {env}")
    assert (c.cpu().numpy().astype(np.uint64) == ce).all()
    assert (st.cpu().numpy().astype(np.uint64) == se).all()


def test_gpu_verdict1_limits(g):
    """More than 128 queues, thread_bits past 7, or VERDICT1 with VERDICT2,
    VERDICT4 or TRANS_HASH does not open; kthreads past 1 << thread_bits are
    refused."""
    clf = g.Classifier(0, 16, 1, g.CFG_VERDICT1, thread_bits=3)
    assert clf.runtime_set(5, 0x0A000001, 8, 8, list(range(8))) == 0
    with pytest.raises(OSError):
        clf.runtime_set(6, 0x0A000002, 9, 0, None)
    for flags, R, tb in [(g.CFG_VERDICT1, 32, 3), (g.CFG_VERDICT1, 1, 8),
                         (g.CFG_VERDICT1 | g.CFG_VERDICT2, 16, 3),
                         (g.CFG_VERDICT1 | g.CFG_VERDICT4, 16, 3),
                         (g.CFG_VERDICT1 | g.CFG_TRANS_HASH, 16, 3)]:
        with pytest.raises(OSError):
            g.Classifier(0, R, 1, flags, thread_bits=tb)
    g.Classifier(0, 128, 1, g.CFG_VERDICT1, thread_bits=0).close()


@pytest.mark.parametrize("wl,stride,R", [(0, 64, 16), (1, 1536, 1024), (2, 9216, 16)])
def test_gpu_generator_matches_oracle(g, orc, wl, stride, R):
    n = 20000
    cdf = orc.zipf_cdf(1 << 16) if wl == 1 else None
    fe, ofe, rse = orc.generate(wl, n, stride, R, cdf=cdf)
    frames = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    olf = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rss = torch.zeros(n, dtype=torch.int32, device="cuda")
    cdf_dev = dev(cdf.view(np.int64)) if cdf is not None else None
    g.generate(wl, n, stride, R, frames, olf, rss, zipf_cdf_dev=cdf_dev, nflows=0 if cdf is None else len(cdf))
    torch.cuda.synchronize()
    assert (frames.cpu().numpy() == fe).all()
    assert (olf.cpu().numpy() == ofe).all()
    assert (rss.cpu().numpy().view(np.uint32) == rse).all()


def test_gpu_generator_sharding(g, orc):
    """Rank r's shard equals blocks r, r+W, ... of the global stream."""
    n, blk, W = 8192, 1024, 4
    full, _, _ = orc.generate(0, n * W, 64, 16)
    full = full.reshape(n * W, 64)
    for r in range(W):
        frames = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        g.generate(0, n, 64, 16, frames, rank=r, world=W, shard_block=blk)
        torch.cuda.synchronize()
        got = frames.cpu().numpy().reshape(n, 64)
        idx = np.concatenate([np.arange(b * blk, (b + 1) * blk) for b in range(r, n * W // blk, W)])
        assert (got == full[idx]).all()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("wl,stride,R,T", [(0, 64, 16, 8), (1, 1536, 1024, 4), (2, 9216, 16, 8)])
def test_gpu_workloads_vs_oracle(g, orc, mode, wl, stride, R, T):
    n = 100000 if wl != 2 else 20000
    cdf = orc.zipf_cdf(1 << 20) if wl == 1 else None
    frames, olf, rss = orc.generate(wl, n, stride, R, cdf=cdf)
    rng = np.random.default_rng(wl)
    t = orc.Tables(R, mode, 0, 0x09, bytes(range(40)))
    clf = g.Classifier(0, R, mode, 0, 0x09, bytes(range(40)))
    for r in range(R):
        act = int(rng.integers(1, T + 1))
        idx = [int(x) for x in rng.choice(T, size=act, replace=False)]
        fl = orc.steer_flows(T, idx)
        assert t.runtime_set(r, orc.runtime_ip(r), T, act, fl) == 0
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
    ve, ce, se = t.classify(frames, n, stride, olflags=olf, rss=rss)
    v, c, st = gpu_run(g, clf, frames, n, stride, olflags=olf, rss=rss)
    assert_same(v, ve)
    assert (c == ce).all() and (st == se).all()
    # the bench path: no per-packet arrays (default flags), stride layout
    ve, ce, se = t.classify(frames, n, stride)
    v, c, st = gpu_run(g, clf, frames, n, stride)
    assert_same(v, ve, "fast path")
    assert (c == ce).all() and (st == se).all()


def test_gpu_table_updates_between_batches(g, orc):
    """Snapshot semantics: a runtime_set between two classify calls is seen by
    the second only (tables change between bursts, iokernel/main.c:144-176)."""
    n, R = 50000, 16
    frames, _, _ = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), 4, 4, [0, 1, 2, 3])
        clf.runtime_set(r, g.runtime_ip(r), 4, 4, [0, 1, 2, 3])
    f = dev(frames)
    outs = []
    for step in range(3):
        v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
        c = torch.zeros(R, dtype=torch.int64, device="cuda")
        s = torch.zeros(8, dtype=torch.int64, device="cuda")
        clf.classify(f, n, 64, verdicts=v, counts=c, stats=s)
        outs.append((v, c, s))
        if step == 0:
            clf.runtime_set(3, g.runtime_ip(3), 3, 0, None)   # no active thread: wake
            clf.runtime_del(5)
        if step == 1:
            clf.runtime_set(5, g.runtime_ip(5), 7, 2, orc.steer_flows(7, [4, 1]))
    torch.cuda.synchronize()
    exp = [t.classify(frames, n, 64)]
    t.runtime_set(3, orc.runtime_ip(3), 3, 0, None)
    t.runtime_del(5)
    exp.append(t.classify(frames, n, 64))
    t.runtime_set(5, orc.runtime_ip(5), 7, 2, orc.steer_flows(7, [4, 1]))
    exp.append(t.classify(frames, n, 64))
    for (v, c, s), (ve, ce, se) in zip(outs, exp):
        assert_same(v.cpu().numpy().view(g.VERDICT_DTYPE), ve)
        assert (c.cpu().numpy().astype(np.uint64) == ce).all()
        assert (s.cpu().numpy().astype(np.uint64) == se).all()


def test_gpu_table_images_across_streams(g, orc):
    """Double-buffered table images with launches in flight on another stream.

    Stream A is held back by a bounded spin, then classifies with tables v0.
    Meanwhile two updates classify on stream B, so the second upload overwrites
    the image A's launch reads: it must wait for that launch.  A final launch
    on A after the updates must wait for B's upload and see v2."""
    n, R = 50000, 16
    frames, _, _ = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), 4, 4, [0, 1, 2, 3])
        clf.runtime_set(r, g.runtime_ip(r), 4, 4, [0, 1, 2, 3])
    f = dev(frames)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    bufs = [torch.zeros(n * 8, dtype=torch.uint8, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        torch.cuda._sleep(200_000_000)  # ~80 ms of GPU spin, then the v0 launch
    clf.classify(f, n, 64, verdicts=bufs[0], stream=sa.cuda_stream)
    clf.runtime_set(3, g.runtime_ip(3), 3, 0, None)
    clf.classify(f, n, 64, verdicts=bufs[1], stream=sb.cuda_stream)      # v1 -> image 1
    clf.runtime_set(5, g.runtime_ip(5), 7, 2, orc.steer_flows(7, [4, 1]))
    clf.classify(f, n, 64, verdicts=bufs[2], stream=sb.cuda_stream)      # v2 -> image 0
    clf.classify(f, n, 64, verdicts=bufs[3], stream=sa.cuda_stream)      # v2, on A
    torch.cuda.synchronize()
    exp = [t.classify(frames, n, 64)[0]]
    t.runtime_set(3, orc.runtime_ip(3), 3, 0, None)
    exp.append(t.classify(frames, n, 64)[0])
    t.runtime_set(5, orc.runtime_ip(5), 7, 2, orc.steer_flows(7, [4, 1]))
    exp.append(t.classify(frames, n, 64)[0])
    exp.append(exp[2])
    for i, (v, ve) in enumerate(zip(bufs, exp)):
        assert_same(v.cpu().numpy().view(g.VERDICT_DTYPE), ve, f"launch {i}")


def test_gpu_table_images_many_streams(g, orc):
    """More streams than an image tracks readers for (8): launches on 10
    streams read one image, the later ones taking over the oldest slot after
    waiting for it; then two table changes overwrite that image, and every
    launch must still see the tables current when it was submitted."""
    n, R = 20000, 16
    frames, _, _ = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), 4, 4, [0, 1, 2, 3])
        clf.runtime_set(r, g.runtime_ip(r), 4, 4, [0, 1, 2, 3])
    f = dev(frames)
    streams = [torch.cuda.Stream() for _ in range(10)]
    bufs = [torch.zeros(n * 8, dtype=torch.uint8, device="cuda") for _ in range(13)]
    torch.cuda.synchronize()
    with torch.cuda.stream(streams[0]):
        torch.cuda._sleep(100_000_000)  # hold the first reader back
    for i, st in enumerate(streams):
        clf.classify(f, n, 64, verdicts=bufs[i], stream=st.cuda_stream)       # v0
    clf.runtime_set(2, g.runtime_ip(2), 5, 3, orc.steer_flows(5, [4, 0, 2]))
    clf.classify(f, n, 64, verdicts=bufs[10], stream=streams[3].cuda_stream)  # v1
    clf.runtime_set(7, g.runtime_ip(7), 2, 0, None)
    clf.classify(f, n, 64, verdicts=bufs[11], stream=streams[9].cuda_stream)  # v2: image of v0
    clf.classify(f, n, 64, verdicts=bufs[12], stream=streams[0].cuda_stream)  # v2
    torch.cuda.synchronize()
    v0 = t.classify(frames, n, 64)[0]
    t.runtime_set(2, orc.runtime_ip(2), 5, 3, orc.steer_flows(5, [4, 0, 2]))
    v1 = t.classify(frames, n, 64)[0]
    t.runtime_set(7, orc.runtime_ip(7), 2, 0, None)
    v2 = t.classify(frames, n, 64)[0]
    assert not (v0 == v1).all() and not (v1 == v2).all()
    for i, (v, ve) in enumerate(zip(bufs, [v0] * 10 + [v1, v2, v2])):
        assert_same(v.cpu().numpy().view(g.VERDICT_DTYPE), ve, f"launch {i}")


def test_gpu_counts_accumulate_and_edge_sizes(g, orc):
    """Counters accumulate across calls; n = 1, ragged tails, empty batch."""
    R = 16
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), 8, 8, list(range(8)))
        clf.runtime_set(r, g.runtime_ip(r), 8, 8, list(range(8)))
    frames, _, _ = orc.generate(0, 70001, 64, R)
    f = dev(frames)
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    s = torch.zeros(8, dtype=torch.int64, device="cuda")
    tot_c = np.zeros(R, dtype=np.uint64)
    tot_s = np.zeros(8, dtype=np.uint64)
    for n in (1, 255, 256, 257, 70001):
        v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
        clf.classify(f, n, 64, verdicts=v, counts=c, stats=s)
        ve, ce, se = t.classify(frames, n, 64)
        torch.cuda.synchronize()
        assert_same(v.cpu().numpy().view(g.VERDICT_DTYPE), ve, f"n={n}")
        tot_c += ce
        tot_s += se
    assert clf.classify(f, 0, 64, verdicts=torch.zeros(8, dtype=torch.uint8, device="cuda")) == 0
    torch.cuda.synchronize()
    assert (c.cpu().numpy().astype(np.uint64) == tot_c).all()
    assert (s.cpu().numpy().astype(np.uint64) == tot_s).all()


def test_gpu_errors(g):
    clf = g.Classifier(0, 16, 1)
    with pytest.raises(OSError):
        clf.runtime_set(16, 1, 4, 4, [0, 1, 2, 3])
    clf.runtime_set(1, 0x0A000001, 4, 4, [0, 1, 2, 3])
    with pytest.raises(OSError):
        clf.runtime_set(2, 0x0A000001, 4, 4, [0, 1, 2, 3])
    with pytest.raises(OSError):
        clf.runtime_del(9)
    f = torch.zeros(640, dtype=torch.uint8, device="cuda")
    v = torch.zeros(80, dtype=torch.uint8, device="cuda")
    with pytest.raises(OSError):
        clf.classify(f, 10, 8, verdicts=v)   # stride not a multiple of 16
    with pytest.raises(OSError):
        g.Classifier(0, 5000, 1)


def test_gpu_full_size_properties(g, orc):
    """Config 2 at full size (32 Mi x 64 B): every packet is accounted for,
    and a 65536-packet random sample matches the oracle bit for bit."""
    n, R, T, stride = 32 << 20, 16, 8, 64
    frames = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    g.generate(0, n, stride, R, frames)
    clf = g.Classifier(0, R, 1)
    t = orc.Tables(R, 1, 0, 0x09)
    rng = np.random.default_rng(5)
    for r in range(R):
        act = int(rng.integers(1, T + 1))
        fl = orc.steer_flows(T, [int(x) for x in rng.choice(T, size=act, replace=False)])
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    s = torch.zeros(8, dtype=torch.int64, device="cuda")
    clf.classify(frames, n, stride, verdicts=v, counts=c, stats=s)
    torch.cuda.synchronize()
    vv = v.view(torch.int64).cpu().numpy().view(g.VERDICT_DTYPE)
    cc = c.cpu().numpy()
    ss = s.cpu().numpy()
    assert cc.sum() == n and ss[g.RX_PULLED] == n and ss[g.RX_UNHANDLED] == 0
    assert (np.bincount(vv["uniqid"], minlength=R)[:R] == cc).all()
    assert ((vv["action"] & 0x3F) == 0).all()
    sample = np.sort(rng.choice(n, size=65536, replace=False))
    fr = frames.view(n, stride)[torch.from_numpy(sample).cuda()].cpu().numpy().reshape(-1)
    ve, _, _ = t.classify(fr, len(sample), stride)
    assert_same(vv[sample], ve, "sample")


def test_gpu_full_size_tcp1500_properties(g, orc):
    """Config 3 at full size (8 Mi x 1536-B slots, Zipf-0.99 over 1 Mi flows,
    1024 runtimes x 4 kthreads): every packet is accounted for per runtime,
    each runtime gets exactly the flows `flow % R` maps to it, and a
    65536-packet random sample matches the oracle bit for bit (hash,
    runtime, kthread, action)."""
    n, R, T, stride, F = 8 << 20, 1024, 4, 1536, 1 << 20
    frames = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    cdf = g.zipf_cdf(F, 0.99)
    g.generate(g.WL_TCP1500_ZIPF, n, stride, R, frames,
               zipf_cdf_dev=torch.from_numpy(cdf.view(np.int64)).cuda(), nflows=F)
    clf = g.Classifier(0, R, 1)
    t = orc.Tables(R, 1, 0, 0x09)
    rng = np.random.default_rng(9)
    for r in range(R):
        act = int(rng.integers(1, T + 1))
        fl = orc.steer_flows(T, [int(x) for x in rng.choice(T, size=act, replace=False)])
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    s = torch.zeros(8, dtype=torch.int64, device="cuda")
    clf.classify(frames, n, stride, verdicts=v, counts=c, stats=s)
    torch.cuda.synchronize()
    vv = v.view(torch.int64).cpu().numpy().view(g.VERDICT_DTYPE)
    cc = c.cpu().numpy()
    ss = s.cpu().numpy()
    assert cc.sum() == n and ss[g.RX_PULLED] == n and ss[g.RX_UNHANDLED] == 0
    assert ss[g.RX_UNREGISTERED_MAC] == 0 and ss[g.RX_HASH_MISSING] == 0
    assert (np.bincount(vv["uniqid"], minlength=R)[:R] == cc).all()
    assert ((vv["action"] & 0x3F) == 0).all() and (vv["thread"] < T).all()
    # Zipf skew survives: the top runtime (flow 0's) carries the most packets
    assert cc.argmax() == 0 and cc[0] > 4 * np.median(cc)
    sample = np.sort(rng.choice(n, size=65536, replace=False))
    fr = frames.view(n, stride)[torch.from_numpy(sample).cuda(), :64].cpu().numpy().reshape(-1)
    del frames
    torch.cuda.empty_cache()
    ve, _, _ = t.classify(fr, len(sample), 64)
    assert_same(vv[sample], ve, "tcp1500 sample")


@pytest.mark.parametrize("name,vb", [("udp64", 1), ("udp64", 2), ("tcp1500", 2), ("tcp1500_hsplit", 2)])
def test_gpu_full_size_bench_format(g, orc, name, vb):
    """The bench lines' own instances at full size, in exactly the format and
    allocation they time: bench.Workload (frame pool placed against the
    verdict ring by gcl_dev_alloc_paired, 1- or 2-byte queue verdicts with
    thread_bits 3 for 16 x 8 and 2 for 1024 x 4, the bench's seeded tables)
    stepped once.  Every verdict is a DELIVER to a queue of a registered
    runtime, the queue histogram equals the device counts, and a
    65536-packet random sample decodes (to_verdict1 / to_verdict2) to the
    oracle's verdicts bit for bit."""
    import bench
    from tests.rxcases import to_verdict2
    dev = torch.device("cuda", 0)
    w = bench.Workload(name, 0, 1, dev, vbytes=vb)
    assert w.vbytes == vb and w.clf.vbytes == vb
    tb = w.clf.thread_bits
    assert tb == {16: 3, 1024: 2}[w.R]
    w.step(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    n, R = w.n, w.R
    hv = torch.empty(n * vb, dtype=torch.uint8).pin_memory()
    bench.hip_copy(hv, w.verdicts, n * vb)
    q = hv.numpy().view(np.uint16 if vb == 2 else np.uint8)
    cc = w.counts[:R].cpu().numpy()
    ss = w.counts[R:].cpu().numpy()
    assert cc.sum() == n and ss[g.RX_PULLED] == n and ss[g.RX_UNHANDLED] == 0
    if vb == 2:
        assert ((q & g.V2_KIND) == g.V2_DELIVER).all()
    else:
        assert ((q & g.V1_OTHER) == 0).all()
    assert (np.bincount(q >> tb, minlength=R)[:R] == cc).all()
    # the sample: the same bytes from the CPU generator, classified by the oracle
    t = orc.Tables(R, 1, 0, 0x09)
    for (r, ip, T, act, fl) in w.tables:
        assert t.runtime_set(r, ip, T, act, fl) == 0
    rng = np.random.default_rng(21)
    sample = np.sort(rng.choice(n, size=65536, replace=False))
    fr_dev = torch.empty(n * w.stride, dtype=torch.uint8, device=dev)
    bench.hip_copy(fr_dev, w.frames, n * w.stride)
    fr = fr_dev.view(n, w.stride)[torch.from_numpy(sample).cuda(), :64].cpu().numpy().reshape(-1)
    del fr_dev
    ve, _, _ = t.classify(fr, len(sample), 64)
    tcs = {r: T for (r, _, T, _, _) in w.tables}
    want = to_verdict2(ve, tcs, tb) if vb == 2 else to_verdict1(ve, tcs, tb)
    assert_same(q[sample], want, f"{name} {vb}-B sample")
    del w
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("wl,stride,R,T,arrays", [(0, 64, 16, 8, False), (1, 1536, 1024, 4, False),
                                                   (2, 9216, 16, 8, True)])
def test_gpu_end_to_end_host_buffers(g, orc, mode, wl, stride, R, T, arrays):
    """gcl_classify_host: frames in pinned host memory, verdicts back in host
    memory, through the DMA-gather (COPY) and PCIe zero-copy transports."""
    n = 300000 if wl != 2 else 40000
    cdf = orc.zipf_cdf(1 << 16) if wl == 1 else None
    frames, olf, rss = orc.generate(wl, n, stride, R, cdf=cdf)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T + 1)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T + 1, fl)
    kw = dict(olflags=olf, rss=rss) if arrays else {}
    ve, ce, se = t.classify(frames, n, stride, **kw)
    hf = torch.from_numpy(frames).pin_memory()
    hv = torch.zeros(n * 8, dtype=torch.uint8).pin_memory()
    pk = {k: torch.from_numpy(a.view(np.uint8) if k == "olflags" else a.view(np.int32)).pin_memory()
          for k, a in kw.items()}
    counts = np.zeros(R, dtype=np.uint64)
    stats = np.zeros(8, dtype=np.uint64)
    clf.classify_host(hf, n, stride, verdicts=hv, counts=counts, stats=stats, mode=mode,
                      chunk=65536 + 17, nstreams=3, **pk)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, f"e2e mode={mode}")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_end_to_end_verdict4(g, orc, mode):
    """Both transports with 4-byte verdicts (half the verdict bytes on PCIe)."""
    n, R, T = 300000, 16, 8
    frames, olf, rss = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1, g.CFG_VERDICT4)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T, fl if r % T else None)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T, fl if r % T else None)
    ve, ce, se = t.classify(frames, n, 64)
    hf = torch.from_numpy(frames).pin_memory()
    hv = torch.zeros(n * 4, dtype=torch.uint8).pin_memory()
    counts = np.zeros(R, dtype=np.uint64)
    stats = np.zeros(8, dtype=np.uint64)
    clf.classify_host(hf, n, 64, verdicts=hv, counts=counts, stats=stats, mode=mode,
                      chunk=65536 + 17, nstreams=3)
    assert_same(hv.numpy().view(g.VERDICT4_DTYPE), to_verdict4(ve, [T] * R), f"e2e4 mode={mode}")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_end_to_end_verdict2(g, orc, mode):
    """Both transports with 2-byte verdicts, chunks of odd length."""
    n, R, T = 300000, 16, 8
    frames, olf, rss = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1, g.CFG_VERDICT2, thread_bits=3)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T, fl if r % T else None)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T, fl if r % T else None)
    ve, ce, se = t.classify(frames, n, 64)
    hf = torch.from_numpy(frames).pin_memory()
    hv = torch.zeros(n * 2, dtype=torch.uint8).pin_memory()
    counts = np.zeros(R, dtype=np.uint64)
    stats = np.zeros(8, dtype=np.uint64)
    clf.classify_host(hf, n, 64, verdicts=hv, counts=counts, stats=stats, mode=mode,
                      chunk=65536 + 17, nstreams=3)
    assert_same(hv.numpy().view(np.uint16), to_verdict2(ve, [T] * R, 3), f"e2e2 mode={mode}")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_end_to_end_verdict1(g, orc, mode):
    """Both transports with 1-byte verdicts, chunks of odd length."""
    n, R, T = 300000, 16, 8
    frames, olf, rss = orc.generate(0, n, 64, R)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1, g.CFG_VERDICT1, thread_bits=3)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T, fl if r % T else None)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T, fl if r % T else None)
    ve, ce, se = t.classify(frames, n, 64)
    hf = torch.from_numpy(frames).pin_memory()
    hv = torch.zeros(n, dtype=torch.uint8).pin_memory()
    counts = np.zeros(R, dtype=np.uint64)
    stats = np.zeros(8, dtype=np.uint64)
    clf.classify_host(hf, n, 64, verdicts=hv, counts=counts, stats=stats, mode=mode,
                      chunk=65536 + 17, nstreams=3)
    assert_same(hv.numpy(), to_verdict1(ve, [T] * R, 3), f"e2e1 mode={mode}")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("base", [4, 8, 12])
def test_gpu_frames_base_misaligned(g, orc, base):
    """A frames pointer that is itself only 4-B aligned: the staging window
    (hdr_window) is placed by address, not by offset; frames within @base
    bytes of the buffer start fall back to bytewise reads, and the window's
    cut at a line end moves with the address."""
    rng = np.random.default_rng(9300 + base)
    rts = random_runtimes(rng, 1024, 300)
    n = 4000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, 1024, slot=256,
                                                          misalign="lineend")
    offs[0], offs[1], offs[2] = 0, 4, 8  # before any 16-B-aligned window start
    t = orc.Tables(1024, 1, g.CFG_TRANS_HASH, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, 1024, 1, g.CFG_TRANS_HASH, 0x09)
    apply_runtimes(clf, rts)
    ve, ce, se, tre = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                                 frames_len=flen, dst_hint=hint, trans=True)
    big = torch.zeros(frames.nbytes + 64, dtype=torch.uint8, device="cuda")
    big[base:base + frames.nbytes] = torch.from_numpy(frames).cuda()
    f = big[base:base + frames.nbytes]
    assert f.data_ptr() % 16 == base
    v = torch.zeros(n * clf.vbytes, dtype=torch.uint8, device="cuda")
    c = torch.zeros(clf.max_runtimes, dtype=torch.int64, device="cuda")
    st = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    tr = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    clf.classify(f, n, 0, verdicts=v, counts=c, stats=st, offs=dev(offs.astype(np.int64)),
                 olflags=dev(olf), trans=tr, rss=dev(rss.view(np.int32)),
                 fdir_hi=dev(fdir.astype(np.int32)), frames_len=flen,
                 dst_hint=dev(hint.view(np.int32)))
    torch.cuda.synchronize()
    assert_same(v.cpu().numpy().view(g.verdict_dtype(clf.vbytes)), ve, f"base={base}")
    assert (tr.cpu().numpy().view(g.TRANS_DTYPE) == tre).all()
    assert (c.cpu().numpy().astype(np.uint64) == ce).all()
    assert (st.cpu().numpy().astype(np.uint64) == se).all()


def test_gpu_ingress_pool_geometry(g, orc):
    """Frames at their real place in the reference's ingress mbuf pool
    (9408-B elements, 222 per 2 MiB page, data at element + 344, so 8-B
    aligned; iokernel/defs.h:503-523), in the order a NIC might have pulled
    the mbufs from the mempool: device-resident and PCIe zero-copy."""
    n, R, T = 20000, 16, 8
    frames, olf, rss = orc.generate(0, n, 64, R)
    rng = np.random.default_rng(5)
    nm = n + 3000
    offs = g.mbuf_data_offsets(nm)[rng.permutation(nm)[:n]]
    region = np.zeros(g.mbuf_region_bytes(nm), dtype=np.uint8)
    region[offs[:, None].astype(np.int64) + np.arange(64)] = frames.reshape(n, 64)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T + 1)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T + 1, fl)
    ve, ce, se = t.classify(region, n, 0, offs=offs)
    v, c, st = gpu_run(g, clf, region, n, 0, offs=offs)
    assert_same(v, ve, "ingress pool, device-resident")
    assert (c == ce).all() and (st == se).all()
    hr = torch.from_numpy(region).pin_memory()
    ho = torch.from_numpy(offs.view(np.int64)).pin_memory()
    hv = torch.zeros(n * 8, dtype=torch.uint8).pin_memory()
    counts = np.zeros(R, dtype=np.uint64)
    stats = np.zeros(8, dtype=np.uint64)
    clf.classify_host(hr, n, 0, verdicts=hv, counts=counts, stats=stats, offs=ho, mode=g.E2E_ZEROCOPY)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, "ingress pool, zero-copy")
    assert (counts == ce).all() and (stats == se).all()
    # COPY: the header gather kernel pulls each mbuf's first 80 B into HBM rows
    hv.zero_()
    counts[:] = 0
    stats[:] = 0
    clf.classify_host(hr, n, 0, verdicts=hv, counts=counts, stats=stats, offs=ho, mode=g.E2E_COPY,
                      chunk=4096 + 3, nstreams=2)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, "ingress pool, header gather")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("tile_lean", [1, 0])
@pytest.mark.parametrize("mode,vb", [(0, 1), (0, 8), (1, 1), (1, 2), (1, 4), (2, 8), (2, 1)])
def test_gpu_tile_lean_waves(g, orc, mode, vb, tile_lean):
    """classify_kernel's lean path (gcl_tune.tile_lean, on by default): dense
    64-B slots where a wave whose 64 packets are all plain IPv4 (IHL 5) takes
    classify_lean and every other wave -- one IPv6, ARP, IHL-6 or fragmented
    frame in it, every 23rd wave -- classify_core; misses, zero-active
    runtimes (WAKE), non-TCP/UDP and the NIC's hash.rss array in NIC mode;
    every hash mode and verdict width, both settings, a ragged last tile;
    bit-exact against the oracle with counts and counters."""
    rng = np.random.default_rng(1700 + 10 * mode + vb)
    R, T, n, stride = 16, 8, 200_000 + 37, 64
    frames, _, rss = orc.generate(0, n, stride, R, seed=41)
    fr = frames.reshape(n, stride)
    odd = np.arange(0, n, 64 * 23) + rng.integers(0, 64, size=len(range(0, n, 64 * 23)))
    odd = odd[odd < n]
    for j, i in enumerate(odd):
        kind = j % 5
        if kind == 0:
            fr[i, 12:14] = (0x86, 0xDD)  # IPv6: dropped
        elif kind == 1:
            fr[i, 12:14] = (0x08, 0x06)  # ARP: looked up by bytes 38-41
        elif kind == 2:
            fr[i, 14] = 0x46  # IHL 6: ports at 38
        elif kind == 3:
            fr[i, 20] |= 0x20  # MF: a fragment, hash 0
        else:
            fr[i, 30:34] = (192, 168, 7, 7)  # unregistered
    fr[::97, 23] = 1  # ICMP: hash 0
    tb = g.thread_bits_for(R, T) if vb <= 2 else 0
    cflags = {8: 0, 4: g.CFG_VERDICT4, 2: g.CFG_VERDICT2, 1: g.CFG_VERDICT1}[vb]
    t = orc.Tables(R, mode, 0, 0x09, g.CALADAN_RSS_KEY)
    clf = g.Classifier(0, R, mode, cflags, 0x09, g.CALADAN_RSS_KEY, thread_bits=tb, tune={"tile_lean": tile_lean})
    for r in range(R):
        act = (r * 5) % (T + 1)
        fl = orc.steer_flows(T, list(range(act))) if act else None
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
    kw = {"rss": rss} if mode == 0 else {}
    ve, ce, se = t.classify(frames, n, stride, **kw)
    v, c, st = gpu_run(g, clf, frames, n, stride, **kw)
    want = {8: lambda: ve, 4: lambda: to_verdict4(ve), 2: lambda: to_verdict2(ve, [T] * R, tb),
            1: lambda: to_verdict1(ve, [T] * R, tb)}[vb]()
    assert_same(v, want, f"tile lean={tile_lean} mode={mode} vb={vb}")
    assert (c == ce).all() and (st == se).all()


@pytest.mark.parametrize("pair_lean", [1, 0])
@pytest.mark.parametrize("mode,vb", [(0, 2), (0, 1), (1, 8), (1, 2), (2, 4), (2, 1)])
def test_gpu_pair_lean_waves(g, orc, mode, vb, pair_lean):
    """classify_pair_kernel's lean path (gcl_tune.pair_lean, on by default):
    a wave whose packets are all plain IPv4 takes classify_lean, a wave with
    one FDIR-marked packet (every 997th, no fdir array: mark 0) or without the
    NIC's hash flag on some frames takes the same counters through either
    path -- mbuf-pool offsets with ol_flags and hash.rss, every hash mode and
    verdict width, both settings, bit-exact against the oracle."""
    n, R, T, P = 40000, 16, 8, 8192
    hdr, olf_p, rss_p = orc.generate(0, P, 64, R)
    rng = np.random.default_rng(23 + mode + 10 * vb)
    pool = g.mbuf_data_offsets(P)
    order = np.concatenate([rng.permutation(P) for _ in range(-(-n // P))])[:n]
    offs = pool[order]
    olf = np.ascontiguousarray(olf_p[order])
    rss = np.ascontiguousarray(rss_p[order])
    olf[::13] &= ~np.uint8(g.F_RSS_HASH)
    olf[::997] |= np.uint8(g.F_FDIR_ID)
    region = np.zeros(g.mbuf_region_bytes(P), dtype=np.uint8)
    region[pool[:, None].astype(np.int64) + np.arange(64)] = hdr.reshape(P, 64)
    tb = g.thread_bits_for(R, T) if vb <= 2 else 0
    cflags = {8: 0, 4: g.CFG_VERDICT4, 2: g.CFG_VERDICT2, 1: g.CFG_VERDICT1}[vb]
    t = orc.Tables(R, mode, 0, 0x09, g.CALADAN_RSS_KEY)
    clf = g.Classifier(0, R, mode, cflags, 0x09, g.CALADAN_RSS_KEY, thread_bits=tb,
                       tune={"pair_lean": pair_lean})
    for r in range(R):
        act = (r * 5) % (T + 1)
        fl = orc.steer_flows(T, list(range(act))) if act else None
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
    ve, ce, se = t.classify(region, n, 0, offs=offs, olflags=olf, rss=rss)
    v, c, st = gpu_run(g, clf, region, n, 0, offs=offs, olflags=olf, rss=rss)
    assert se[g.RX_FLOW_TAG_MATCH] > 0 and se[g.RX_HASH_MISSING] > 0
    want = {8: lambda: ve, 4: lambda: to_verdict4(ve), 2: lambda: to_verdict2(ve, [T] * R, tb),
            1: lambda: to_verdict1(ve, [T] * R, tb)}[vb]()
    assert_same(v, want, f"pair lean={pair_lean} mode={mode} vb={vb}")
    assert (c == ce).all() and (st == se).all()


def test_gpu_ingress_integrated_nic_verdict2(g, orc):
    """The bench's integrated ingress shape (e2e.ingress_pool.integrated_nic,
    INTEGRATION.md §4): descriptors into the reference's mbuf pool geometry
    in random pool order, each with its mbuf's ol_flags and hash.rss,
    GCL_HASH_NIC, 2-byte queue verdicts -- bit-exact against the oracle."""
    n, R, T, P = 60000, 16, 8, 8192
    hdr, olf_p, rss_p = orc.generate(0, P, 64, R)
    rng = np.random.default_rng(17)
    pool = g.mbuf_data_offsets(P)
    order = np.concatenate([rng.permutation(P) for _ in range(-(-n // P))])[:n]
    offs = pool[order]
    olf = np.ascontiguousarray(olf_p[order])
    rss = np.ascontiguousarray(rss_p[order])
    olf[::7] &= ~np.uint8(g.F_RSS_HASH)  # some frames without the NIC's hash flag
    region = np.zeros(g.mbuf_region_bytes(P), dtype=np.uint8)
    region[pool[:, None].astype(np.int64) + np.arange(64)] = hdr.reshape(P, 64)
    tb = g.thread_bits_for(R, T)
    t = orc.Tables(R, g.HASH_NIC, 0, 0x09)
    clf = g.Classifier(0, R, g.HASH_NIC, g.CFG_VERDICT2, 0x09, thread_bits=tb)
    for r in range(R):
        act = (r * 5) % (T + 1)  # includes runtimes with no active kthread (WAKE)
        fl = orc.steer_flows(T, list(range(act))) if act else None
        t.runtime_set(r, orc.runtime_ip(r), T, act, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, act, fl)
    ve, ce, se = t.classify(region, n, 0, offs=offs, olflags=olf, rss=rss)
    v, c, st = gpu_run(g, clf, region, n, 0, offs=offs, olflags=olf, rss=rss)
    assert ((ve["action"] & 0x3F) == g.ACT_WAKE).any() and se[g.RX_HASH_MISSING] > 0
    assert_same(v, to_verdict2(ve, [T] * R, tb), "integrated ingress shape")
    assert (c == ce).all() and (st == se).all()


def test_gpu_trace_replay_zero_copy(g, orc, tmp_path):
    """Config 5's path: a pcap trace loaded into host memory, registered, and
    classified by the kernel straight over PCIe (gcl_classify_host ZEROCOPY)."""
    n, R, T = 20000, 16, 8
    pl = np.zeros(n, dtype=np.uint16)
    frames, olf, _ = orc.generate(2, n, 9216, R, pkt_len=pl)
    path = str(tmp_path / "t.pcap")
    g.pcap_write(path, frames, pl, stride=9216)
    tr = g.Trace(path)
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T + 1)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T + 1, fl)
    ve, ce, se = t.classify(tr.frames, n, 0, offs=tr.offs, olflags=olf, frames_len=tr.frames_len)
    hv = np.zeros(n, dtype=g.VERDICT_DTYPE)
    olf = np.ascontiguousarray(olf)
    for a in (tr.frames, tr.offs, olf, hv):
        g.host_register(a)
    try:
        counts = np.zeros(R, dtype=np.uint64)
        stats = np.zeros(8, dtype=np.uint64)
        clf.classify_host(tr.frames, n, 0, verdicts=hv, counts=counts, stats=stats, offs=tr.offs,
                          olflags=olf, frames_len=tr.frames_len, mode=g.E2E_ZEROCOPY)
    finally:
        for a in (tr.frames, tr.offs, olf, hv):
            g.host_unregister(a)
    assert_same(hv, ve, "trace replay")
    assert (counts == ce).all() and (stats == se).all()


@pytest.mark.parametrize("partner_mib", [24, 300])
def test_gpu_pair_probe_write_bound(g, partner_mib):
    """gcl_dev_alloc_paired's probe stores into the written side (the partner
    verdict ring here) only within min(partner_bytes, 256 MiB): a guard area
    past partner_bytes, and the ring's bytes past 256 MiB, keep their
    pattern.  The returned info names the bound and the classes seen."""
    import ctypes
    pb = partner_mib << 20
    guard = 4 << 20
    buf = torch.full((pb + guard,), 0xA5, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    out = ctypes.c_void_p()
    info = g.GclPairInfo()
    assert g.lib.gcl_dev_alloc_paired(0, 64 << 20, buf.data_ptr(), pb, g.PAIR_NEW_READS,
                                      ctypes.byref(out), ctypes.byref(info)) == 0
    try:
        wb = min(pb, 256 << 20)
        assert info.probe_write_bytes == wb
        assert 1 <= info.candidates <= g.PAIR_TRIES and info.classes in (1, 2)
        assert 0 < info.chosen_us <= info.worst_us
        tail = buf[wb:].cpu()
        assert bool((tail == 0xA5).all()), "probe wrote past min(partner_bytes, 256 MiB)"
    finally:
        g.lib.gcl_dev_free(out)


def test_gpu_dev_alloc_paired(g, orc):
    """Placement-aware allocation (gcl_dev_alloc_paired): both directions give
    working buffers, the probe times are sane, and a classify through the
    paired frame pool / verdict ring is bit-exact against the oracle."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    n, stride, R, T = 1 << 18, 64, 16, 8
    ring = g.DeviceBuffer(n * 4)
    pool = g.DeviceBuffer(n * stride, partner=ring, new_reads=True)
    assert pool.probe_us is not None and 0 < pool.probe_us[0] <= pool.probe_us[1]
    ring2 = g.DeviceBuffer(n * 4, partner=pool, new_reads=False)
    assert 0 < ring2.probe_us[0] <= ring2.probe_us[1]
    frames, _, _ = orc.generate(0, n, stride, R)
    assert hip.hipMemcpy(pool.data_ptr(), frames.ctypes.data, n * stride, 1) == 0  # H2D
    t = orc.Tables(R, 1, 0, 0x09)
    clf = g.Classifier(0, R, 1, g.CFG_VERDICT4, 0x09)
    for r in range(R):
        fl = orc.steer_flows(T, list(range(r % T + 1)))
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, fl)
        clf.runtime_set(r, g.runtime_ip(r), T, r % T + 1, fl)
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    s = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    clf.classify(pool, n, stride, verdicts=ring2, counts=c, stats=s)
    torch.cuda.synchronize()
    got = np.empty(n, dtype=g.VERDICT4_DTYPE)
    assert hip.hipMemcpy(got.ctypes.data, ring2.data_ptr(), n * 4, 2) == 0  # D2H
    ve, ce, se = t.classify(frames, n, stride)
    assert_same(got, to_verdict4(ve, [T] * R), "paired buffers")
    assert (c.cpu().numpy().astype(np.uint64) == ce).all()
    assert (s.cpu().numpy().astype(np.uint64) == se).all()
    for b in (ring2, pool, ring):
        b.free()


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gpu_tables_past_lds(g, orc, mode):
    """1500 runtimes of GCL_MAX_PROC = 4096, thread counts up to NCPU = 256
    (control.c:233): ~380 KiB of flow tables, past the 96 KiB LDS budget, so
    the kernel reads its tables from HBM."""
    rng = np.random.default_rng(8100 + mode)
    R = 4096
    rts = random_runtimes(rng, R, 1500, max_threads=256)
    assert sum(r["thread_count"] for r in rts) * 2 > 96 * 1024
    n = 20000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, R)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    t = orc.Tables(R, mode, 0, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, R, mode, 0, 0x09, key)
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                       frames_len=flen, hint=hint)
    assert_same(v, ve, f"tables past LDS mode={mode}")
    assert (c == ce).all() and (st == se).all()
    # the persistent loop keeps its tables in LDS: it refuses these
    g.host_register(frames)
    try:
        with pytest.raises(OSError) as e:
            clf.rxloop(frames)
        assert e.value.errno == 7  # E2BIG
    finally:
        g.host_unregister(frames)


def test_gpu_tables_in_hbm_forced(g, orc):
    """gcl_tune.tables = 1 keeps small tables in HBM too: same verdicts."""
    rng = np.random.default_rng(8200)
    R = 64
    rts = random_runtimes(rng, R, 40)
    n = 8000
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, R)
    t = orc.Tables(R, 1, 0, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, R, 1, 0, 0x09, tune={"tables": 1})
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                       frames_len=flen, hint=hint)
    assert_same(v, ve, "tables forced to HBM")
    assert (c == ce).all() and (st == se).all()


def test_gpu_ctx_tune_validation(g):
    """gcl_ctx_tune refuses a wrong struct size or a field out of range
    (-EINVAL) and keeps the previous settings; NULL restores the defaults."""
    clf = g.Classifier(0, 16, 1)
    ok = g.make_tune(threads=512, defer=0)
    assert g.lib.gcl_ctx_tune(clf._ctx, ctypes.byref(ok)) == 0
    bad = [g.make_tune(threads=300), g.make_tune(depth=3), g.make_tune(defer=3), g.make_tune(grid=0),
           g.make_tune(loop_phase=(2000, 1, 1)), g.make_tune(loop_phase=(10, 0, 0)), g.make_tune(loop_spec=-5),
           g.make_tune(rec_prefetch=65), g.make_tune(rec_prefetch=-2), g.make_tune(slot_prefetch=2),
           g.make_tune(vstage=3), g.make_tune(pair_i32=2), g.make_tune(tile_order=2)]
    half = g.make_tune()
    half.loop_phase_max = 50  # up / down left AUTO: the three go together
    bad.append(half)
    wrong = g.make_tune()
    wrong.size = 64
    bad.append(wrong)
    for t in bad:
        assert g.lib.gcl_ctx_tune(clf._ctx, ctypes.byref(t)) == -22
    assert g.lib.gcl_ctx_tune(clf._ctx, None) == 0
    clf.tune(tables=1, grid=3, depth=1)
    clf.close()


LOOP_GEOMETRIES = [
    {},
    {"grid": 3},
    {"grid": 16},
    {"grid": 24, "threads": 512},
    {"depth": 1, "grid": 5},
    {"depth": 1, "threads": 512},
    {"threads": 1024, "grid": 7},
    {"threads": 512, "grid": 5},
    {"blocks_per_cu": 1},
    {"tile_lean": 0, "grid": 16},
    {"tile_lean": 0, "depth": 1, "grid": 5},
]


@pytest.mark.parametrize("geo", range(len(LOOP_GEOMETRIES)))
@pytest.mark.parametrize("general", [False, True, "stride"])
def test_gpu_loop_geometries(g, orc, geo, general):
    """The loops' edges under every launch shape the geometry knobs allow:
    few blocks walking many tiles (odd counts per block, so the second half
    of the DEPTH-2 loop runs past the end as an empty tile), DEPTH 1,
    512/1024-lane tiles, one block per CU, for the dense tile kernel and the
    lane-pair GENERAL kernel; dense slots, per-frame offsets with
    ol_flags / hash.rss (NIC mode), and fixed slots with ol_flags / hash.rss
    and a buffer ending inside the last frame ("stride": the GENERAL path
    without offs[]), ragged n.  Same verdicts, counts, stats."""
    env = LOOP_GEOMETRIES[geo]
    rng = np.random.default_rng(9700 + 10 * geo + {False: 0, True: 1, "stride": 2}[general])
    R = 64
    rts = random_runtimes(rng, R, 40)
    mode = 0 if general is True else 1 if general is False else 2
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    t = orc.Tables(R, mode, 0, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, R, mode, 0, 0x09, key, tune=env)
    apply_runtimes(clf, rts)
    if general == "stride":
        n = 30011
        frames, _, _ = orc.generate(0, n, 64, R)
        olf = rng.integers(0, 16, size=n, dtype=np.uint8)
        rss = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        flen = (n - 1) * 64 + 37  # the last frame cut inside its header
        ve, ce, se = t.classify(frames, n, 64, olflags=olf, rss=rss, frames_len=flen)
        v, c, st = gpu_run(g, clf, frames, n, 64, olflags=olf, rss=rss, frames_len=flen)
    elif general:
        n = 20011
        frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, R, misalign="mixed")
        ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                                frames_len=flen)
        v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir,
                           frames_len=flen)
    else:
        n = 50001
        frames, _, _ = orc.generate(0, n, 64, R)
        ve, ce, se = t.classify(frames, n, 64)
        v, c, st = gpu_run(g, clf, frames, n, 64)
    assert_same(v, ve, f"geometry {env} general={general}")
    assert (c == ce).all() and (st == se).all()


def test_gpu_reference_struct_frames(g, orc):
    """Frames written through the reference's own inc/net structs classify on
    the GPU as the values put into the structs say.  The frames and expected
    (uniqid, hash) come from the committed fixture
    tests/golden/struct_frames_ref.npz (tests/golden/make_struct_frames.py,
    run in the container against oracle/_ref), so nothing built from
    reference sources is loaded here."""
    from tests.rxcases import load_struct_frames
    ips, frames, exp_u, hashes, hit = load_struct_frames()
    R, n = 64, len(frames)
    clf = g.Classifier(0, R, 1, 0, 0x09)
    for u, ip in enumerate(ips):
        clf.runtime_set(u, int(ip), 4, 4, [0, 1, 2, 3])
    v, c, st = gpu_run(g, clf, frames.reshape(-1), n, 64)
    exp_h = np.where(hit, hashes, 0).astype(np.uint32)
    assert (v["uniqid"] == exp_u).all()
    assert (v["hash"][hit] == exp_h[hit]).all()
    assert (v["thread"][hit] == exp_h[hit] % 4).all()
    assert ((v["action"][~hit] & 0x3F) == g.ACT_DROP_UNREG).all()
    assert int(c.sum()) == int(hit.sum())


@pytest.mark.parametrize("vbytes", [8, 4, 2, 1])
def test_gpu_post_pass_live_flow_tbl(g, orc, vbytes):
    """A GPU batch's verdicts through the host post-pass while sched_add_core
    side effects re-steer OTHER runtimes mid-batch (tests/schedmodel.py,
    sched.c:174-216): ring contents, counters and callbacks equal the serial
    per-packet model of rx.c:50-92, for all four verdict widths."""
    from tests.rxcases import fuzz_batch
    from tests.schedmodel import Sched, make_cprocs, rx_model, run_post_pass
    from tests.test_cabi import Ring
    R, ring, tb = (16 if vbytes == 1 else 64), 32, 3
    rng = np.random.default_rng(21)
    rts = random_runtimes(rng, R, 12 if vbytes == 1 else 24, max_threads=6)
    n = 3000
    frames, flen, offs, olf, rss, fdir, _ = fuzz_batch(rng, n, rts, R, tail_runts=False)
    t = orc.Tables(R, 0, 0x1, 0x09)
    apply_runtimes(t, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    flag = {8: 0, 4: g.CFG_VERDICT4, 2: g.CFG_VERDICT2, 1: g.CFG_VERDICT1}[vbytes]
    clf = g.Classifier(0, R, 0, 0x1 | flag, 0x09, thread_bits=tb if vbytes <= 2 else 0)
    apply_runtimes(clf, rts)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir, frames_len=flen)
    tc = {r["uniqid"]: r["thread_count"] for r in rts}
    exp = {8: ve, 4: to_verdict4(ve), 2: to_verdict2(ve, tc, tb), 1: to_verdict1(ve, tc, tb)}[vbytes]
    assert_same(v, exp, f"post-pass batch, {vbytes}-B verdicts")
    assert (c == ce).all() and (st == se).all()
    pkt_len = rng.integers(60, 1515, size=n).astype(np.uint16)
    shm, bh = offs.astype(np.uint64), rss.astype(np.uint32)
    order = [r["uniqid"] for r in rts]
    arp_ok = lambda i: i % 2 == 0  # noqa: E731
    want = rx_model(Sched(rts, 5, np.random.default_rng(5)), ve, order, ring, pkt_len, olf, shm, bh,
                    arp_ok)
    assert any(e[0] == "disable" and e[3] == 0 for e in want[2])
    S = Sched(rts, 5, np.random.default_rng(5))
    cprocs, rings = make_cprocs(g, S, ring, Ring)
    got = run_post_pass(g, S, cprocs, rings, vbytes, np.ascontiguousarray(v), R, order, pkt_len, olf,
                        shm, bh, arp_ok, thread_bits=tb)
    assert got == want


def test_gpu_rejects_oversized_batch(g):
    """n > 2^40 is refused before any launch (n * stride must not wrap)."""
    import ctypes
    clf = g.Classifier(0, 16, 1)
    f = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    v = torch.zeros(64, dtype=torch.uint8, device="cuda")
    b = g.GclBatch(frames=f.data_ptr(), frames_len=4096, stride=64, n=(1 << 40) + 1)
    o = g.GclOut(verdicts=v.data_ptr())
    assert g.lib.gcl_classify_ex(clf._ctx, ctypes.byref(b), ctypes.byref(o), None) == -22


def test_gpu_toeplitz_reference_vectors(g):
    """TOEPLITZ mode on the GPU reproduces the reference's own do_toeplitz
    outputs (tests/golden/toeplitz_ref.json, generated by the reference
    compiled in place): one Eth/IPv4/TCP frame per vector, every key of the
    fixture in its own context, the hash read from the 8-B verdict."""
    import struct
    from tests.rxcases import load_json
    d = load_json("toeplitz_ref.json")
    for ki, khex in enumerate(d["keys"]):
        vecs = [v for v in d["vectors"] if v["key"] == ki]
        n = len(vecs)
        frames = np.zeros(n * 64, dtype=np.uint8)
        for i, v in enumerate(vecs):
            ip = struct.pack("!BBHHHBBHII", 0x45, 0, 40, 1, 0, 64, 6, 0, v["saddr"], v["daddr"])
            fr = bytes(12) + b"\x08\x00" + ip + struct.pack("!HH", v["sport"], v["dport"])
            frames[64 * i:64 * i + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
        clf = g.Classifier(0, 16, g.HASH_TOEPLITZ, 0, 0x09, bytes.fromhex(khex))
        ver, _, _ = gpu_run(g, clf, frames, n, 64)
        want = np.array([v["hash"] for v in vecs], dtype=np.uint32)
        bad = np.nonzero(ver["hash"] != want)[0]
        assert len(bad) == 0, f"key {ki}: {len(bad)} hashes differ, first {vecs[bad[0]]} gpu={ver['hash'][bad[0]]:#x}"


def test_gpu_trans_hash_reference_vectors(g):
    """The transport demux pre-hash on the GPU (GCL_CFG_TRANS_HASH) equals
    the reference's own trans_hash_5tuple/3tuple (tests/golden/trans_ref.json,
    generated by runtime/net/transport.c compiled in place) for IPv4 TCP/UDP
    frames delivered to 16 runtimes, each with its own trans_seed."""
    import struct
    from tests.rxcases import load_json
    d = load_json("trans_ref.json")
    vecs = d["frames"]
    n = len(vecs)
    frames = np.zeros(n * 64, dtype=np.uint8)
    for i, v in enumerate(vecs):
        ip = struct.pack("!BBHHHBBHII", 0x45, 0, 40, 1, 0x4000, 64, v["proto"], 0, v["saddr"],
                         d["runtime_ips"][v["runtime"]])
        fr = bytes(12) + b"\x08\x00" + ip + struct.pack("!HH", v["sport"], v["dport"])
        frames[64 * i:64 * i + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
    clf = g.Classifier(0, 16, g.HASH_NIC, g.CFG_TRANS_HASH, 0x09)
    for r, (ip, seed) in enumerate(zip(d["runtime_ips"], d["trans_seeds"])):
        clf.runtime_set(r, ip, 4, 4, [0, 1, 2, 3])
        clf.set_trans_seed(r, seed)
    ver, _, _, tr = gpu_run(g, clf, frames, n, 64, trans=True)
    assert (ver["uniqid"] == np.array([v["runtime"] for v in vecs])).all()
    assert (tr["h5"] == np.array([v["h5"] for v in vecs], dtype=np.uint32)).all()
    assert (tr["h3"] == np.array([v["h3"] for v in vecs], dtype=np.uint32)).all()


def test_gpu_ip_hdr_supported_reference(g):
    """The GPU sets the transport pre-hash (GCL_ACT_F_TRANS) exactly on the
    frames the reference's own ip_hdr_supported accepts
    (tests/golden/iphdr_ref.json: 256 version/IHL bytes x 10 fragment
    fields, generated by runtime/net/core.c compiled in place)."""
    from tests.rxcases import load_json
    from tests.test_kats import _iphdr_frames
    d = load_json("iphdr_ref.json")
    ip = 0x0A000001
    clf = g.Classifier(0, 16, g.HASH_NIC, g.CFG_TRANS_HASH, 0x09)
    clf.runtime_set(0, ip, 4, 4, [0, 1, 2, 3])
    n = len(d["headers"])
    v, _, _, _ = gpu_run(g, clf, _iphdr_frames(d, ip), n, 64, trans=True)
    got = (v["action"] & g.ACT_F_TRANS) != 0
    want = np.array([h["supported"] for h in d["headers"]])
    assert (got == want).all(), np.nonzero(got != want)[0][:5]


@pytest.mark.parametrize("pattern", ["arp", "ipv4"])
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_general_frames_at_the_end(g, orc, mode, pattern):
    """Frames at every byte offset from 80 bytes before frames_len to 8
    past it, over a tail whose bytes repeat 08 06 (ARP) or 08 00 (IPv4), so
    every other offset parses as that Ethertype and its destination (the ARP
    target at bytes 38-41, daddr at 30-33) is a registered runtime -- until
    the bytes it needs run past frames_len and read 0 (the build's rule; the
    bytes behind frames_len hold 0xEE).  This walks the pair kernel from its
    16-B loads of [8, 40) to bytewise reads and the ARP target from one
    dword load to bytewise, each against the oracle."""
    kernel = "pair"
    rng = np.random.default_rng(4400 + mode + 100 * (pattern == "ipv4"))
    R = 16
    unit = b"\x08\x06" if pattern == "arp" else b"\x08\x00"
    word = int.from_bytes(unit * 2, "big")  # the IP the pattern reads as, host order
    ips = [word, int.from_bytes(unit[::-1] * 2, "big")] + [0x0A000001 + r for r in range(R - 2)]
    flen = 4096 + 37
    frames = np.full(flen + 256, 0xEE, dtype=np.uint8)
    frames[:flen] = rng.integers(0, 256, size=flen, dtype=np.uint8)
    frames[flen - 96:flen] = np.frombuffer(unit * 48, dtype=np.uint8)
    offs = np.arange(flen - 80, flen + 8, dtype=np.uint64)
    offs = np.concatenate([offs, offs[::-1]])
    n = len(offs)
    olf = rng.integers(0, 16, size=n, dtype=np.uint8)
    rss = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    t = orc.Tables(R, mode, 0, 0x09)
    for r, ip in enumerate(ips):
        assert t.runtime_set(r, ip, 4, 4, [0, 1, 2, 3]) == 0
    clf = g.Classifier(0, R, mode, 0, 0x09)
    for r, ip in enumerate(ips):
        clf.runtime_set(r, ip, 4, 4, [0, 1, 2, 3])
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, frames_len=flen)
    assert_same(v, ve, f"{kernel} mode={mode} {pattern} at the end")
    assert (c == ce).all() and (st == se).all()
    acts = ve["action"] & 0x3F
    # both outcomes occur: registered destinations, and ones cut by frames_len
    assert (acts == g.ACT_DELIVER).sum() > 10 and (acts == g.ACT_DROP_UNREG).sum() > 4


@pytest.mark.parametrize("order", ["random", "working_set"])
def test_gpu_full_size_ingress_pool(g, orc, order):
    """The integrated rx_burst shape at the bench's full size, on the GENERAL
    path's default kernel (the lane-pair kernel): 8 Mi descriptors into the
    reference's 131072-mbuf ingress pool (9408-B elements, frame data at
    element + 344), each with its mbuf's ol_flags and hash.rss, NIC mode,
    2-byte queue verdicts, the region placed against the verdict ring as
    bench.ingress_pool_bench places it -- in random order over the whole
    pool and over a 4096-mbuf working set.  Every packet is accounted for,
    the queue histogram equals the device counts, and a 65536-descriptor
    sample equals the oracle bit for bit."""
    import bench
    from tests.rxcases import to_verdict2
    dev = torch.device("cuda", 0)
    wl, _, _, R, T, _ = bench.WORKLOADS["udp64"]
    P, n = g.IOKERNEL_NUM_MBUFS, 8 << 20
    hdr = torch.zeros(P * 64, dtype=torch.uint8, device=dev)
    olf_p = torch.zeros(P, dtype=torch.uint8, device=dev)
    rss_p = torch.zeros(P, dtype=torch.int32, device=dev)
    g.generate(wl, P, 64, R, hdr, olflags=olf_p, rss=rss_p, seed=bench.SEED)
    pool_offs = torch.from_numpy(g.mbuf_data_offsets(P).view(np.int64)).to(dev)
    region = torch.zeros(g.mbuf_region_bytes(P), dtype=torch.uint8, device=dev)
    region[(pool_offs[:, None] + torch.arange(64, device=dev)).view(-1)] = hdr
    gen = torch.Generator(device="cpu").manual_seed(bench.SEED + (order == "working_set"))
    if order == "random":
        sel = torch.cat([torch.randperm(P, generator=gen) for _ in range(n // P)])
    else:
        sub = torch.randperm(P, generator=gen)[:bench.INGRESS_WORKING_SET]
        sel = torch.cat([sub[torch.randperm(len(sub), generator=gen)] for _ in range(n // len(sub))])
    sel = sel.to(dev)
    offs, olf, rss = pool_offs[sel].contiguous(), olf_p[sel].contiguous(), rss_p[sel].contiguous()
    dv = g.DeviceBuffer(n * 2, 0)
    placed = g.DeviceBuffer(region.numel(), 0, partner=dv, vbytes=2)
    torch.cuda.synchronize()
    bench.hip_copy(placed, region, region.numel())
    clf = bench.classifier(dev, R, T, 2, hash_mode=g.HASH_NIC)
    tables = bench.setup_tables(clf, R, T)
    assert clf.thread_bits == 3
    cnt = torch.zeros(R + g.NR_STATS, dtype=torch.int64, device=dev)
    clf.classify(placed, n, 0, verdicts=dv, counts=cnt[:R], stats=cnt[R:], offs=offs, olflags=olf,
                 rss=rss, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hv = torch.empty(n * 2, dtype=torch.uint8).pin_memory()
    bench.hip_copy(hv, dv, n * 2)
    q = hv.numpy().view(np.uint16)
    cc, ss = cnt[:R].cpu().numpy(), cnt[R:].cpu().numpy()
    assert cc.sum() == n and ss[g.RX_PULLED] == n and ss[g.RX_UNHANDLED] == 0
    assert ((q & g.V2_KIND) == g.V2_DELIVER).all()
    assert (np.bincount(q >> 3, minlength=R)[:R] == cc).all()
    rng = np.random.default_rng(77)
    sample = np.sort(rng.choice(n, size=65536, replace=False))
    sidx = torch.from_numpy(sample).to(dev)
    so = offs[sidx]
    fr = region[(so[:, None] + torch.arange(64, device=dev)).view(-1)].cpu().numpy()
    t = orc.Tables(R, g.HASH_NIC, 0, 0x09)
    for (r, ip, TT, act, fl) in tables:
        assert t.runtime_set(r, ip, TT, act, fl) == 0
    ve, _, _ = t.classify(fr, len(sample), 64, olflags=olf[sidx].cpu().numpy(),
                          rss=rss[sidx].cpu().numpy().view(np.uint32))
    want = to_verdict2(ve, {r: TT for (r, _, TT, _, _) in tables}, 3)
    assert_same(q[sample], want, f"ingress pool {order} sample")
    del region, placed, dv
    torch.cuda.empty_cache()


@pytest.mark.parametrize("vbytes", [2, 4, 8])
def test_gpu_access_probe(g, vbytes):
    """gcl_access_probe's minimal-request form (GCL_PROBE_MIN; the layout's
    ceiling) reads what it claims: packet p's stored word is the XOR of the
    four dwords of the 16-B chunk holding its frame byte 0 and of the first
    dword of the next line's chunk when frame bytes [0, 40) cross into it
    (fixed slots, and offsets that straddle lines)."""
    rng = np.random.default_rng(99)
    n, stride = 5000, 1536
    frames = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    clf = g.Classifier(0, 16, 1)
    f = dev(frames)
    out = torch.zeros(n * vbytes, dtype=torch.uint8, device="cuda")
    dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[vbytes]
    mask = {2: 0xFFFF, 4: 0xFFFFFFFF, 8: 0xFFFFFFFF}[vbytes]

    def want(offs):
        x = np.zeros(n, dtype=np.uint64)
        for i, o in enumerate(offs):
            a0 = int(o) & ~15
            w = frames[a0:a0 + 16].view(np.uint32)
            v = int(w[0] ^ w[1] ^ w[2] ^ w[3])
            a1 = (int(o) + 39) & ~127
            if a1 > a0:
                v ^= int(frames[a1:a1 + 4].view(np.uint32)[0])
            x[i] = v
        return x & np.uint64(mask)

    clf.access_probe(f, n, stride, out=out, vbytes=vbytes, minimal=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(dt).astype(np.uint64)
    assert (got == want(np.arange(n, dtype=np.uint64) * np.uint64(stride))).all()
    offs = rng.permutation(n).astype(np.uint64) * np.uint64(stride) + \
        rng.choice([0, 8, 88, 96, 100, 120], size=n).astype(np.uint64)
    out.zero_()
    clf.access_probe(f, n, 0, out=out, vbytes=vbytes, offs=dev(offs.astype(np.int64)), minimal=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(dt).astype(np.uint64)
    assert (got == want(offs)).all()


@pytest.mark.parametrize("vb,R,T,stride,tune", [(1, 16, 8, 64, {}), (2, 16, 8, 64, {"defer": 2, "grid": 7}),
                                                (2, 1024, 4, 1536, {}), (8, 16, 8, 64, {}),
                                                (1, 16, 8, 64, {"defer": 0, "depth": 1}),
                                                (1, 16, 8, 64, {"vstage": 1, "grid": 40})])
def test_gpu_access_probe_kernel_shape(g, vb, R, T, stride, tune):
    """gcl_access_probe on a dense batch at the context's verdict width is the
    classify launch itself with rx_one_pkt folded away (the kernel's own
    ceiling): packet p's output is the low vb bytes of the XOR of the header
    dwords rx_one_pkt reads (frame dwords 3 and 5-10), written through the
    same deferred or per-packet verdict path; the ragged last tile is cut at
    n (a guard byte past it stays)."""
    rng = np.random.default_rng(1500 + vb + stride + len(tune))
    n = (1 << 18) + 77
    frames = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    fl, tb = {1: (g.CFG_VERDICT1, 3), 2: (g.CFG_VERDICT2, 2 if R == 1024 else 3), 8: (0, 0)}[vb]
    clf = g.Classifier(0, R, 1, fl, thread_bits=tb, tune=tune)
    clf.runtime_set(0, g.runtime_ip(0), T, T, g.steer_flows(T, list(range(T))))
    out = torch.full((n * vb + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    clf.access_probe(dev(frames), n, stride, out=out)
    torch.cuda.synchronize()
    d = frames.reshape(n, stride)[:, :44].view(np.uint32)
    x = d[:, 3] ^ d[:, 5] ^ d[:, 6] ^ d[:, 7] ^ d[:, 8] ^ d[:, 9] ^ d[:, 10]
    got = out.cpu().numpy()
    if vb == 8:
        assert (got[:n * 8].view(np.uint64) == x.astype(np.uint64)).all()
    else:
        want = (x & np.uint32((1 << (8 * vb)) - 1)).astype({1: np.uint8, 2: np.uint16}[vb])
        assert (got[:n * vb].view(want.dtype) == want).all()
    assert (got[n * vb:] == 0xEE).all()
    clf.close()


@pytest.mark.parametrize("vb,mode,side", [(2, 0, True), (2, 1, True), (8, 0, False), (4, 0, True), (1, 2, True)])
def test_gpu_access_probe_pair_shape(g, vb, mode, side):
    """gcl_access_probe on a batch with offsets at the context's verdict
    width is classify_pair_kernel in probe mode: packet p's output is the low
    vb bytes of the XOR of frame dwords 3 and 5-9 at its offset (bytes past
    frames_len read 0; frames at every alignment, some straddling the end),
    its ol_flags byte, and its hash.rss in a NIC-mode context only."""
    rng = np.random.default_rng(1700 + vb + 10 * mode + side)
    n, flen = 20000 + 37, 1 << 21
    frames = rng.integers(0, 256, size=flen, dtype=np.uint8)
    offs = rng.integers(0, flen - 40, size=n).astype(np.uint64)
    offs[:50] = flen - rng.integers(1, 40, size=50)  # ragged at the end
    offs[50:60] = flen + rng.integers(0, 1000, size=10)  # past it: zeros
    olf = rng.integers(0, 256, size=n, dtype=np.uint8)
    rss = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    fl = {1: g.CFG_VERDICT1, 2: g.CFG_VERDICT2, 4: g.CFG_VERDICT4, 8: 0}[vb]
    clf = g.Classifier(0, 16, mode, fl, thread_bits=3)
    out = torch.full((n * vb + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    kw = {"olflags": dev(olf), "rss": dev(rss.view(np.int32))} if side else {}
    clf.access_probe(dev(frames), n, 0, out=out, offs=dev(offs.astype(np.int64)), **kw)
    torch.cuda.synchronize()
    pad = np.concatenate([frames, np.zeros(64, dtype=np.uint8)])
    x = np.zeros(n, dtype=np.uint32)
    for i, o in enumerate(offs):
        o = int(o)
        h = pad[o:o + 40] if o < flen else np.zeros(40, dtype=np.uint8)
        h = np.concatenate([h[:max(0, flen - o)], np.zeros(40, dtype=np.uint8)])[:40].view(np.uint32)
        x[i] = h[3] ^ h[5] ^ h[6] ^ h[7] ^ h[8] ^ h[9]
    if side:
        x ^= olf.astype(np.uint32)
        if mode == 0:  # NIC mode: the context's launch loads hash.rss
            x ^= rss
    got = out.cpu().numpy()
    want = {1: x.astype(np.uint8), 2: x.astype(np.uint16), 4: x, 8: x.astype(np.uint64)}[vb]
    assert (got[:n * vb].view(want.dtype) == want).all()
    assert (got[n * vb:] == 0xEE).all()
    clf.close()


@pytest.mark.parametrize("i32", [1, 0])
def test_gpu_offsets_at_the_top_of_u64(g, orc, i32):
    """Offsets at and near 2^64 - 1 (the kernels' no-packet sentinel, ~0),
    2^63 and frames_len read as frames of zeros like any offset past the
    buffer in the GENERAL kernel, in its 32- and 64-bit forms; gcl_classify
    refuses frames_len == ~0."""
    kernel = "pair"
    rng = np.random.default_rng(9501)
    rts = random_runtimes(rng, 16, 12)
    n = 3001
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, 16, tail_runts=False)
    top = np.array([2**64 - 1, 2**64 - 2, 2**64 - 16, 2**63, flen, flen - 1, flen + 7], dtype=np.uint64)
    idx = rng.choice(n, size=300, replace=False)
    offs = offs.copy()
    offs[idx] = top[np.arange(300) % len(top)]
    t = orc.Tables(16, 1, 0, 0x09)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, 16, 1, 0, 0x09, tune={"pair_i32": i32})
    apply_runtimes(clf, rts)
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir, frames_len=flen)
    v, c, st = gpu_run(g, clf, frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir=fdir, frames_len=flen)
    assert_same(v, ve, f"top-of-u64 offsets, {kernel} i32={i32}")
    assert (c == ce).all() and (st == se).all()
    import ctypes
    f, o = dev(frames), dev(offs.astype(np.int64))
    vb = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    b = g.GclBatch(frames=f.data_ptr(), frames_len=2**64 - 1, stride=0, offs=o.data_ptr(), n=n)
    out = g.GclOut(verdicts=vb.data_ptr())
    assert g.lib.gcl_classify_ex(clf._ctx, ctypes.byref(b), ctypes.byref(out), None) == -22


@pytest.mark.parametrize("misalign", [None, "mixed", "lineend"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gpu_copy_transport_fuzz(g, orc, misalign, mode):
    """gcl_classify_host's COPY transport on the fuzz: per-packet offsets at
    any alignment through the header gather kernel (frames straddling
    frames_len, IHL up to 15 with ports up to byte 78, ARP target IPs), and
    fixed 128-B slots through the 2D DMA of 80-B rows -- both bit-exact
    against the oracle with ol_flags, hash.rss, FDIR marks and hints."""
    rng = np.random.default_rng(9700 + 10 * mode + [None, "mixed", "lineend"].index(misalign))
    rts = random_runtimes(rng, 64, 40)
    n = 6001
    slot = 256 if misalign == "lineend" else 128
    frames, flen, offs, olf, rss, fdir, hint = fuzz_batch(rng, n, rts, 64, slot=slot, misalign=misalign)
    key = bytes(rng.integers(0, 256, size=40, dtype=np.uint8))
    t = orc.Tables(64, mode, 0, 0x09, key)
    apply_runtimes(t, rts)
    clf = g.Classifier(0, 64, mode, 0, 0x09, key)
    apply_runtimes(clf, rts)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory()  # noqa: E731
    hr = pin(frames)
    side = dict(olflags=pin(olf), rss=pin(rss.view(np.int32)), fdir_hi=pin(fdir.view(np.int32)),
                dst_hint=pin(hint.view(np.int32)))
    # offsets
    ve, ce, se = t.classify(frames, n, 0, offs=offs, olflags=olf, rss=rss, fdir_hi=fdir,
                            frames_len=flen, dst_hint=hint)
    hv = torch.zeros(n * 8, dtype=torch.uint8).pin_memory()
    counts, stats = np.zeros(64, dtype=np.uint64), np.zeros(8, dtype=np.uint64)
    clf.classify_host(hr, n, 0, verdicts=hv, counts=counts, stats=stats, offs=pin(offs.view(np.int64)),
                      frames_len=flen, mode=g.E2E_COPY, chunk=2048 + 5, nstreams=3, **side)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, f"copy offsets {misalign} mode={mode}")
    assert (counts == ce).all() and (stats == se).all()
    # offsets in pageable memory: copied into the chunk's side buffer beside
    # the other arrays, whose sub-arrays stay 16-B aligned at an odd chunk
    hv.zero_()
    counts, stats = np.zeros(64, dtype=np.uint64), np.zeros(8, dtype=np.uint64)
    clf.classify_host(hr, n, 0, verdicts=hv, counts=counts, stats=stats,
                      offs=np.ascontiguousarray(offs.view(np.int64)), frames_len=flen, mode=g.E2E_COPY,
                      chunk=1000 + 3, nstreams=2, **side)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, f"copy pageable offsets {misalign} mode={mode}")
    assert (counts == ce).all() and (stats == se).all()
    if misalign is not None:
        return
    # fixed slots: the same buffer as n_slots x 128-B frames in slot order
    ns = len(frames) // slot
    ve, ce, se = t.classify(frames, ns, slot)
    hv = torch.zeros(ns * 8, dtype=torch.uint8).pin_memory()
    counts, stats = np.zeros(64, dtype=np.uint64), np.zeros(8, dtype=np.uint64)
    clf.classify_host(hr, ns, slot, verdicts=hv, counts=counts, stats=stats, mode=g.E2E_COPY,
                      chunk=1000, nstreams=2)
    assert_same(hv.numpy().view(g.VERDICT_DTYPE), ve, f"copy slots mode={mode}")
    assert (counts == ce).all() and (stats == se).all()
