"""The multi-GPU group behind the C ABI (include/gcl_group.h) on the GPU.

* A one-GPU group whose counters go through RCCL (ncclCommInitAll +
  ncclAllGather): three classify + exchange rounds give node-wide counts and
  counters exactly k times the single-context run, and the same verdicts.
* Two contexts of one group sharing the box's GPU (host exchange: RCCL
  refuses two ranks of one communicator on one device) classify the two
  round-robin shards of one batch: every verdict equals the oracle's on the
  whole batch at the shard's global positions, and the node-wide counts equal
  the single-context counts of the whole batch.
* One host batch split by the C splitter over two contexts (zero-copy and
  header DMA-gather, fixed slots and per-packet offsets, NIC-mode side
  arrays, a ragged last block) equals the oracle.
* torch.distributed's RCCL path (ProcessGroupNCCL, one rank) runs the bench's
  all_gather of the counts vector.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

R, T = 16, 8


@pytest.fixture(scope="module")
def g():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from caladan_amd import gclassify
    gclassify.group_lib()
    return gclassify


def tables(target):
    rng = np.random.default_rng(0xCA1ADA4)
    from oracle import orc
    for r in range(R):
        act = int(rng.integers(0, T + 1))  # zero-active runtimes too (WAKE)
        idx = [int(x) for x in rng.choice(T, size=act, replace=False)]
        fl = orc.steer_flows(T, idx) if act else None
        ret = target.runtime_set(r, orc.runtime_ip(r), T, act, fl)
        assert ret in (0, None)


def pinned(a):
    """A copy of numpy array @a in pinned host memory (hipHostMalloc through
    torch), as a numpy view: mapped for zero-copy without registration."""
    t = torch.empty(a.nbytes, dtype=torch.uint8).pin_memory()
    v = t.numpy().view(a.dtype)
    v[:] = a.reshape(-1)
    pinned.keep.append(t)
    return v


pinned.keep = []


def single_run(g, frames_dev, n, stride, hash_mode=1, flags=0, **side):
    clf = g.Classifier(0, R, hash_mode, flags)
    tables(clf)
    v = torch.zeros(n * clf.vbytes, dtype=torch.uint8, device="cuda")
    c = torch.zeros(R, dtype=torch.int64, device="cuda")
    s = torch.zeros(g.NR_STATS, dtype=torch.int64, device="cuda")
    clf.classify(frames_dev, n, stride, verdicts=v, counts=c, stats=s, **side)
    torch.cuda.synchronize()
    out = (v.cpu().numpy().view(g.verdict_dtype(clf.vbytes)), c.cpu().numpy().astype(np.uint64),
           s.cpu().numpy().astype(np.uint64))
    clf.close()
    return out


def test_gpu_group_rccl_one_device(g):
    """RCCL executes: a 1-GPU group, three classify + exchange rounds, each
    read equal to k x the single-context counts and counters."""
    n, stride = (1 << 20) + 4321, 64
    fr = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    g.generate(g.WL_UDP64, n, stride, R, fr)
    ve, ce, se = single_run(g, fr, n, stride)
    grp = g.Group([0], R, g.HASH_JENKINS, exchange=g.XCHG_RCCL)
    tables(grp)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    shard = {"frames": fr, "n": n, "stride": stride}
    for k in range(1, 4):
        grp.classify([shard], [v])
        grp.exchange()
        c, s, per = grp.read()
        assert (c == k * ce).all(), (k, c, ce)
        assert (s == k * se).all(), (k, s, se)
        assert (per[0, :R] == c).all() and (per[0, R:] == s).all()
    grp.sync()
    assert (v.cpu().numpy().view(g.VERDICT_DTYPE) == ve).all()
    # overlapped: two batches per exchange, exchanges back to back, one read
    for _ in range(4):
        grp.classify([shard], [v])
        grp.classify([shard], [v])
        grp.exchange()
    c, s, _ = grp.read()
    assert (c == 11 * ce).all() and (s == 11 * se).all()
    grp.reset()
    grp.exchange()
    c, s, _ = grp.read()
    assert not c.any() and not s.any()
    grp.close()


@pytest.mark.parametrize("xchg", ["rccl", "host"])
def test_gpu_group_reset_orders_before_exchange(g, xchg):
    """gcl_group_reset's zeroing completes before it returns, ahead of any
    later work on the group's non-blocking streams: 25 rounds of classify,
    exchange, reset, exchange, classify, exchange each read zero after the
    reset and exactly one batch after it (round 5 caught a null-stream
    hipMemset racing the next exchange's snapshot)."""
    n, stride = (1 << 18) + 77, 64
    fr = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    g.generate(g.WL_UDP64, n, stride, R, fr)
    _, ce, se = single_run(g, fr, n, stride)
    grp = g.Group([0], R, g.HASH_JENKINS, exchange=g.XCHG_RCCL if xchg == "rccl" else g.XCHG_HOST)
    tables(grp)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    shard = {"frames": fr, "n": n, "stride": stride}
    try:
        for k in range(25):
            grp.classify([shard], [v])
            grp.exchange()
            grp.reset()
            grp.exchange()
            c, s, _ = grp.read()
            assert not c.any() and not s.any(), (k, c, s)
            grp.classify([shard], [v])
            grp.exchange()
            c, s, _ = grp.read()
            assert (c == ce).all() and (s == se).all(), (k, c, ce)
            grp.reset()
    finally:
        grp.close()


@pytest.mark.parametrize("vbytes", [8, 2])
def test_gpu_group_shards_two_contexts(g, orc, vbytes):
    """Two contexts on the one GPU, each classifying its round-robin shard
    (generated in place with rank/world, as each GPU's HBM would hold it):
    verdicts equal the oracle's on the whole batch at the shard positions,
    node counts equal the whole batch's."""
    from caladan_amd import shard
    from tests.rxcases import to_verdict2
    W, B = 2, 64 << 10
    n_glob = 5 * B + 1234
    stride = 64
    flags = g.CFG_VERDICT2 if vbytes == 2 else 0
    tb = 3 if vbytes == 2 else 0
    grp = g.Group([0, 0], R, g.HASH_JENKINS, flags=flags, thread_bits=tb, block=B,
                  exchange=g.XCHG_HOST)
    tables(grp)
    shards, vs = [], []
    for r in range(W):
        m = g.shard_count(n_glob, W, r, B)
        fr = torch.zeros(max(m, 1) * stride, dtype=torch.uint8, device="cuda")
        g.generate(g.WL_UDP64, m, stride, R, fr, rank=r, world=W, shard_block=B)
        shards.append({"frames": fr, "n": m, "stride": stride})
        vs.append(torch.zeros(max(m, 1) * vbytes, dtype=torch.uint8, device="cuda"))
    grp.classify(shards, vs)
    grp.exchange()
    c, s, per = grp.read()
    frames, _, _ = orc.generate(g.WL_UDP64, n_glob, stride, R)
    t = orc.Tables(R, 1, 0, 0x09)
    tables(t)
    ve, ce, se = t.classify(frames, n_glob, stride)
    if vbytes == 2:
        tc = {r: T for r in range(R)}
        ve = to_verdict2(ve, tc, tb)
    for r in range(W):
        idx = shard.shard_indices(n_glob, r, W, B)
        got = vs[r].cpu().numpy().view(g.verdict_dtype(vbytes))[:len(idx)]
        assert (got == ve[idx]).all(), r
    assert (c == ce).all() and (s == se).all()
    assert (per.sum(axis=0)[:R] == ce).all()
    assert int(per[0, R + g.RX_PULLED]) == g.shard_count(n_glob, W, 0, B)
    grp.close()


@pytest.mark.parametrize("nstreams", [1, 4])
@pytest.mark.parametrize("mode", ["zerocopy", "copy"])
@pytest.mark.parametrize("layout", ["slots1536", "offs"])
def test_gpu_group_classify_host_split(g, orc, mode, layout, nstreams):
    """One host batch split round-robin by the C splitter over two contexts:
    the verdicts land at their batch positions and equal the oracle's; the
    node-wide counts and counters equal the oracle's (NIC mode with ol_flags
    and hash.rss, a ragged last block).  COPY over per-packet offsets goes
    through gcl_header_gather on each GPU, fixed slots through 2D DMA."""
    B = 4096
    n = 5 * B + 77
    rng = np.random.default_rng(3)
    if layout == "slots1536":
        stride = 1536
        frames, olf, rss = orc.generate(g.WL_TCP1500_ZIPF, n, stride, R, cdf=g.zipf_cdf(1 << 12))
        offs = None
    else:
        stride = 0
        hdr, olf, rss = orc.generate(g.WL_UDP64, n, 64, R)
        slots = rng.permutation(n + 100)[:n].astype(np.uint64)
        offs = slots * np.uint64(192) + np.uint64(8)  # mbuf-like 8-B-aligned data
        frames = np.zeros((n + 100) * 192, dtype=np.uint8)
        for i in range(n):
            o = int(offs[i])
            frames[o:o + 64] = hdr[i * 64:(i + 1) * 64]
    hv = pinned(np.zeros(n, dtype=g.VERDICT_DTYPE))
    # opened with one stream per GPU; the batch asks for `nstreams`
    grp = g.Group([0, 0], R, g.HASH_NIC, block=B, exchange=g.XCHG_HOST, nstreams=1)
    tables(grp)
    kw = dict(verdicts=hv, nstreams=nstreams, offs=None if offs is None else pinned(offs),
              olflags=pinned(olf), rss=pinned(rss),
              mode=g.E2E_ZEROCOPY if mode == "zerocopy" else g.E2E_COPY)
    grp.classify_host(pinned(frames), n, stride, **kw)
    grp.exchange()
    c, s, per = grp.read()
    t = orc.Tables(R, 0, 0, 0x09)
    tables(t)
    ve, ce, se = t.classify(frames, n, stride, offs=offs, olflags=olf, rss=rss)
    assert (hv == ve).all(), np.nonzero(hv != ve)[0][:5]
    assert (c == ce).all() and (s == se).all()
    # GPU 0 took blocks 0, 2, 4; GPU 1 blocks 1, 3 and the ragged 5
    assert int(per[0, R + g.RX_PULLED]) == 3 * B and int(per[1, R + g.RX_PULLED]) == 2 * B + 77
    grp.close()


def test_gpu_group_rccl_classify_host(g, orc):
    """The host-batch split through a 1-GPU RCCL group (zero-copy)."""
    n, B = 3 * 4096 + 5, 4096
    frames, olf, rss = orc.generate(g.WL_UDP64, n, 64, R)
    hv = pinned(np.zeros(n, dtype=g.VERDICT_DTYPE))
    grp = g.Group([0], R, g.HASH_JENKINS, block=B)
    tables(grp)
    grp.classify_host(pinned(frames), n, 64, verdicts=hv, mode=g.E2E_ZEROCOPY)
    grp.exchange()
    c, s, _ = grp.read()
    t = orc.Tables(R, 1, 0, 0x09)
    tables(t)
    ve, ce, se = t.classify(frames, n, 64)
    assert (hv == ve).all() and (c == ce).all() and (s == se).all()
    grp.close()


def test_gpu_grouppipe_c_driver(g):
    """tools/grouppipe (the group driven from C, as the iokernel would link
    it): a ragged 1 Mi + 77 packet host batch over every visible GPU, both
    transports; it checks the last batch's verdicts against one context and the
    RCCL-gathered counts against the packets submitted, and exits 2 on a
    mismatch."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "grouppipe")
    if not os.access(exe, os.X_OK):
        pytest.fail("tools/grouppipe not built (python -c 'import __graft_entry__ as g; g.build()')")
    ndev = min(torch.cuda.device_count(), 16)
    r = subprocess.run([exe, str(ndev), str((1 << 20) + 77), "2"], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-500:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["counts_check"] == "ok" and out["verdicts_check"] == "ok" and out["n_gpus"] == ndev
    assert out["zerocopy_mpps"] > 0 and out["copy_hdr_mpps"] > 0


def test_gpu_group_table_fanout(g):
    """Table changes reach every context; the first one decides errors."""
    grp = g.Group([0, 0], R, g.HASH_JENKINS, exchange=g.XCHG_HOST)
    tables(grp)
    with pytest.raises(OSError) as e:  # IP already owned by runtime 0
        grp.runtime_set(R - 1, g.runtime_ip(0), T, T, list(range(T)))
    assert e.value.errno == 17
    grp.runtime_del(3)
    with pytest.raises(OSError) as e:
        grp.runtime_del(3)
    assert e.value.errno == 2
    # runtime 3 gone on both contexts: its packets drop as unregistered
    n = 4 * 65536
    shards, vs = [], []
    for r in range(2):
        m = g.shard_count(n, 2, r, 65536)
        fr = torch.zeros(m * 64, dtype=torch.uint8, device="cuda")
        g.generate(g.WL_UDP64, m, 64, R, fr, rank=r, world=2, shard_block=65536)
        shards.append({"frames": fr, "n": m, "stride": 64})
        vs.append(torch.zeros(m * 8, dtype=torch.uint8, device="cuda"))
    grp.classify(shards, vs)
    grp.exchange()
    c, s, per = grp.read()
    assert c[3] == 0 and (per[:, 3] == 0).all()
    assert int(s[g.RX_UNREGISTERED_MAC]) > 0 and (per[:, R + g.RX_UNREGISTERED_MAC] > 0).all()
    grp.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_torch_nccl_one_rank_exchange(g):
    """torch.distributed's RCCL path executes: a one-rank "nccl" process
    group runs shard.allgather_counts (the bench's exchange of the
    [counts | stats] vector) and global_counts sums it."""
    import torch.distributed as dist
    from caladan_amd import shard
    if dist.is_initialized():
        pytest.skip("a process group is already up")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    shard.init(0, 1, backend="nccl", device=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        local = torch.arange(R + g.NR_STATS, dtype=torch.int64, device="cuda") * 7 + 1
        gathered = torch.zeros_like(local)
        work = shard.allgather_counts(local, gathered, async_op=True)
        work.wait()
        torch.cuda.synchronize()
        assert torch.equal(gathered, local)
        assert torch.equal(shard.global_counts(gathered, 1), local)
    finally:
        dist.destroy_process_group()


def test_gpu_group_errors(g):
    """The group's error returns, as the reference's init paths fail:
    RCCL with one GPU twice (-EINVAL), a read before any exchange
    (-ENODATA), a zero-copy batch in memory that is not registered
    (-EFAULT), and the binding's shape checks."""
    with pytest.raises(OSError) as e:
        g.Group([0, 0], R, g.HASH_JENKINS, exchange=g.XCHG_RCCL)
    assert e.value.errno == 22
    grp = g.Group([0], R, g.HASH_JENKINS)
    try:
        tables(grp)
        with pytest.raises(OSError) as e:
            grp.read()
        assert e.value.errno == 61  # ENODATA
        frames = np.zeros(4096 * 64, dtype=np.uint8)  # pageable, not registered
        hv = np.zeros(4096 * 8, dtype=np.uint8)
        with pytest.raises(OSError) as e:
            grp.classify_host(frames, 4096, 64, verdicts=hv, mode=g.E2E_ZEROCOPY)
        assert e.value.errno == 14  # EFAULT
        with pytest.raises(ValueError):
            grp.classify([], [])
        # the host batch was refused before any launch: nothing was counted
        grp.exchange()
        c, s, _ = grp.read()
        assert not c.any() and not s.any()
    finally:
        grp.close()


def test_gpu_group_eight_contexts(g, orc):
    """The driver's 8-GPU shape rehearsed on the one GPU: a group of 8
    contexts (host exchange), a ragged batch generated in place per rank
    (gcl_group_classify) and one host batch split by the C splitter over the
    8 (gcl_group_classify_host): every verdict equals the oracle's at its
    global position, node counts and counters equal the oracle's, and each
    rank's RX_PULLED is gcl_shard_count for that rank."""
    from caladan_amd import shard
    W, B, stride = 8, 4096, 64
    n = 11 * B + 333  # blocks 0..10 plus a ragged block 11: ranks 0-3 take 2
    grp = g.Group([0] * W, R, g.HASH_JENKINS, block=B, exchange=g.XCHG_HOST)
    tables(grp)
    t = orc.Tables(R, 1, 0, 0x09)
    tables(t)
    frames, _, _ = orc.generate(g.WL_UDP64, n, stride, R)
    ve, ce, se = t.classify(frames, n, stride)
    # device-resident shards
    shards, vs = [], []
    for r in range(W):
        m = g.shard_count(n, W, r, B)
        fr = torch.zeros(max(m, 1) * stride, dtype=torch.uint8, device="cuda")
        g.generate(g.WL_UDP64, m, stride, R, fr, rank=r, world=W, shard_block=B)
        shards.append({"frames": fr, "n": m, "stride": stride})
        vs.append(torch.zeros(max(m, 1) * 8, dtype=torch.uint8, device="cuda"))
    grp.classify(shards, vs)
    grp.exchange()
    c, s, per = grp.read()
    for r in range(W):
        idx = shard.shard_indices(n, r, W, B)
        got = vs[r].cpu().numpy().view(g.VERDICT_DTYPE)[:len(idx)]
        assert (got == ve[idx]).all(), r
        assert int(per[r, R + g.RX_PULLED]) == g.shard_count(n, W, r, B), r
    assert (c == ce).all() and (s == se).all()
    # one host batch, split by the C splitter
    grp.reset()
    hv = pinned(np.zeros(n, dtype=g.VERDICT_DTYPE))
    grp.classify_host(pinned(frames), n, stride, verdicts=hv, mode=g.E2E_ZEROCOPY)
    grp.exchange()
    c, s, per = grp.read()
    assert (hv == ve).all(), np.nonzero(hv != ve)[0][:5]
    assert (c == ce).all() and (s == se).all()
    for r in range(W):
        assert int(per[r, R + g.RX_PULLED]) == g.shard_count(n, W, r, B), r
    assert sum(g.shard_count(n, W, r, B) for r in range(W)) == n
    grp.close()


def test_gpu_group_rccl_init_bounded(g):
    """gcl_group_open's RCCL init is non-blocking and bounded: with a 1 ms
    bound it either finishes or returns -ETIMEDOUT having aborted the
    partial communicator; a group opened afterwards with the default bound
    initialises and its all-gather runs."""
    try:
        grp = g.Group([0], R, g.HASH_JENKINS, init_timeout_ms=1)
        grp.close()
    except OSError as e:
        assert e.errno == 110, e  # ETIMEDOUT
    grp = g.Group([0], R, g.HASH_JENKINS)
    tables(grp)
    n = 4096
    fr = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    g.generate(g.WL_UDP64, n, 64, R, fr)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    grp.classify([{"frames": fr, "n": n, "stride": 64}], [v])
    grp.exchange()
    c, s, _ = grp.read()
    assert int(c.sum()) + int(s[g.RX_UNHANDLED]) == n and int(s[g.RX_PULLED]) == n
    grp.close()


def test_gpu_group_failed_exchange_is_sticky(g):
    """An exchange whose RCCL enqueue fails or times out (injected with
    gcl_group_test_fault) aborts the communicators and leaves the group
    failed: the exchange returns -ETIMEDOUT, and every later classify,
    exchange, read, table change, reset and sync returns -EIO instead of
    reusing the exchange's buffers or the aborted communicators (sync still
    drains the streams); close still works, and a new group runs normally."""
    grp = g.Group([0], R, g.HASH_JENKINS, init_timeout_ms=5000)
    tables(grp)
    n = 4096
    fr = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    g.generate(g.WL_UDP64, n, 64, R, fr)
    v = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    grp.classify([{"frames": fr, "n": n, "stride": 64}], [v])
    grp.test_fault(g.GROUP_FAULT_EXCHANGE)
    with pytest.raises(OSError) as e:
        grp.exchange()
    assert e.value.errno == 110  # ETIMEDOUT
    grp.test_fault(0)
    for call in (lambda: grp.classify([{"frames": fr, "n": n, "stride": 64}], [v]),
                 grp.exchange, grp.read,
                 lambda: grp.runtime_set(0, g.runtime_ip(0), 8, 8, g.steer_flows(8, list(range(8)))),
                 grp.reset, grp.sync):
        with pytest.raises(OSError) as e:
            call()
        assert e.value.errno == 5, call  # EIO
    grp.close()
    grp = g.Group([0], R, g.HASH_JENKINS)
    tables(grp)
    grp.classify([{"frames": fr, "n": n, "stride": 64}], [v])
    grp.exchange()
    c, s, _ = grp.read()
    assert int(s[g.RX_PULLED]) == n
    grp.close()
