"""The multi-GPU step on real hardware, rehearsed with 2 gloo ranks sharing
the one GPU of the test box (the 8-GPU RCCL run is the
driver's).

* bench.Exchange -- classify into a [counts | stats] vector, all_gather it on
  a side stream every `period` steps, accumulate node-wide totals -- over
  three full exchange periods and a partial one flushed by drain(): the
  accumulated vector equals the single-process classification of the whole
  packet stream, times the steps, exactly.
* bench.e2e_multi -- config 5's per-rank shard of the mixed 9000-B trace
  classified from pinned host memory: each rank's verdicts equal the oracle
  on that rank's round-robin shard, and RX_PULLED summed over the ranks is
  world x n x calls.

The unit being sharded is the rx_burst batch (iokernel/rx.c:270-290)."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["GCL_BENCH_PLACEMENT"] = "0"  # two ranks on one GPU: no placement probe
    sys.path.insert(0, ROOT)
    import torch as t
    t.cuda.set_device(0)
    import bench
    from caladan_amd import shard
    shard.init(rank, WORLD, backend="gloo")
    return bench, shard


def _exchange_worker(rank, port, q, n, steps, period):
    bench, shard = _setup(rank, port)
    try:
        device = torch.device("cuda", 0)
        w = bench.Workload("udp64", rank, WORLD, device, vbytes=4, n=n)
        ex = bench.Exchange(w, WORLD, device, period)
        for _ in range(steps):
            ex.step(w)
        ex.drain()
        torch.cuda.synchronize()
        q.put((rank, ex.acc.cpu().numpy().tolist(), ex.k, None))
    except Exception as e:  # report, do not hang the peer
        q.put((rank, None, None, repr(e)))
    finally:
        shard.finish()


def _e2e_worker(rank, port, q, n):
    bench, shard = _setup(rank, port)
    try:
        keep = {}
        res = bench.e2e_multi(torch.device("cuda", 0), rank, WORLD, 4, reps=2, n=n, keep=keep)
        q.put((rank, res, keep, None))
    except Exception as e:
        q.put((rank, None, None, repr(e)))
    finally:
        shard.finish()


def _spawn(target, *args):
    if torch.cuda.device_count() < 1:  # counts devices without initialising HIP here
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, port, q, *args)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(WORLD):
            r = q.get(timeout=100)
            out[r[0]] = r[1:]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        assert v[-1] is None, f"rank {r}: {v[-1]}"
    return out


def _oracle_tables(orc, bench, R, T):
    t = orc.Tables(R, 1, 0, 0x09)
    bench.setup_tables(t, R, T)
    return t


def test_gpu_exchange_two_ranks_match_single_process(orc):
    sys.path.insert(0, ROOT)
    import bench
    n, steps, period = 2 * bench.SHARD_BLOCK, 7, 3  # periods 3 + 3 + a partial 1
    out = _spawn(_exchange_worker, n, steps, period)
    _, _, _, R, T, _ = bench.WORKLOADS["udp64"]
    frames, _, _ = orc.generate(0, WORLD * n, 64, R, seed=bench.SEED)
    _, counts, stats = _oracle_tables(orc, bench, R, T).classify(frames, WORLD * n, 64)
    want = (np.concatenate([counts, stats]).astype(np.int64) * steps).tolist()
    for r in range(WORLD):
        acc, k, _ = out[r]
        assert k == 3, f"rank {r}: {k} exchanges"
        assert acc == want, f"rank {r}: node-wide counts differ from the single-process run"


def test_gpu_e2e_multi_shards_match_oracle(orc):
    sys.path.insert(0, ROOT)
    import bench
    n = 2 * bench.SHARD_BLOCK
    out = _spawn(_e2e_worker, n)
    wl, _, stride, R, T, _ = bench.WORKLOADS["mixed"]
    pulled = 0
    for r in range(WORLD):
        res, keep, _ = out[r]
        assert res["rx_pulled_check"] == "ok", res
        frames, _, _ = orc.generate(wl, n, stride, R, seed=bench.SEED, rank=r, world=WORLD,
                                    shard_block=bench.SHARD_BLOCK)
        v, _, _ = _oracle_tables(orc, bench, R, T).classify(frames, n, stride)
        from caladan_amd.gclassify import VERDICT4_DTYPE
        from tests.rxcases import to_verdict4
        got = keep["verdicts"].view(np.uint8).view(VERDICT4_DTYPE)
        assert (got == to_verdict4(v, [T] * R)).all(), f"rank {r}: shard verdicts differ from the oracle"
        pulled += int(keep["stats"][6])  # GCL_RX_PULLED
        assert keep["calls"] * n == int(keep["stats"][6])
    assert pulled == WORLD * n * out[0][1]["calls"]
