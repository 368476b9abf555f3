"""Multi-rank path on CPU (gloo, world_size 2): round-robin block sharding of
the packet stream plus the all_gather of per-runtime counts reproduces the
single-process classification of the whole batch."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

R, T, N_LOCAL, BLOCK, SEED = 16, 8, 24 * 1024, 4096, 0xCA1ADA4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tables(orc):
    t = orc.Tables(R, 1, 0, 0x09)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), T, r % T + 1, orc.steer_flows(T, list(range(r % T + 1))))
    return t


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from caladan_amd import shard
    from oracle import orc
    shard.init(rank, world, backend="gloo")
    try:
        frames, _, _ = orc.generate(0, N_LOCAL, 64, R, seed=SEED, rank=rank, world=world,
                                    shard_block=BLOCK)
        _, counts, stats = _tables(orc).classify(frames, N_LOCAL, 64)
        local = torch.from_numpy(np.concatenate([counts, stats]).astype(np.int64))
        gathered = torch.zeros(world * local.numel(), dtype=torch.int64)
        shard.allgather_counts(local, gathered)
        q.put((rank, shard.global_counts(gathered, world).numpy().tolist(),
               gathered.view(world, -1)[rank].numpy().tolist() == local.numpy().tolist()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_sharded_counts_equal_single_process(orc):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames, _, _ = orc.generate(0, N_LOCAL * world, 64, R, seed=SEED)
    _, counts, stats = _tables(orc).classify(frames, N_LOCAL * world, 64)
    want = np.concatenate([counts, stats]).astype(np.int64).tolist()
    for rank, got, own_ok in res:
        assert own_ok
        assert got == want


def test_shard_indices_match_generator_mapping(orc):
    from caladan_amd import shard
    n_global, world, block = 10 * 1000 + 123, 3, 1000
    seen = []
    for r in range(world):
        idx = shard.shard_indices(n_global, r, world, block)
        j = np.arange(len(idx))
        assert (np.array([shard.global_index(int(x), r, world, block) for x in j]) == idx).all()
        seen.append(idx)
    allidx = np.sort(np.concatenate(seen))
    assert (allidx == np.arange(n_global)).all()
    # the oracle generator's rank-r shard is exactly those global packets
    full, _, _ = orc.generate(0, 4 * 1024, 64, R, seed=SEED)
    part, _, _ = orc.generate(0, 2 * 1024, 64, R, seed=SEED, rank=1, world=2, shard_block=512)
    idx = shard.shard_indices(4 * 1024, 1, 2, 512)
    assert (part.reshape(-1, 64) == full.reshape(-1, 64)[idx]).all()
