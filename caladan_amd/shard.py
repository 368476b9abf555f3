"""Multi-GPU sharding of the rx batch.

Packets are independent, so a batch is split round-robin in blocks of
`block` packets: block b goes to rank b mod W (contiguous, coalesced slabs per
GPU; the generator reproduces this mapping with gcl_gen_params.shard_block).
Tables are replicated.  The only cross-rank output is the per-runtime packet
count vector (plus the rx counters), exchanged with one all_gather -- RCCL over
xGMI on GPUs (backend "nccl"), gloo on CPU for tests.
"""
import os

import torch
import torch.distributed as dist


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init(rank, world, backend="nccl", device=None):
    """Join the process group.  With nccl (RCCL) the rank's GPU is bound at
    init (`device`), so barriers and collectives use it, never a guess."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    kw = {"device_id": device} if backend == "nccl" and device is not None else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)


def finish():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def global_index(j, rank, world, block):
    """Global packet index of this rank's local packet j (gcl_generate)."""
    if world <= 1 or block == 0:
        return j
    return ((j // block) * world + rank) * block + j % block


def shard_indices(n_global, rank, world, block):
    """Global indices owned by `rank` for a batch of n_global packets."""
    import numpy as np
    nb = (n_global + block - 1) // block
    idx = [np.arange(b * block, min((b + 1) * block, n_global)) for b in range(rank, nb, world)]
    return np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)


def allgather_counts(local, gathered, async_op=False):
    """all_gather of this rank's [counts | stats] vector into gathered[W * len].

    On GPUs this is one RCCL all_gather (ProcessGroupNCCL) over xGMI; gloo
    (CPU tests, single-GPU rehearsal) goes through host tensors."""
    if dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(gathered, local, async_op=async_op)
    parts = [torch.empty_like(local, device="cpu") for _ in range(dist.get_world_size())]
    dist.all_gather(parts, local.cpu())
    gathered.copy_(torch.cat(parts).to(gathered.device))
    return None


def global_counts(gathered, world):
    """Sum the gathered per-rank vectors: the node-wide per-runtime counts."""
    return gathered.view(world, -1).sum(dim=0)
