"""The multi-GPU group's C ABI without a GPU (include/gcl_group.h,
caladan_amd/libgclgroup.so): every declared symbol is exported, the C
splitter's round-robin block math equals the Python shard math the bench and
the generator use (caladan_amd/shard.py), and bad arguments are refused
before any device work."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    from caladan_amd import gclassify
    gclassify.group_lib()
    return gclassify


def test_group_library_exports_every_declared_symbol(g):
    src = open(os.path.join(ROOT, "include", "gcl_group.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = sorted(set(re.findall(r"\b(gcl_\w+)\s*\(", src)))
    assert len(names) >= 14, names
    lib = ctypes.CDLL(g.GROUP_LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_group_cfg_layout(g):
    assert ctypes.sizeof(g.GclGroupCfg) == 24
    assert g.GclGroupCfg().size == 24  # GCL_GROUP_CFG_INIT's size, filled in by the binding


@pytest.mark.parametrize("block", [256, 4096, 64 << 10])
def test_c_splitter_matches_shard_math(g, block):
    """gcl_shard_count / gcl_shard_global against shard.shard_indices /
    shard.global_index: every packet owned by exactly one rank, in order,
    ragged last blocks included."""
    from caladan_amd import shard
    rng = np.random.default_rng(5)
    sizes = [0, 1, block - 1, block, block + 1, 3 * block, 7 * block + 5,
             int(rng.integers(1, 40 * block))]
    for n in sizes:
        for world in (1, 2, 3, 4, 8):
            seen = np.zeros(n, dtype=np.int64)
            for rank in range(world):
                idx = shard.shard_indices(n, rank, world, block)
                c = g.shard_count(n, world, rank, block)
                assert c == len(idx), (n, world, rank)
                js = np.unique(np.concatenate([np.arange(min(c, 3)), np.arange(max(0, c - 3), c),
                                               rng.integers(0, max(c, 1), size=min(c, 50))]))
                for j in js[js < c]:
                    gj = g.shard_global(int(j), world, rank, block)
                    assert gj == shard.global_index(int(j), rank, world, block) == idx[j]
                seen[idx] += 1
            assert (seen == 1).all()


def test_shard_global_matches_generator_rule(g):
    """The generator's sharding rule (include/gclassify.h, gcl_gen_params):
    local j -> ((j / B) * W + rank) * B + j % B."""
    B = 64 << 10
    for j in (0, 1, B - 1, B, 5 * B + 17):
        for W, r in ((2, 1), (8, 7), (4, 0)):
            assert g.shard_global(j, W, r, B) == ((j // B) * W + r) * B + j % B
    assert g.shard_count(10, 4, 4, B) == 0  # a rank past the world holds nothing
    assert g.shard_count(10, 1, 0, B) == 10


def test_group_open_refuses_bad_args(g):
    gl = g.group_lib()
    cfg = g.GclCfg(max_runtimes=16, hash_mode=1)
    out = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    for op in (gl.gcl_group_open_v2, gl.gcl_group_open):
        assert op(0, devs, ctypes.byref(cfg), None, ctypes.byref(out)) == -22
        assert op(17, devs, ctypes.byref(cfg), None, ctypes.byref(out)) == -22
    bad_block = g.GclGroupCfg(block=1000, exchange=0, nstreams=2)
    assert gl.gcl_group_open_v2(1, devs, ctypes.byref(cfg), ctypes.byref(bad_block), ctypes.byref(out)) == -22
    bad_x = g.GclGroupCfg(block=0, exchange=2, nstreams=2)
    assert gl.gcl_group_open_v2(1, devs, ctypes.byref(cfg), ctypes.byref(bad_x), ctypes.byref(out)) == -22
    bad_s = g.GclGroupCfg(block=0, exchange=0, nstreams=5)
    assert gl.gcl_group_open_v2(1, devs, ctypes.byref(cfg), ctypes.byref(bad_s), ctypes.byref(out)) == -22
    # a struct of another layout (no size, or an ABI-1 caller's) is refused
    # by the v2 entry point before anything else is read
    bad_size = g.GclGroupCfg(block=0, exchange=0, nstreams=2, size=16)
    assert gl.gcl_group_open_v2(1, devs, ctypes.byref(cfg), ctypes.byref(bad_size), ctypes.byref(out)) == -22
    for f in ("gcl_group_exchange", "gcl_group_sync", "gcl_group_reset"):
        assert getattr(gl, f)(None) == -22
    assert gl.gcl_group_read(None, None, None, None) == -22
    assert gl.gcl_group_size(None) == -22
    assert gl.gcl_group_ctx(None, 0) is None


def test_group_abi1_entry_point_reads_16_bytes(g):
    """The exported ABI-1 symbol gcl_group_open takes the 16-B struct of
    rounds 1-3 (block, exchange, nstreams) and validates it like the v2
    entry point: a bad block or exchange in it is refused."""
    gl = g.group_lib()
    cfg = g.GclCfg(max_runtimes=16, hash_mode=1)
    out = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)

    class V1(ctypes.Structure):
        _fields_ = [("block", ctypes.c_uint64), ("exchange", ctypes.c_uint32),
                    ("nstreams", ctypes.c_uint32)]
    assert ctypes.sizeof(V1) == 16
    assert gl.gcl_group_open(1, devs, ctypes.byref(cfg), ctypes.byref(V1(1000, 0, 2)), ctypes.byref(out)) == -22
    assert gl.gcl_group_open(1, devs, ctypes.byref(cfg), ctypes.byref(V1(0, 2, 2)), ctypes.byref(out)) == -22


def test_group_open_without_gpu_is_enodev(g):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(OSError) as e:
        g.Group([0], 16)
    assert e.value.errno in (19, 22)
