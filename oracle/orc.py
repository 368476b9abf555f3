"""ctypes binding of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liborc.so")
LIB_NATIVE = os.path.join(HERE, "build", "liborc_native.so")
REF_JHASH = os.path.join(HERE, "_ref", "libjhash_ref.so")
REF_CRC = os.path.join(HERE, "_ref", "libcrc_ref.so")
REF_HOST = os.path.join(HERE, "_ref", "libhost_ref.so")
REF_CORE = os.path.join(HERE, "_ref", "libcore_ref.so")
REF_TRANS = os.path.join(HERE, "_ref", "libtrans_ref.so")
TRANS_DTYPE = np.dtype([("h5", "<u4"), ("h3", "<u4")])

NR_STATS = 8


class _Cfg(ctypes.Structure):
    pass


class Batch(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_void_p), ("frames_len", ctypes.c_uint64),
                ("stride", ctypes.c_uint64), ("offs", ctypes.c_void_p),
                ("olflags", ctypes.c_void_p), ("rss", ctypes.c_void_p),
                ("fdir_hi", ctypes.c_void_p), ("pkt_len", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("dst_hint", ctypes.c_void_p)]


class GenParams(ctypes.Structure):
    _fields_ = [("workload", ctypes.c_uint32), ("nruntimes", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("n", ctypes.c_uint64), ("stride", ctypes.c_uint64),
                ("rank", ctypes.c_uint32), ("world", ctypes.c_uint32),
                ("shard_block", ctypes.c_uint64), ("zipf_cdf", ctypes.c_void_p),
                ("nflows", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("pkt_len", ctypes.c_void_p)]


VERDICT_DTYPE = np.dtype([("hash", "<u4"), ("uniqid", "<u2"), ("thread", "u1"), ("action", "u1")])


def build(native=False):
    target = "native" if native else "all"
    subprocess.check_call(["make", "-s", "-C", HERE, target])


def _bind(path):
    lib = ctypes.CDLL(path)
    vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "orc_jhash": (u32, [ctypes.c_char_p, ctypes.c_size_t]),
        "orc_do_toeplitz": (u32, [ctypes.c_char_p, u32, u32, u16, u16]),
        "orc_toeplitz_bytes": (u32, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]),
        "orc_steer_flows": (None, [u16, ctypes.POINTER(u16), u16, ctypes.POINTER(u16)]),
        "orc_tables_new": (vp, [u32, u32, u32, ctypes.c_uint8, ctypes.c_char_p]),
        "orc_tables_free": (None, [vp]),
        "orc_runtime_set": (i32, [vp, u16, u32, u16, u16, ctypes.POINTER(u16)]),
        "orc_runtime_del": (i32, [vp, u16]),
        "orc_classify": (None, [vp, ctypes.POINTER(Batch), vp, vp, vp]),
        "orc_classify_lrpc": (None, [vp, ctypes.POINTER(Batch), vp, vp, vp]),
        "orc_classify_ex": (None, [vp, ctypes.POINTER(Batch), vp, vp, vp, vp]),
        "orc_crc32c_u64": (u32, [u32, u64]),
        "orc_runtime_set_trans_seed": (i32, [vp, u16, u32]),
        "orc_bench": (ctypes.c_double, [vp, ctypes.POINTER(Batch), i32, i32, i32]),
        "orc_bench_ex": (ctypes.c_double, [vp, ctypes.POINTER(Batch), i32, i32, u32]),
        "orc_bench_pinned": (ctypes.c_double, [vp, ctypes.POINTER(Batch), i32, i32, u32, vp]),
        "orc_classify_direct": (None, [vp, ctypes.POINTER(Batch), vp, vp, vp]),
        "orc_generate": (i32, [ctypes.POINTER(GenParams), vp, vp, vp, vp]),
        "orc_runtime_ip": (u32, [u32]),
        "orc_zipf_cdf": (i32, [u32, ctypes.c_double, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_libs = {}


def lib(native=False):
    path = LIB_NATIVE if native else LIB
    if path not in _libs:
        if not os.path.exists(path):
            build(native)
        _libs[path] = _bind(path)
    return _libs[path]


def ref_jhash():
    """The reference's own base/jenkins_hash.c (oracle/_ref), or None."""
    if not os.path.exists(REF_JHASH):
        return None
    l = ctypes.CDLL(REF_JHASH)
    l.jenkins_hash.restype = ctypes.c_uint32
    l.jenkins_hash.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return l


def ref_crc():
    """The reference's hash_crc32c_one/two (oracle/_ref/libcrc_ref.so), or None."""
    if not os.path.exists(REF_CRC):
        return None
    l = ctypes.CDLL(REF_CRC)
    l.ref_crc32c_one.restype = ctypes.c_uint32
    l.ref_crc32c_one.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    l.ref_crc32c_two.restype = ctypes.c_uint32
    l.ref_crc32c_two.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
    return l


def ref_toeplitz():
    """The reference's own do_toeplitz (runtime/net/core.c:120-139, compiled in
    place into oracle/_ref/libcore_ref.so by oracle/ref_core.c), as
    f(key, saddr, daddr, sport, dport), or None."""
    if not os.path.exists(REF_CORE):
        return None
    l = ctypes.CDLL(REF_CORE)
    f = l.ref_do_toeplitz
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint16, ctypes.c_uint16]
    return lambda key, s, d, sp, dp: f(bytes(key), len(key), s, d, sp, dp)


def ref_ip_hdr_supported():
    """The reference's own ip_hdr_supported (runtime/net/core.c:203-209,
    oracle/_ref/libcore_ref.so) as f(20-byte wire header) -> bool, or None."""
    if not os.path.exists(REF_CORE):
        return None
    f = ctypes.CDLL(REF_CORE).ref_ip_hdr_supported
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p]
    return lambda hdr: bool(f(bytes(hdr)))


def ref_trans():
    """The reference's own trans_hash_5tuple/3tuple (runtime/net/transport.c:29-42,
    compiled in place into oracle/_ref/libtrans_ref.so by oracle/ref_trans.c),
    as f(seed, proto, lip, lport, rip, rport) -> (h5, h3), or None."""
    if not os.path.exists(REF_TRANS):
        return None
    l = ctypes.CDLL(REF_TRANS)
    f = l.ref_trans_hash
    f.restype = None
    u32 = ctypes.c_uint32
    f.argtypes = [u32, ctypes.c_uint8, u32, ctypes.c_uint16, u32, ctypes.c_uint16,
                  ctypes.POINTER(u32 * 2)]

    def call(seed, proto, lip, lport, rip, rport):
        out = (u32 * 2)()
        f(seed, proto, lip, lport, rip, rport, ctypes.byref(out))
        return out[0], out[1]
    return call


def ref_host():
    """The reference's base/lrpc.c and header-only rx host helpers
    (oracle/_ref/libhost_ref.so, exported by oracle/ref_host.c), or None."""
    if not os.path.exists(REF_HOST):
        return None
    l = ctypes.CDLL(REF_HOST)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    for name, res, args in [
            ("ref_lrpc_send", ctypes.c_bool, [vp, u64, ctypes.c_ulong]),
            ("ref_lrpc_recv", ctypes.c_bool, [vp, vp, vp]),
            ("lrpc_init_out", ctypes.c_int, [vp, vp, ctypes.c_uint, vp]),
            ("lrpc_init_in", ctypes.c_int, [vp, vp, ctypes.c_uint, vp]),
            ("ref_lrpc_layout", None, [vp]),
            ("ref_rxq_cmd", u64, [ctypes.c_uint16, ctypes.c_int]),
            ("ref_rss_from_txpkt_payload", u64, [u64]),
            ("ref_txpkt_to_payload", u64, [u64, ctypes.c_uint16]),
            ("ref_txflag_local_hint", u32, []),
            ("ref_ncpu", u32, []),
            ("ref_build_frame", ctypes.c_int, [vp, ctypes.c_int, u32, u32, ctypes.c_uint16,
                                               ctypes.c_uint16, ctypes.c_uint8, ctypes.c_uint16,
                                               ctypes.c_uint16]),
            ("ref_net_consts", None, [vp])]:
        f = getattr(l, name)
        f.restype, f.argtypes = res, args
    return l


def crc32c_u64(crc, val):
    return lib().orc_crc32c_u64(crc, val)


def jhash(key: bytes) -> int:
    return lib().orc_jhash(key, len(key))


def do_toeplitz(key, saddr, daddr, sport, dport):
    return lib().orc_do_toeplitz(bytes(key), saddr, daddr, sport, dport)


def toeplitz_bytes(key, data):
    return lib().orc_toeplitz_bytes(bytes(key), len(key), bytes(data), len(data))


def steer_flows(thread_count, active_idx):
    n = len(active_idx)
    act = (ctypes.c_uint16 * max(n, 1))(*active_idx)
    out = (ctypes.c_uint16 * thread_count)(*([0xEEEE] * thread_count))
    lib().orc_steer_flows(thread_count, act, n, out)
    return list(out)


def runtime_ip(r):
    return lib().orc_runtime_ip(r)


def zipf_cdf(nflows, s=0.99):
    cdf = np.empty(nflows, dtype=np.uint64)
    assert lib().orc_zipf_cdf(nflows, s, cdf.ctypes.data) == 0
    return cdf


def _p(a):
    return None if a is None else a.ctypes.data


class Tables:
    """The oracle's dp state: clients_by_id + ip_to_proc + flow tables."""

    def __init__(self, max_runtimes=16, hash_mode=1, flags=0, default_olflags=0x09,
                 rss_key=b"\0" * 40, native=False):
        self._lib = lib(native)
        self.max_runtimes = max_runtimes
        self.h = self._lib.orc_tables_new(max_runtimes, hash_mode, flags, default_olflags,
                                          bytes(rss_key)[:40].ljust(40, b"\0"))
        if not self.h:
            raise ValueError("orc_tables_new failed")

    def __del__(self):
        if getattr(self, "h", None):
            self._lib.orc_tables_free(self.h)
            self.h = None

    def runtime_set(self, uniqid, ip, thread_count, active, flow_tbl=None):
        tbl = None
        if flow_tbl is not None:
            tbl = (ctypes.c_uint16 * max(len(flow_tbl), 1))(*flow_tbl)
        return self._lib.orc_runtime_set(self.h, uniqid, ip, thread_count, active, tbl)

    def runtime_del(self, uniqid):
        return self._lib.orc_runtime_del(self.h, uniqid)

    def set_trans_seed(self, uniqid, seed):
        return self._lib.orc_runtime_set_trans_seed(self.h, uniqid, seed)

    def _batch(self, frames, n, stride, offs, olflags, rss, fdir_hi, pkt_len, frames_len,
               dst_hint=None):
        self._keep = [frames, offs, olflags, rss, fdir_hi, pkt_len, dst_hint]
        return Batch(frames=frames.ctypes.data, frames_len=frames.nbytes if frames_len is None else frames_len,
                     stride=stride, offs=_p(offs), olflags=_p(olflags), rss=_p(rss),
                     fdir_hi=_p(fdir_hi), pkt_len=_p(pkt_len), n=n, dst_hint=_p(dst_hint))

    def classify(self, frames, n, stride=0, offs=None, olflags=None, rss=None, fdir_hi=None,
                 pkt_len=None, frames_len=None, lrpc=False, dst_hint=None, trans=False):
        """Returns (verdicts structured array, counts u64[R], stats u64[8])
        [+ trans (h5, h3) array when trans=True]."""
        b = self._batch(frames, n, stride, offs, olflags, rss, fdir_hi, pkt_len, frames_len,
                        dst_hint)
        v = np.zeros(n, dtype=VERDICT_DTYPE)
        counts = np.zeros(self.max_runtimes, dtype=np.uint64)
        stats = np.zeros(NR_STATS, dtype=np.uint64)
        if trans:
            tr = np.zeros(n, dtype=TRANS_DTYPE)
            self._lib.orc_classify_ex(self.h, ctypes.byref(b), v.ctypes.data, counts.ctypes.data,
                                      stats.ctypes.data, tr.ctypes.data)
            return v, counts, stats, tr
        fn = self._lib.orc_classify_lrpc if lrpc else self._lib.orc_classify
        fn(self.h, ctypes.byref(b), v.ctypes.data, counts.ctypes.data, stats.ctypes.data)
        return v, counts, stats

    def classify_direct(self, frames, n, stride=0, offs=None, olflags=None, rss=None,
                        fdir_hi=None):
        """The CPU-baseline form (rx.c's direct header loads): every frame's
        first 54 bytes must lie inside `frames`."""
        last = (int(offs.max()) if offs is not None and n else (n - 1) * stride) + 54
        if n and last > frames.nbytes:
            raise ValueError("classify_direct: a frame's header runs past the buffer")
        b = self._batch(frames, n, stride, offs, olflags, rss, fdir_hi, None, None)
        v = np.zeros(n, dtype=VERDICT_DTYPE)
        counts = np.zeros(self.max_runtimes, dtype=np.uint64)
        stats = np.zeros(NR_STATS, dtype=np.uint64)
        self._lib.orc_classify_direct(self.h, ctypes.byref(b), v.ctypes.data, counts.ctypes.data,
                                      stats.ctypes.data)
        return v, counts, stats

    def bench(self, frames, n, stride, threads=1, passes=1, lrpc=False, offs=None, olflags=None,
              rss=None, fdir_hi=None, pkt_len=None, direct=False, cpus=None, nosend=False):
        """Wall seconds of `passes` classifications on `threads` threads
        (contiguous shards); direct=True times rx.c's direct-load form;
        `cpus`: thread i pinned to CPU cpus[i]."""
        if direct and n and (n - 1) * stride + 54 > frames.nbytes and offs is None:
            raise ValueError("direct bench: a frame's header runs past the buffer")
        b = self._batch(frames, n, stride, offs, olflags, rss, fdir_hi, pkt_len, None)
        flags = (1 if lrpc else 0) | (2 if direct else 0) | (4 if nosend else 0)
        if cpus is None:
            return self._lib.orc_bench_ex(self.h, ctypes.byref(b), threads, passes, flags)
        c = np.full(max(threads, 1), -1, dtype=np.int32)
        c[:min(len(cpus), len(c))] = cpus[:len(c)]
        return self._lib.orc_bench_pinned(self.h, ctypes.byref(b), threads, passes, flags, c.ctypes.data)


def generate(workload, n, stride, nruntimes, seed=0xCA1ADA4, rank=0, world=1, shard_block=0,
             cdf=None, native=False, pkt_len=None):
    """CPU copy of the synthetic streams: returns (frames, olflags, rss); fills
    the optional uint16 `pkt_len` array in place."""
    frames = np.zeros(n * stride, dtype=np.uint8)
    olflags = np.zeros(n, dtype=np.uint8)
    rss = np.zeros(n, dtype=np.uint32)
    p = GenParams(workload=workload, nruntimes=nruntimes, seed=seed, n=n, stride=stride,
                  rank=rank, world=world, shard_block=shard_block,
                  zipf_cdf=None, nflows=0 if cdf is None else len(cdf), pkt_len=_p(pkt_len))
    ret = lib(native).orc_generate(ctypes.byref(p), _p(cdf), frames.ctypes.data,
                                   olflags.ctypes.data, rss.ctypes.data)
    if ret:
        raise ValueError(f"orc_generate: {ret}")
    return frames, olflags, rss
