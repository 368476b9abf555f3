"""Python binding of libgclassify.so (ctypes), for tests and bench.py.

The product boundary is the C ABI in include/gclassify.h; the dataplane side
that consumes verdicts is C (include/gcl_host.h).  This module is a thin
mirror of that ABI with the reference's names and error behaviour: every call
that returns -errno raises OSError(errno) here, the way the reference's init
paths fail (rx_init, dp_clients_init return -1/-errno).

There is no CPU fallback: if the shared library is missing, importing the
binding raises, and classify() needs device (HBM) buffers.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgclassify.so")

GCL_MAX_PROC = 4096
GCL_NCPU = 256
GCL_RX_BURST_SIZE = 64

HASH_NIC, HASH_JENKINS, HASH_TOEPLITZ = 0, 1, 2
HASH_MODES = {"nic": HASH_NIC, "jenkins": HASH_JENKINS, "toeplitz": HASH_TOEPLITZ}

CFG_AZURE_ARP, CFG_HASH16, CFG_PROFILE, CFG_TRANS_HASH, CFG_VERDICT4 = 0x1, 0x2, 0x4, 0x8, 0x10
CFG_VERDICT2, CFG_VERDICT1 = 0x20, 0x40
# GCL_CFG_VERDICT2: u16 q = uniqid << thread_bits | flow_tbl slot; kind in the top two bits
V2_Q_MASK, V2_KIND, V2_DELIVER, V2_WAKE, V2_OTHER, V2_QUEUES = 0x3FFF, 0xC000, 0, 0x4000, 0xC000, 0x4000
# GCL_CFG_VERDICT1: u8 q (DELIVER or WAKE, unmarked) or V1_OTHER | action
V1_Q_MASK, V1_OTHER, V1_QUEUES = 0x7F, 0x80, 0x80
PAIR_NEW_READS, PAIR_NEW_WRITES, PAIR_TRIES, PAIR_RUN = 0x1, 0x2, 24, 2
PAIR_QUIET, PAIR_VERBOSE = 0x10000, 0x20000
PROBE_MIN = 0x100  # gcl_access_probe: the layout's minimal-request probe

F_RSS_HASH, F_FDIR_ID = 0x01, 0x02
F_IP_CKSUM_MASK, F_IP_CKSUM_UNKNOWN, F_IP_CKSUM_BAD = 0x0C, 0x00, 0x04
F_IP_CKSUM_GOOD, F_IP_CKSUM_NONE = 0x08, 0x0C

ACT_DELIVER, ACT_WAKE, ACT_DROP_ETHERTYPE, ACT_DROP_UNREG = 0, 1, 2, 3
ACT_BROADCAST, ACT_ARP_RESPOND = 4, 5
ACT_MASK, ACT_F_FDIR, ACT_F_TRANS = 0x3F, 0x80, 0x40
NO_RUNTIME, NO_THREAD = 0xFFFF, 0xFF

(RX_UNREGISTERED_MAC, RX_UNICAST_FAIL, RX_BROADCAST_FAIL, RX_FLOW_TAG_MATCH,
 RX_UNHANDLED, RX_HASH_MISSING, RX_PULLED) = range(7)
NR_STATS = 8
STAT_NAMES = ["RX_UNREGISTERED_MAC", "RX_UNICAST_FAIL", "RX_BROADCAST_FAIL",
              "RX_FLOW_TAG_MATCH", "RX_UNHANDLED", "RX_HASH_MISSING", "RX_PULLED"]

WL_UDP64, WL_TCP1500_ZIPF, WL_MIXED = 0, 1, 2

# Fixed 40-B Toeplitz key of the reference (iokernel/directpath/core.c:35-39)
CALADAN_RSS_KEY = bytes([
    0x82, 0x19, 0xFA, 0x80, 0xA4, 0x31, 0x06, 0x59, 0x3E, 0x3F, 0x9A,
    0xAC, 0x3D, 0xAE, 0xD6, 0xD9, 0xF5, 0xFC, 0x0C, 0x63, 0x94, 0xBF,
    0x8F, 0xDE, 0xD2, 0xC5, 0xE2, 0x04, 0xB1, 0xCF, 0xB1, 0xB1, 0xA1,
    0x0D, 0x6D, 0x86, 0xBA, 0x61, 0x78, 0xEB])

VERDICT_DTYPE = np.dtype([("hash", "<u4"), ("uniqid", "<u2"), ("thread", "u1"), ("action", "u1")])
# every DELIVER / WAKE verdict carries the flow_tbl slot (hash % thread_count) in `thread`:
# the host post-pass reads flow_tbl[slot] at delivery time (rx.c:55-72)
VERDICT4_DTYPE = np.dtype([("uniqid", "<u2"), ("thread", "u1"), ("action", "u1")])
TRANS_DTYPE = np.dtype([("h5", "<u4"), ("h3", "<u4")])
# struct gcl_loop_rec: one persistent-loop verdict record (gcl_rxloop_peek)
LOOP_REC_DTYPE = np.dtype([("hash", "<u4"), ("verdict", "<u4"), ("ticket", "<u8")])


class GclCfg(ctypes.Structure):
    _fields_ = [("max_runtimes", ctypes.c_uint32), ("hash_mode", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("default_olflags", ctypes.c_uint8),
                ("rss_key", ctypes.c_uint8 * 40), ("thread_bits", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 2)]


class GclBatch(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_void_p), ("frames_len", ctypes.c_uint64),
                ("stride", ctypes.c_uint64), ("offs", ctypes.c_void_p),
                ("olflags", ctypes.c_void_p), ("rss", ctypes.c_void_p),
                ("fdir_hi", ctypes.c_void_p), ("pkt_len", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("dst_hint", ctypes.c_void_p)]


class GclGenParams(ctypes.Structure):
    _fields_ = [("workload", ctypes.c_uint32), ("nruntimes", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("n", ctypes.c_uint64), ("stride", ctypes.c_uint64),
                ("rank", ctypes.c_uint32), ("world", ctypes.c_uint32),
                ("shard_block", ctypes.c_uint64), ("zipf_cdf", ctypes.c_void_p),
                ("nflows", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("pkt_len", ctypes.c_void_p)]


class GclOut(ctypes.Structure):
    _fields_ = [("verdicts", ctypes.c_void_p), ("runtime_counts", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("trans", ctypes.c_void_p)]


class GclTrans(ctypes.Structure):
    _fields_ = [("h5", ctypes.c_uint32), ("h3", ctypes.c_uint32)]


class GclTrace(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_void_p), ("frames_len", ctypes.c_uint64),
                ("alloc_len", ctypes.c_uint64), ("offs", ctypes.c_void_p),
                ("pkt_len", ctypes.c_void_p), ("orig_len", ctypes.c_void_p),
                ("ts_ns", ctypes.c_void_p), ("n", ctypes.c_uint64), ("skipped", ctypes.c_uint64)]


class GclE2eOpts(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_uint32), ("nstreams", ctypes.c_uint32), ("chunk", ctypes.c_uint64)]


E2E_COPY, E2E_ZEROCOPY = 0, 1


class GclPairInfo(ctypes.Structure):
    _fields_ = [("chosen_us", ctypes.c_double), ("worst_us", ctypes.c_double),
                ("candidates", ctypes.c_uint32), ("classes", ctypes.c_uint32),
                ("spacer_bytes", ctypes.c_uint64), ("probe_write_bytes", ctypes.c_uint64)]


class GclRxloopCfg(ctypes.Structure):
    _fields_ = [("slots", ctypes.c_uint32), ("max_burst", ctypes.c_uint32),
                ("workers", ctypes.c_uint32), ("lifetime_ms", ctypes.c_uint32),
                ("region", ctypes.c_void_p), ("region_len", ctypes.c_uint64),
                ("counts", ctypes.c_void_p), ("stats", ctypes.c_void_p),
                ("flags", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


LOOP_INLINE_HDRS = 0x1
LOOP_HDR_RECORDS = 0x2
LOOP_STAMPS = 0x4


class GclTune(ctypes.Structure):
    """struct gcl_tune: test / A-B overrides of the library's defaults
    (GCL_TUNE_AUTO = -1 everywhere: the library's own choice)."""
    _fields_ = [("size", ctypes.c_uint32), ("tables", ctypes.c_int32), ("depth", ctypes.c_int32),
                ("threads", ctypes.c_int32), ("grid", ctypes.c_int32), ("blocks_per_cu", ctypes.c_int32),
                ("defer", ctypes.c_int32), ("pair_lean", ctypes.c_int32),
                ("tile_lean", ctypes.c_int32), ("loop64", ctypes.c_int32),
                ("loop_lean", ctypes.c_int32), ("loop_spec", ctypes.c_int32),
                ("loop_phase_max", ctypes.c_int32), ("loop_phase_up", ctypes.c_int32),
                ("loop_phase_down", ctypes.c_int32), ("loop_prefetch", ctypes.c_int32),
                ("debug", ctypes.c_uint32), ("rec_prefetch", ctypes.c_int32),
                ("slot_prefetch", ctypes.c_int32), ("vstage", ctypes.c_int32), ("pair_i32", ctypes.c_int32),
                ("tile_order", ctypes.c_int32), ("loop_t0", ctypes.c_uint64)]


TUNE_AUTO = -1


class GclVerdict(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint32), ("uniqid", ctypes.c_uint16),
                ("thread", ctypes.c_uint8), ("action", ctypes.c_uint8)]


assert ctypes.sizeof(GclVerdict) == 8 and VERDICT_DTYPE.itemsize == 8


class GclLrpcMsg(ctypes.Structure):
    _fields_ = [("cmd", ctypes.c_uint64), ("payload", ctypes.c_ulong)]


class GclLrpcChanOut(ctypes.Structure):
    _fields_ = [("send_head", ctypes.c_uint32), ("send_tail", ctypes.c_uint32),
                ("tbl", ctypes.POINTER(GclLrpcMsg)), ("recv_head_wb", ctypes.POINTER(ctypes.c_uint32)),
                ("size", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class GclHostProc(ctypes.Structure):
    _fields_ = [("uniqid", ctypes.c_uint16), ("thread_count", ctypes.c_uint16),
                ("active_thread_count", ctypes.c_uint16), ("idle_top", ctypes.c_int16),
                ("flow_tbl", ctypes.c_uint16 * GCL_NCPU),
                ("rxq", ctypes.POINTER(GclLrpcChanOut) * GCL_NCPU)]


SCHED_ADD_CORE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(GclHostProc))
ENABLE_POLL_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(GclHostProc), ctypes.c_uint)
FREE_PKT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64)
OWNED_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(GclHostProc), ctypes.c_uint64)
REFCNT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int)
ARP_RESPOND_FN = ctypes.CFUNCTYPE(ctypes.c_bool, ctypes.c_void_p, ctypes.c_uint64)


class GclHostOps(ctypes.Structure):
    _fields_ = [("arg", ctypes.c_void_p), ("sched_add_core", SCHED_ADD_CORE_FN),
                ("enable_poll", ENABLE_POLL_FN), ("free_pkt", FREE_PKT_FN),
                ("owned", OWNED_FN), ("refcnt_update", REFCNT_FN),
                ("arp_respond", ARP_RESPOND_FN)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `python caladan_amd/build.py` "
                          "(the classifier has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "gcl_open": (i32, [i32, ctypes.POINTER(GclCfg), ctypes.POINTER(vp)]),
        "gcl_close": (None, [vp]),
        "gcl_runtime_set": (i32, [vp, u16, u32, u16, u16, ctypes.POINTER(u16)]),
        "gcl_runtime_del": (i32, [vp, u16]),
        "gcl_steer_flows": (i32, [u16, ctypes.POINTER(u16), u16, ctypes.POINTER(u16)]),
        "gcl_classify": (i32, [vp, ctypes.POINTER(GclBatch), vp, vp, vp, vp]),
        "gcl_classify_ex": (i32, [vp, ctypes.POINTER(GclBatch), ctypes.POINTER(GclOut), vp]),
        "gcl_access_probe": (i32, [vp, ctypes.POINTER(GclBatch), vp, u32, vp]),
        "gcl_runtime_set_trans_seed": (i32, [vp, u16, u32]),
        "gcl_crc32c_u64": (u32, [u32, u64]),
        "gcl_trans_hash": (None, [u32, ctypes.c_uint8, u32, u16, u32, u16, ctypes.POINTER(GclTrans)]),
        "gcl_sync": (i32, [vp]),
        "gcl_kernel_time": (i32, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64), i32]),
        "gcl_profile_sample": (i32, [vp, u32]),
        "gcl_generate": (i32, [ctypes.POINTER(GclGenParams), vp, vp, vp, vp]),
        "gcl_runtime_ip": (u32, [u32]),
        "gcl_loopback_olflags": (ctypes.c_uint8, [ctypes.c_uint8]),
        "gcl_txpkt_rss": (u32, [u64]),
        "gcl_zipf_cdf": (i32, [u32, ctypes.c_double, vp]),
        "gcl_jenkins_hash": (u32, [ctypes.c_char_p, ctypes.c_size_t]),
        "gcl_toeplitz": (u32, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]),
        "gcl_version": (ctypes.c_char_p, []),
        "gcl_lrpc_init_out": (i32, [ctypes.POINTER(GclLrpcChanOut), ctypes.POINTER(GclLrpcMsg), ctypes.c_uint, ctypes.POINTER(u32)]),
        "gcl_lrpc_send": (ctypes.c_bool, [ctypes.POINTER(GclLrpcChanOut), u64, ctypes.c_ulong]),
        "gcl_rx_make_cmd": (u64, [u16, ctypes.c_uint8]),
        "gcl_classify_host": (i32, [vp, ctypes.POINTER(GclBatch), vp, vp, vp, ctypes.POINTER(GclE2eOpts)]),
        "gcl_host_register": (i32, [vp, ctypes.c_size_t]),
        "gcl_dev_alloc": (i32, [i32, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "gcl_dev_free": (i32, [vp]),
        "gcl_rxloop_start": (i32, [vp, ctypes.POINTER(GclRxloopCfg), ctypes.POINTER(vp)]),
        "gcl_rxloop_submit": (ctypes.c_int64, [vp, u32, vp, vp, vp, vp, vp]),
        "gcl_rxloop_wait": (i32, [vp, ctypes.c_int64, vp, u64]),
        "gcl_rxloop_stop": (i32, [vp]),
        "gcl_rxloop_drive": (i32, [vp, u32, vp, u32, u32, vp, ctypes.POINTER(u64)]),
        "gcl_dev_alloc_paired": (i32, [i32, ctypes.c_size_t, vp, ctypes.c_size_t, u32,
                                       ctypes.POINTER(vp), ctypes.POINTER(GclPairInfo)]),
        "gcl_host_unregister": (i32, [vp]),
        "gcl_pcap_write": (i32, [ctypes.c_char_p, vp, u64, vp, vp, vp, u64, u32]),
        "gcl_pcap_load": (i32, [ctypes.c_char_p, ctypes.POINTER(GclTrace), u64]),
        "gcl_pcap_free": (None, [ctypes.POINTER(GclTrace)]),
        "gcl_host_deliver": (u64, [vp, u32, vp, i32, vp, vp, vp, ctypes.c_uint8, vp, u64,
                                   ctypes.POINTER(GclHostOps), vp]),
        "gcl_host_deliver4": (u64, [vp, u32, vp, i32, vp, vp, vp, vp, ctypes.c_uint8, vp, u64,
                                    ctypes.POINTER(GclHostOps), vp]),
        "gcl_host_deliver2": (u64, [vp, u32, vp, i32, vp, ctypes.c_uint8, vp, vp, vp,
                                    ctypes.c_uint8, vp, u64, ctypes.POINTER(GclHostOps), vp]),
        "gcl_verdict2_to4": (ctypes.c_uint32, [ctypes.c_uint16, ctypes.c_uint8]),
        "gcl_host_deliver1": (u64, [vp, u32, vp, i32, vp, ctypes.c_uint8, vp, vp, vp,
                                    ctypes.c_uint8, vp, u64, ctypes.POINTER(GclHostOps), vp]),
        "gcl_verdict1_to4": (ctypes.c_uint32, [ctypes.c_uint8, ctypes.c_uint8]),
        "gcl_host_deliver_recs": (u64, [vp, u32, vp, i32, vp, ctypes.c_uint8, ctypes.c_uint8, vp, vp,
                                        vp, ctypes.c_uint8, vp, u64, ctypes.POINTER(GclHostOps), vp]),
        "gcl_host_prefetch_rxq": (None, [vp, i32]),
        "gcl_rxloop_peek": (i32, [vp, ctypes.c_int64, u64, ctypes.POINTER(vp), ctypes.POINTER(u32)]),
        "gcl_rxloop_release": (i32, [vp, ctypes.c_int64]),
        "gcl_rxloop_poll_stats": (i32, [vp, vp]),
        "gcl_rxloop_lean_bursts": (i32, [vp, vp]),
        "gcl_rxloop_trans": (i32, [vp, ctypes.c_int64, vp]),
        "gcl_tune_init": (None, [ctypes.POINTER(GclTune)]),
        "gcl_ctx_tune": (i32, [vp, ctypes.POINTER(GclTune)]),
        "gcl_abi_version": (i32, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def _check(ret, what):
    if ret < 0:
        raise OSError(-ret, f"{what}: {os.strerror(-ret)}")
    return ret


def _ptr(x):
    """Device/host address of a torch tensor or numpy array (None -> NULL)."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return int(x)


def _nbytes(x):
    if hasattr(x, "numel"):
        return x.numel() * x.element_size()
    if isinstance(x, int):  # raw device address: caller vouches for the size
        return 1 << 62
    return x.nbytes


def _frames_len(frames, frames_len):
    """The readable length the kernel is given: the whole buffer, or a
    caller's shorter limit -- never more than the buffer holds (the kernel
    trusts it as the bound of every frame read)."""
    size = _nbytes(frames)
    if frames_len is None:
        return size
    if frames_len < 0 or frames_len > size:
        raise ValueError(f"frames_len {frames_len} exceeds the {size}-byte frame buffer")
    return frames_len


def make_tune(**kw):
    """A struct gcl_tune with the library's defaults (gcl_tune_init) and the
    fields in @kw set; loop_phase=(max, up, down) sets the three phase fields
    together (0 as max: off)."""
    t = GclTune()
    lib.gcl_tune_init(ctypes.byref(t))
    ph = kw.pop("loop_phase", None)
    if ph is not None:
        ph = tuple(ph) if not isinstance(ph, int) else (ph,)
        t.loop_phase_max = ph[0]
        t.loop_phase_up = ph[1] if len(ph) > 1 else 16
        t.loop_phase_down = ph[2] if len(ph) > 2 else 1
    for k, v in kw.items():
        if not hasattr(t, k) or k in ("size", "pad"):
            raise AttributeError(f"struct gcl_tune has no field {k}")
        setattr(t, k, int(v))
    return t


def jenkins_hash(key: bytes) -> int:
    return lib.gcl_jenkins_hash(key, len(key))


def toeplitz(key: bytes, data: bytes) -> int:
    return lib.gcl_toeplitz(key, len(key), data, len(data))


def crc32c_u64(crc, val):
    return lib.gcl_crc32c_u64(crc, val)


def trans_hash(seed, proto, lip, lport, rip, rport):
    t = GclTrans()
    lib.gcl_trans_hash(seed, proto, lip, lport, rip, rport, ctypes.byref(t))
    return t.h5, t.h3


def runtime_ip(r: int) -> int:
    return lib.gcl_runtime_ip(r)


def steer_flows(thread_count, active_idx):
    """sched_steer_flows (iokernel/sched.c:122-147); returns the flow table."""
    n = len(active_idx)
    act = (ctypes.c_uint16 * max(n, 1))(*active_idx)
    out = (ctypes.c_uint16 * thread_count)(*([0] * thread_count))
    _check(lib.gcl_steer_flows(thread_count, act, n, out), "gcl_steer_flows")
    return list(out)


class DeviceBuffer:
    """hipMalloc'd device memory owned by the library (gcl_dev_alloc): a raw
    address with the duck-typed interface the binding accepts (data_ptr,
    numel, element_size)."""

    def __init__(self, nbytes, device=0, partner=None, new_reads=True, vbytes=4):
        """partner: another buffer (data_ptr/numel); the new one is then placed
        by gcl_dev_alloc_paired so that reading the frame side while writing
        the verdict side does not hit the same-placement-class slowdown.
        new_reads: the new buffer is the frame (read) side.
        vbytes: the verdict width the classifier will write (1, 2, 4 or 8)."""
        p = ctypes.c_void_p()
        self.probe_us = None
        self.pair_info = None
        if partner is None:
            _check(lib.gcl_dev_alloc(device, nbytes, ctypes.byref(p)), "gcl_dev_alloc")
        else:
            info = GclPairInfo()
            _check(lib.gcl_dev_alloc_paired(device, nbytes, _ptr(partner), _nbytes(partner),
                                            (PAIR_NEW_READS if new_reads else PAIR_NEW_WRITES) |
                                            vbytes << 8,
                                            ctypes.byref(p), ctypes.byref(info)), "gcl_dev_alloc_paired")
            self.probe_us = (info.chosen_us, info.worst_us)
            self.pair_info = {"probe_us_chosen": round(info.chosen_us, 2),
                              "probe_us_worst": round(info.worst_us, 2),
                              "candidates": info.candidates, "classes_seen": info.classes,
                              "spacer_MiB": info.spacer_bytes >> 20,
                              "probe_write_bytes": info.probe_write_bytes}
        self.ptr, self.nbytes = p.value, nbytes

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes

    def element_size(self):
        return 1

    def free(self):
        if self.ptr:
            lib.gcl_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Trace:
    """A pcap trace loaded by gcl_pcap_load: packed 16-B-aligned frames in
    host memory with numpy views of offsets, lengths and timestamps."""

    def __init__(self, path, max_pkts=0):
        self.t = GclTrace()
        _check(lib.gcl_pcap_load(os.fsencode(path), ctypes.byref(self.t), max_pkts), "gcl_pcap_load")
        n = self.t.n
        self.n = n
        self.skipped = self.t.skipped  # records longer than 65535 bytes, not loaded

        def view(ptr, ctype, count, dtype):
            if not count:
                return np.zeros(0, dtype=dtype)
            return np.ctypeslib.as_array((ctype * count).from_address(ptr)).view(dtype)
        self.frames = view(self.t.frames, ctypes.c_uint8, self.t.alloc_len, np.uint8)
        self.frames_len = self.t.frames_len
        self.offs = view(self.t.offs, ctypes.c_uint64, n, np.uint64)
        self.pkt_len = view(self.t.pkt_len, ctypes.c_uint16, n, np.uint16)
        self.orig_len = view(self.t.orig_len, ctypes.c_uint32, n, np.uint32)
        self.ts_ns = view(self.t.ts_ns, ctypes.c_uint64, n, np.uint64)

    def close(self):
        if self.t.frames:
            lib.gcl_pcap_free(ctypes.byref(self.t))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_register(arr):
    """Pin + map a host numpy array for ZEROCOPY (gcl_host_register)."""
    _check(lib.gcl_host_register(arr.ctypes.data, arr.nbytes), "gcl_host_register")


def host_unregister(arr):
    return lib.gcl_host_unregister(arr.ctypes.data)


def pcap_write(path, frames, pkt_len, stride=0, offs=None, ts_ns=None, snaplen=0):
    n = len(pkt_len)
    pl = np.ascontiguousarray(pkt_len, dtype=np.uint16)
    o = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    ts = None if ts_ns is None else np.ascontiguousarray(ts_ns, dtype=np.uint64)
    _check(lib.gcl_pcap_write(os.fsencode(path), _ptr(frames), stride, _ptr(o), _ptr(pl),
                              _ptr(ts), n, snaplen), "gcl_pcap_write")


# The reference's ingress mbuf pool (iokernel/defs.h:70, :503-523; rx.c:398-415):
# 2 MiB pages of 9408-B elements, 222 per page; an element is a 64-B mempool
# object header, the 128-B rte_mbuf, 24 B of rx_priv_data and 128 B of
# headroom before the frame, so frame data sits at element + 344 (8-B aligned).
RX_ELT_SIZE = 9408
RX_ELT_PER_PAGE = (2 << 20) // RX_ELT_SIZE
RX_DATA_OFF = 64 + 128 + 24 + 128
IOKERNEL_NUM_MBUFS = 8192 * 16


def mbuf_data_offsets(nmbufs=IOKERNEL_NUM_MBUFS):
    """Offset of mbuf i's frame data from the ingress region base
    (rte_pktmbuf_mtod(m) - dp.ingress_mbuf_region.base, rx.c:82), u64[nmbufs]."""
    i = np.arange(nmbufs, dtype=np.uint64)
    return ((i // RX_ELT_PER_PAGE) * np.uint64(2 << 20) + (i % RX_ELT_PER_PAGE) * np.uint64(RX_ELT_SIZE)
            + np.uint64(RX_DATA_OFF))


def mbuf_region_bytes(nmbufs=IOKERNEL_NUM_MBUFS):
    """Bytes of ingress region holding @nmbufs elements (whole 2 MiB pages)."""
    return -(-nmbufs // RX_ELT_PER_PAGE) * (2 << 20)


def zipf_cdf(nflows, s=0.99):
    cdf = np.empty(nflows, dtype=np.uint64)
    _check(lib.gcl_zipf_cdf(nflows, s, cdf.ctypes.data), "gcl_zipf_cdf")
    return cdf


def generate(workload, n, stride, nruntimes, frames, olflags=None, rss=None, seed=0xCA1ADA4,
             rank=0, world=1, shard_block=0, zipf_cdf_dev=None, nflows=0, stream=None,
             pkt_len=None):
    """Fill device buffers with synthetic rx traffic (gcl_generate)."""
    if _nbytes(frames) < n * stride:
        raise ValueError("frames buffer too small")
    if pkt_len is not None and _nbytes(pkt_len) < 2 * n:
        raise ValueError("pkt_len buffer too small")
    p = GclGenParams(workload=workload, nruntimes=nruntimes, seed=seed, n=n, stride=stride,
                     rank=rank, world=world, shard_block=shard_block,
                     zipf_cdf=_ptr(zipf_cdf_dev), nflows=nflows, pkt_len=_ptr(pkt_len))
    _check(lib.gcl_generate(ctypes.byref(p), _ptr(frames), _ptr(olflags), _ptr(rss), stream),
           "gcl_generate")


def verdict_bytes(flags):
    return 1 if flags & CFG_VERDICT1 else 2 if flags & CFG_VERDICT2 else 4 if flags & CFG_VERDICT4 else 8


def verdict_dtype(vbytes):
    return {1: np.dtype("u1"), 2: np.dtype("<u2"), 4: VERDICT4_DTYPE, 8: VERDICT_DTYPE}[vbytes]


def thread_bits_for(max_runtimes, max_threads):
    """Smallest GclCfg.thread_bits that holds @max_threads kthreads per runtime;
    None when max_runtimes << thread_bits would exceed the 2-byte verdict."""
    tb = max(0, (int(max_threads) - 1).bit_length())
    return tb if tb <= 8 and (max_runtimes << tb) <= V2_QUEUES else None


class Classifier:
    """One gcl_ctx: the GPU side of one dataplane (iokernel/dpdk.c:276-280)."""

    def __init__(self, device=0, max_runtimes=16, hash_mode=HASH_JENKINS, flags=0,
                 default_olflags=F_RSS_HASH | F_IP_CKSUM_GOOD, rss_key=CALADAN_RSS_KEY,
                 thread_bits=0, tune=None):
        if isinstance(hash_mode, str):
            hash_mode = HASH_MODES[hash_mode]
        cfg = GclCfg(max_runtimes=max_runtimes, hash_mode=hash_mode, flags=flags,
                     default_olflags=default_olflags, thread_bits=thread_bits)
        key = bytes(rss_key)[:40].ljust(40, b"\0")
        for i in range(40):
            cfg.rss_key[i] = key[i]
        self.cfg = cfg
        self.max_runtimes = max_runtimes
        self.vbytes = verdict_bytes(flags)  # bytes per verdict
        self.thread_bits = thread_bits
        self._ctx = ctypes.c_void_p()
        _check(lib.gcl_open(device, ctypes.byref(cfg), ctypes.byref(self._ctx)), "gcl_open")
        if tune:
            self.tune(**tune)

    def tune(self, **kw):
        """gcl_ctx_tune: the library's defaults with the fields in @kw
        overridden (make_tune); no arguments: back to the defaults.  Batch
        fields apply from the next classify, loop fields from the next rxloop."""
        t = make_tune(**kw)
        return _check(lib.gcl_ctx_tune(self._ctx, ctypes.byref(t)), "gcl_ctx_tune")

    def close(self):
        loop = getattr(self, "_loop", None)
        if loop is not None:
            loop.stop()  # gcl_close would free it under the RxLoop object
        if self._ctx:
            lib.gcl_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def runtime_set(self, uniqid, ip, thread_count, active_count, flow_tbl=None):
        tbl = None
        if flow_tbl is not None:
            tbl = (ctypes.c_uint16 * max(len(flow_tbl), 1))(*flow_tbl)
        return _check(lib.gcl_runtime_set(self._ctx, uniqid, ip, thread_count, active_count, tbl),
                      "gcl_runtime_set")

    def runtime_del(self, uniqid):
        return _check(lib.gcl_runtime_del(self._ctx, uniqid), "gcl_runtime_del")

    def set_trans_seed(self, uniqid, seed):
        return _check(lib.gcl_runtime_set_trans_seed(self._ctx, uniqid, seed),
                      "gcl_runtime_set_trans_seed")

    def classify(self, frames, n, stride=0, verdicts=None, counts=None, stats=None, offs=None,
                 olflags=None, rss=None, fdir_hi=None, frames_len=None, stream=None,
                 dst_hint=None, trans=None):
        """Launch the classify kernel on device buffers (asynchronous)."""
        if verdicts is not None and _nbytes(verdicts) < self.vbytes * n:
            raise ValueError("verdict buffer too small")
        if counts is not None and _nbytes(counts) < 8 * self.max_runtimes:
            raise ValueError("counts buffer too small")
        if stats is not None and _nbytes(stats) < 8 * NR_STATS:
            raise ValueError("stats buffer too small")
        for arr, w in ((offs, 8), (olflags, 1), (rss, 4), (fdir_hi, 4), (dst_hint, 4)):
            if arr is not None and _nbytes(arr) < w * n:
                raise ValueError("per-packet array too small")
        b = GclBatch(frames=_ptr(frames),
                     frames_len=_frames_len(frames, frames_len),
                     stride=stride, offs=_ptr(offs), olflags=_ptr(olflags), rss=_ptr(rss),
                     fdir_hi=_ptr(fdir_hi), pkt_len=None, n=n, dst_hint=_ptr(dst_hint))
        if trans is not None and _nbytes(trans) < 8 * n:
            raise ValueError("trans buffer too small")
        o = GclOut(verdicts=_ptr(verdicts), runtime_counts=_ptr(counts), stats=_ptr(stats),
                   trans=_ptr(trans))
        return _check(lib.gcl_classify_ex(self._ctx, ctypes.byref(b), ctypes.byref(o), stream),
                      "gcl_classify_ex")

    def access_probe(self, frames, n, stride=0, out=None, vbytes=None, offs=None, olflags=None,
                     rss=None, frames_len=None, stream=None, minimal=False):
        """gcl_access_probe: at the context's verdict width, the classify
        launch itself (tile or pair kernel) with rx_one_pkt folded away (the
        kernel's own ceiling); at another width, or with @minimal, the fewest
        requests the frame layout allows (the layout's ceiling).  Asynchronous."""
        vbytes = self.vbytes if vbytes is None else vbytes
        if out is None or _nbytes(out) < vbytes * n:
            raise ValueError("probe output buffer too small")
        if minimal:
            vbytes |= PROBE_MIN
        b = GclBatch(frames=_ptr(frames), frames_len=_frames_len(frames, frames_len),
                     stride=stride, offs=_ptr(offs), olflags=_ptr(olflags), rss=_ptr(rss),
                     fdir_hi=None, pkt_len=None, n=n, dst_hint=None)
        return _check(lib.gcl_access_probe(self._ctx, ctypes.byref(b), _ptr(out), vbytes, stream),
                      "gcl_access_probe")

    def classify_host(self, frames, n, stride=0, verdicts=None, counts=None, stats=None,
                      olflags=None, rss=None, fdir_hi=None, offs=None, frames_len=None,
                      mode=E2E_COPY, nstreams=2, chunk=1 << 20, dst_hint=None):
        """End-to-end: host (pinned) frames in, host verdicts out (synchronous)."""
        if verdicts is not None and _nbytes(verdicts) < self.vbytes * n:
            raise ValueError("verdict buffer too small")
        b = GclBatch(frames=_ptr(frames),
                     frames_len=_frames_len(frames, frames_len),
                     stride=stride, offs=_ptr(offs), olflags=_ptr(olflags), rss=_ptr(rss),
                     fdir_hi=_ptr(fdir_hi), pkt_len=None, n=n, dst_hint=_ptr(dst_hint))
        o = GclE2eOpts(mode=mode, nstreams=nstreams, chunk=chunk)
        return _check(lib.gcl_classify_host(self._ctx, ctypes.byref(b), _ptr(verdicts), _ptr(counts),
                                            _ptr(stats), ctypes.byref(o)), "gcl_classify_host")

    def rxloop(self, region, slots=64, max_burst=GCL_RX_BURST_SIZE, workers=1, lifetime_ms=20000,
               counts=None, stats=None, region_len=None, flags=0):
        """Start the persistent rx loop over a registered host region."""
        return RxLoop(self, region, slots, max_burst, workers, lifetime_ms, counts, stats,
                      region_len, flags)

    def sync(self):
        return _check(lib.gcl_sync(self._ctx), "gcl_sync")

    def profile_sample(self, every):
        """Time one launch in `every` (GCL_CFG_PROFILE); see gcl_profile_sample."""
        return _check(lib.gcl_profile_sample(self._ctx, int(every)), "gcl_profile_sample")

    def kernel_time(self, reset=False):
        ms = ctypes.c_double()
        nl = ctypes.c_uint64()
        _check(lib.gcl_kernel_time(self._ctx, ctypes.byref(ms), ctypes.byref(nl), int(reset)),
               "gcl_kernel_time")
        return ms.value, nl.value


def version():
    return lib.gcl_version().decode()


# ------------------------------------------------------------- multi-GPU group
GROUP_LIB_PATH = os.path.join(HERE, "libgclgroup.so")
GROUP_BLOCK = 64 << 10
XCHG_RCCL, XCHG_HOST = 0, 1
GROUP_FAULT_EXCHANGE = 0x1


class GclGroupCfg(ctypes.Structure):
    """struct gcl_group_cfg (GCL_GROUP_ABI 2): `size` is filled in here."""
    _fields_ = [("block", ctypes.c_uint64), ("exchange", ctypes.c_uint32),
                ("nstreams", ctypes.c_uint32), ("init_timeout_ms", ctypes.c_uint32),
                ("size", ctypes.c_uint32)]

    def __init__(self, **kw):
        kw.setdefault("size", ctypes.sizeof(GclGroupCfg))
        super().__init__(**kw)


_glib = None


def group_lib():
    """libgclgroup.so (include/gcl_group.h), loaded on first use: the
    single-GPU binding never pulls in RCCL."""
    global _glib
    if _glib is not None:
        return _glib
    if not os.path.exists(GROUP_LIB_PATH):
        raise ImportError(f"{GROUP_LIB_PATH} missing: run `python caladan_amd/build.py`")
    gl = ctypes.CDLL(GROUP_LIB_PATH)
    vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "gcl_group_open_v2": (i32, [i32, ctypes.POINTER(i32), ctypes.POINTER(GclCfg),
                                    ctypes.POINTER(GclGroupCfg), ctypes.POINTER(vp)]),
        # the ABI-1 symbol (16-B struct gcl_group_cfg_v1), kept for old binaries
        "gcl_group_open": (i32, [i32, ctypes.POINTER(i32), ctypes.POINTER(GclCfg),
                                 vp, ctypes.POINTER(vp)]),
        "gcl_group_close": (None, [vp]),
        "gcl_group_size": (i32, [vp]),
        "gcl_group_ctx": (vp, [vp, i32]),
        "gcl_group_stream": (vp, [vp, i32]),
        "gcl_group_runtime_set": (i32, [vp, u16, u32, u16, u16, ctypes.POINTER(u16)]),
        "gcl_group_runtime_del": (i32, [vp, u16]),
        "gcl_group_runtime_set_trans_seed": (i32, [vp, u16, u32]),
        "gcl_shard_count": (u64, [u64, u32, u32, u64]),
        "gcl_shard_global": (u64, [u64, u32, u32, u64]),
        "gcl_group_classify": (i32, [vp, ctypes.POINTER(GclBatch), ctypes.POINTER(vp)]),
        "gcl_group_classify_host": (i32, [vp, ctypes.POINTER(GclBatch), vp, ctypes.POINTER(GclE2eOpts)]),
        "gcl_group_exchange": (i32, [vp]),
        "gcl_group_read": (i32, [vp, vp, vp, vp]),
        "gcl_group_reset": (i32, [vp]),
        "gcl_group_sync": (i32, [vp]),
        "gcl_group_test_fault": (i32, [vp, u32]),
        "gcl_group_rccl_ranks": (i32, [vp, ctypes.POINTER(i32)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(gl, name)
        f.restype = res
        f.argtypes = args
    _glib = gl
    return gl


def shard_count(n, world, rank, block=GROUP_BLOCK):
    return group_lib().gcl_shard_count(n, world, rank, block)


def shard_global(j, world, rank, block=GROUP_BLOCK):
    return group_lib().gcl_shard_global(j, world, rank, block)


class Group:
    """gcl_group: one dataplane driving several GPUs (include/gcl_group.h) --
    a gcl_ctx per GPU, round-robin block shards, RCCL all-gather of the
    per-runtime counts and rx counters."""

    def __init__(self, devices, max_runtimes=16, hash_mode=HASH_JENKINS, flags=0,
                 default_olflags=F_RSS_HASH | F_IP_CKSUM_GOOD, rss_key=CALADAN_RSS_KEY,
                 thread_bits=0, block=GROUP_BLOCK, exchange=XCHG_RCCL, nstreams=2,
                 init_timeout_ms=0):
        gl = group_lib()
        if isinstance(hash_mode, str):
            hash_mode = HASH_MODES[hash_mode]
        cfg = GclCfg(max_runtimes=max_runtimes, hash_mode=hash_mode, flags=flags,
                     default_olflags=default_olflags, thread_bits=thread_bits)
        key = bytes(rss_key)[:40].ljust(40, b"\0")
        for i in range(40):
            cfg.rss_key[i] = key[i]
        self.devices = list(devices)
        self.n = len(self.devices)
        self.max_runtimes = max_runtimes
        self.vbytes = verdict_bytes(flags)
        self.block = block
        devs = (ctypes.c_int * self.n)(*self.devices)
        gc = GclGroupCfg(block=block, exchange=exchange, nstreams=nstreams,
                         init_timeout_ms=init_timeout_ms)
        self._g = ctypes.c_void_p()
        _check(gl.gcl_group_open_v2(self.n, devs, ctypes.byref(cfg), ctypes.byref(gc), ctypes.byref(self._g)),
               "gcl_group_open_v2")

    def close(self):
        if self._g:
            group_lib().gcl_group_close(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self, i=0):
        return group_lib().gcl_group_stream(self._g, i)

    def runtime_set(self, uniqid, ip, thread_count, active_count, flow_tbl=None):
        tbl = None
        if flow_tbl is not None:
            tbl = (ctypes.c_uint16 * max(len(flow_tbl), 1))(*flow_tbl)
        return _check(group_lib().gcl_group_runtime_set(self._g, uniqid, ip, thread_count, active_count, tbl),
                      "gcl_group_runtime_set")

    def runtime_del(self, uniqid):
        return _check(group_lib().gcl_group_runtime_del(self._g, uniqid), "gcl_group_runtime_del")

    def classify(self, shards, verdicts):
        """shards: one dict per GPU (frames, n, stride, and optional offs,
        olflags, rss, fdir_hi, dst_hint, frames_len) of device buffers on that
        GPU; verdicts: one device buffer per GPU.  Asynchronous."""
        if len(shards) != self.n or len(verdicts) != self.n:
            raise ValueError("one shard and one verdict buffer per GPU")
        bs = (GclBatch * self.n)()
        vs = (ctypes.c_void_p * self.n)()
        for i, (s, v) in enumerate(zip(shards, verdicts)):
            if _nbytes(v) < self.vbytes * s["n"]:
                raise ValueError("verdict buffer too small")
            bs[i] = GclBatch(frames=_ptr(s["frames"]), frames_len=_frames_len(s["frames"], s.get("frames_len")),
                             stride=s.get("stride", 0), offs=_ptr(s.get("offs")),
                             olflags=_ptr(s.get("olflags")), rss=_ptr(s.get("rss")),
                             fdir_hi=_ptr(s.get("fdir_hi")), pkt_len=None, n=s["n"],
                             dst_hint=_ptr(s.get("dst_hint")))
            vs[i] = _ptr(v)
        return _check(group_lib().gcl_group_classify(self._g, bs, vs), "gcl_group_classify")

    def classify_host(self, frames, n, stride=0, verdicts=None, offs=None, olflags=None, rss=None,
                      fdir_hi=None, dst_hint=None, frames_len=None, mode=E2E_ZEROCOPY, nstreams=0):
        """One host batch split round-robin over the GPUs (synchronous)."""
        if verdicts is None or _nbytes(verdicts) < self.vbytes * n:
            raise ValueError("verdict buffer too small")
        b = GclBatch(frames=_ptr(frames), frames_len=_frames_len(frames, frames_len), stride=stride,
                     offs=_ptr(offs), olflags=_ptr(olflags), rss=_ptr(rss), fdir_hi=_ptr(fdir_hi),
                     pkt_len=None, n=n, dst_hint=_ptr(dst_hint))
        o = GclE2eOpts(mode=mode, nstreams=nstreams, chunk=0)
        return _check(group_lib().gcl_group_classify_host(self._g, ctypes.byref(b), _ptr(verdicts),
                                                          ctypes.byref(o)), "gcl_group_classify_host")

    def exchange(self):
        return _check(group_lib().gcl_group_exchange(self._g), "gcl_group_exchange")

    def read(self):
        """(node counts u64[R], node stats u64[8], per-GPU vectors u64[n, R + 8])
        of the last exchange."""
        c = np.zeros(self.max_runtimes, dtype=np.uint64)
        s = np.zeros(NR_STATS, dtype=np.uint64)
        p = np.zeros((self.n, self.max_runtimes + NR_STATS), dtype=np.uint64)
        _check(group_lib().gcl_group_read(self._g, c.ctypes.data, s.ctypes.data, p.ctypes.data),
               "gcl_group_read")
        return c, s, p

    def reset(self):
        return _check(group_lib().gcl_group_reset(self._g), "gcl_group_reset")

    def sync(self):
        return _check(group_lib().gcl_group_sync(self._g), "gcl_group_sync")

    def rccl_ranks(self):
        """gcl_group_rccl_ranks: ranks of the RCCL communicators (ncclCommCount), 0 for a host exchange."""
        r = ctypes.c_int()
        _check(group_lib().gcl_group_rccl_ranks(self._g, ctypes.byref(r)), "gcl_group_rccl_ranks")
        return r.value

    def test_fault(self, what=GROUP_FAULT_EXCHANGE):
        """gcl_group_test_fault (tests): every later RCCL exchange fails as a
        timed-out enqueue would; 0 clears it."""
        return _check(group_lib().gcl_group_test_fault(self._g, what), "gcl_group_test_fault")


__all__ = [n for n in dir() if not n.startswith("_")]


class RxLoop:
    """gcl_rxloop_*: burst-at-a-time classification by a persistent kernel."""

    def __init__(self, clf, region, slots, max_burst, workers, lifetime_ms, counts, stats,
                 region_len=None, flags=0):
        self.clf, self.max_burst = clf, max_burst
        cfg = GclRxloopCfg(slots=slots, max_burst=max_burst, workers=workers,
                           lifetime_ms=lifetime_ms, region=_ptr(region),
                           region_len=_nbytes(region) if region_len is None else region_len,
                           counts=_ptr(counts), stats=_ptr(stats), flags=flags)
        h = ctypes.c_void_p()
        _check(lib.gcl_rxloop_start(clf._ctx, ctypes.byref(cfg), ctypes.byref(h)), "gcl_rxloop_start")
        self._h = h
        clf._loop = self

    def submit(self, offs, olflags=None, rss=None, fdir_hi=None, dst_hint=None):
        """Returns the ticket, or a negative errno (-EAGAIN: ring full)."""
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        conv = lambda a, dt: None if a is None else np.ascontiguousarray(a, dtype=dt)
        self._keep = [conv(olflags, np.uint8), conv(rss, np.uint32), conv(fdir_hi, np.uint32),
                      conv(dst_hint, np.uint32)]
        o, r, f, d = self._keep
        return lib.gcl_rxloop_submit(self._h, len(offs), _ptr(offs), _ptr(o), _ptr(r), _ptr(f), _ptr(d))

    def wait(self, ticket, n, spin_ns=2_000_000_000):
        """Verdicts of a burst of @n packets (numpy structured array)."""
        out = np.zeros(n, dtype=verdict_dtype(self.clf.vbytes))
        ret = lib.gcl_rxloop_wait(self._h, ticket, out.ctypes.data, spin_ns)
        if ret:
            raise OSError(-ret, f"gcl_rxloop_wait: {os.strerror(-ret)}")
        return out

    def peek(self, ticket, spin_ns=2_000_000_000):
        """The burst's verdict records in place in the ring slot (a numpy
        view of LOOP_REC_DTYPE, valid until release(ticket))."""
        p = ctypes.c_void_p()
        n = ctypes.c_uint32()
        ret = lib.gcl_rxloop_peek(self._h, ticket, spin_ns, ctypes.byref(p), ctypes.byref(n))
        if ret:
            raise OSError(-ret, f"gcl_rxloop_peek: {os.strerror(-ret)}")
        buf = (ctypes.c_uint8 * (16 * n.value)).from_address(p.value)
        return np.frombuffer(buf, dtype=LOOP_REC_DTYPE)

    def release(self, ticket):
        return _check(lib.gcl_rxloop_release(self._h, ticket), "gcl_rxloop_release")

    def trans(self, ticket, n):
        """The burst's transport demux hashes (TRANS_DTYPE[n]), GCL_CFG_TRANS_HASH contexts."""
        out = np.zeros(n, dtype=TRANS_DTYPE)
        _check(lib.gcl_rxloop_trans(self._h, ticket, out.ctypes.data), "gcl_rxloop_trans")
        return out

    def poll_stats(self):
        """{early, stale, late}: how the bursts so far arrived (gcl_rxloop_poll_stats)."""
        out = np.zeros(3, dtype=np.uint64)
        _check(lib.gcl_rxloop_poll_stats(self._h, out.ctypes.data), "gcl_rxloop_poll_stats")
        return dict(zip(("early", "stale", "late"), (int(x) for x in out)))

    def lean_bursts(self):
        """Bursts classified on rxloop64_kernel's lean path (gcl_rxloop_lean_bursts)."""
        out = np.zeros(1, dtype=np.uint64)
        _check(lib.gcl_rxloop_lean_bursts(self._h, out.ctypes.data), "gcl_rxloop_lean_bursts")
        return int(out[0])

    def drive(self, offs, iters, depth=1):
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lat = np.zeros(iters, dtype=np.uint64)
        el = ctypes.c_uint64()
        _check(lib.gcl_rxloop_drive(self._h, len(offs), _ptr(offs), iters, depth, lat.ctypes.data,
                                    ctypes.byref(el)), "gcl_rxloop_drive")
        return lat, el.value

    def stop(self):
        if self._h:
            h, self._h = self._h, None
            if getattr(self.clf, "_loop", None) is self:
                self.clf._loop = None
            _check(lib.gcl_rxloop_stop(h), "gcl_rxloop_stop")

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass
