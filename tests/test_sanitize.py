"""ASan + UBSan CPU build of the host C that parses untrusted input
(caladan_amd/build.py --sanitize: csrc/gcl_pcap.c, csrc/gcl_host.c and the
oracle's classifier), driven by tests/fuzz/host_fuzz.c: malformed pcaps
(truncated, oversized incl_len, foreign byte order, cut-off record headers,
random garbage), out-of-range verdicts into the lrpc post-pass, and random
frames straddling frames_len into the oracle.  Any sanitizer report fails
the run.  The ring-consumer side of the post-pass follows
inc/base/lrpc.h:121-140."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

EPROTO = 71


@pytest.fixture(scope="module")
def fuzz_exe(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc missing")
    from caladan_amd import build
    return build.build_sanitized(str(tmp_path_factory.mktemp("san")))


def run(exe, *args, timeout=240):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def _hdr(endian="<", magic=0xA1B23C4D, linktype=1):
    return struct.pack(endian + "IHHiIII", magic, 2, 4, 0, 0, 65535, linktype)


def _rec(endian, data, incl=None, orig=None):
    incl = len(data) if incl is None else incl
    return struct.pack(endian + "IIII", 1, 2, incl, len(data) if orig is None else orig) + data


def test_pcap_malformed_files(fuzz_exe, tmp_path):
    rng = np.random.default_rng(5)
    fr = [bytes(rng.integers(0, 256, size=k, dtype=np.uint8)) for k in (60, 1514, 9014, 65535)]
    cases = {
        # name: (file, return code, packets loaded, records skipped)
        "ok_le": (_hdr() + b"".join(_rec("<", f) for f in fr), 0, 4, 0),
        "ok_be_usec": (_hdr(">", 0xA1B2C3D4) + b"".join(_rec(">", f) for f in fr), 0, 4, 0),
        "header_only": (_hdr(), 0, 0, 0),
        "empty": (b"", -EPROTO, 0, 0),
        "short_header": (_hdr()[:20], -EPROTO, 0, 0),
        "truncated_data": (_hdr() + _rec("<", fr[0]) + _rec("<", fr[1])[:-7], -EPROTO, 0, 0),
        "cut_record_header": (_hdr() + _rec("<", fr[0]) + b"\x01\x02\x03", -EPROTO, 0, 0),
        # a capture longer than a u16 pkt_len (lo MTU 65536, GRO/TSO): skipped, counted
        "incl_65536": (_hdr() + _rec("<", b"\0" * 65536), 0, 0, 1),
        "oversize_between": (_hdr() + _rec("<", fr[0]) + _rec("<", b"\1" * 70000) + _rec("<", fr[1]),
                             0, 2, 1),
        "oversize_be": (_hdr(">", 0xA1B2C3D4) + _rec(">", b"\2" * 262144) + _rec(">", fr[2]), 0, 1, 1),
        # ... but one running past the end of the file is still refused
        "incl_huge": (_hdr() + struct.pack("<IIII", 1, 2, 0xFFFFFFF0, 60) + b"\0" * 64, -EPROTO, 0, 0),
        "incl_past_eof": (_hdr() + struct.pack("<IIII", 1, 2, 4000, 4000) + b"\0" * 100, -EPROTO, 0, 0),
        "oversize_past_eof": (_hdr() + _rec("<", fr[0]) + struct.pack("<IIII", 1, 2, 70000, 70000)
                              + b"\0" * 1000, -EPROTO, 0, 0),
        "zero_len_record": (_hdr() + _rec("<", b"") + _rec("<", fr[0]), 0, 2, 0),
        "not_ethernet": (_hdr(linktype=101) + _rec("<", fr[0]), -EPROTO, 0, 0),
    }
    paths = []
    for name, (data, _, _, _) in cases.items():
        p = tmp_path / f"{name}.pcap"
        p.write_bytes(data)
        paths.append(p)
    for k in range(40):  # random garbage after a valid header, and random files
        p = tmp_path / f"garbage{k}.pcap"
        body = bytes(rng.integers(0, 256, size=int(rng.integers(0, 3000)), dtype=np.uint8))
        p.write_bytes((_hdr() if k % 2 else b"") + body)
        paths.append(p)
    out = run(fuzz_exe, "pcap", *paths)
    got = {}
    for line in out.splitlines():
        path, rc, n, sk, _ = line.rsplit(" ", 4)
        got[os.path.basename(path)[:-5]] = (int(rc), int(n), int(sk))
    for name, (_, rc, n, sk) in cases.items():
        assert got[name] == (rc, n, sk), (name, got[name])
    for k in range(40):
        assert got[f"garbage{k}"][0] in (0, -EPROTO)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_deliver_out_of_range_verdicts(fuzz_exe, seed):
    assert "deliver ok" in run(fuzz_exe, "deliver", seed, 400)


@pytest.mark.parametrize("seed", [11, 12])
def test_oracle_random_frames(fuzz_exe, seed):
    assert "oracle ok" in run(fuzz_exe, "oracle", seed, 300)
