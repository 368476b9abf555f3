"""The CPU leg of the cold-header pipeline rows (tools/cpupipe over the NIC
emulation of tools/nicsim.h) runs here without a GPU: every packet of every
burst delivered, the rings never full, the pool in 2 MiB pages where the
kernel grants them, for each form bench.py times."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "cpupipe")


@pytest.mark.parametrize("args", [("classify",), ("lrpc",), ("lrpc", "prefetch")])
def test_cpupipe_cold_headers(args):
    if not os.access(EXE, os.X_OK):
        pytest.skip("tools/cpupipe not built (__graft_entry__.build())")
    env = {**os.environ, "RXPIPE_HASH": "nic", "RXPIPE_NIC_THREADS": "2", "RXPIPE_POOL_MBUFS": "4096"}
    r = subprocess.run([EXE, "3000", *args], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-500:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["delivered_check"] == "ok" and d["unicast_fail"] == 0, d
    assert d["mpps_one_core"] > 0 and 0.0 <= d["nic_wait_frac"] <= 1.0
    assert 0.0 <= d["pool_huge_frac"] <= 1.0
    assert d["post"] == ("classify only" if args[0] == "classify" else "classify + rx_make_cmd + lrpc_send")
    assert d["prefetch"].startswith("the burst's") == (len(args) > 1)
