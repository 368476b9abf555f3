"""bench.py's pieces of the JSON contract that need no GPU: the roofline
object (algorithmic bytes per packet over the measured kernel time, the PMC
traffic committed under profiles/), the verdict configurations, and the
metric/config names BASELINE.json quotes."""
import json
import os
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    pytest.importorskip("torch")
    import bench as b
    return b


def test_metric_matches_baseline(bench):
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert bench.METRIC == base["metric"]
    assert bench.HBM_PEAK_GBS == 8000.0


@pytest.mark.parametrize("vbytes", [8, 4, 2])
def test_roofline_object(bench, vbytes):
    name, n = "udp64", 32 << 20
    w = types.SimpleNamespace(name=name, n=n, vbytes=vbytes, bytes_per_pkt=bench.HDR_BYTES + vbytes)
    r = bench.roofline(w, 0.35)
    algo = n * (64 + vbytes)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["bytes_per_pkt"] == 64 + vbytes
    assert abs(r["achieved"] - algo / 0.35e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-4
    prof = os.path.join(ROOT, "profiles", f"pmc_{name}{'' if vbytes == 8 else f'_v{vbytes}'}.json")
    if os.path.exists(prof):
        # corrected PMC bytes per launch, within 1% of the algorithmic bytes
        assert abs(r["traffic"] / algo - 1) < 0.01
    else:
        assert r["traffic"] is None


def test_verdict_configs(bench):
    from caladan_amd import gclassify as g
    assert bench.verdict_cfg(8, 16, 8) == (0, 0)
    assert bench.verdict_cfg(4, 1024, 4) == (g.CFG_VERDICT4, 0)
    assert bench.verdict_cfg(2, 16, 8) == (g.CFG_VERDICT2, 3)
    assert bench.verdict_cfg(2, 1024, 4) == (g.CFG_VERDICT2, 2)
    assert set(bench.VERDICT_NAMES) == {8, 4, 2}


def test_workloads_match_baseline_configs(bench):
    """configs[1] (32 Mi x 64 B, 16 runtimes) is the headline workload,
    configs[2] (1500 B, 1024 runtimes, Zipf) the secondary one."""
    wl, n, stride, R, T, _ = bench.WORKLOADS["udp64"]
    assert (n, stride, R) == (32 << 20, 64, 16)
    wl, n, stride, R, T, _ = bench.WORKLOADS["tcp1500"]
    assert (stride, R) == (1536, 1024) and n == 8 << 20
