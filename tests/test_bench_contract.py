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


@pytest.mark.parametrize("vbytes", [8, 4, 2, 1])
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
    assert bench.verdict_cfg(1, 16, 8) == (g.CFG_VERDICT1, 3)
    with pytest.raises(ValueError):
        bench.verdict_cfg(1, 1024, 4)
    assert bench.fit_vbytes(1, 16, 8) == 1 and bench.fit_vbytes(1, 1024, 4) == 2
    assert bench.fit_vbytes(4, 1024, 4) == 4
    assert set(bench.VERDICT_NAMES) == {8, 4, 2, 1}


def test_workloads_match_baseline_configs(bench):
    """configs[1] (32 Mi x 64 B, 16 runtimes) is the headline workload,
    configs[2] (1500 B, 1024 runtimes, Zipf) the secondary one."""
    wl, n, stride, R, T, _ = bench.WORKLOADS["udp64"]
    assert (n, stride, R) == (32 << 20, 64, 16)
    wl, n, stride, R, T, _ = bench.WORKLOADS["tcp1500"]
    assert (stride, R) == (1536, 1024) and n == 8 << 20


def test_pick_device_refuses_ranks_past_gpus(bench, monkeypatch):
    """One process per GPU: a LOCAL_RANK past the visible GPUs is refused
    (two ranks on one GPU would read as bad scaling), unless the rehearsal
    flag asks for it."""
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 2)
    assert bench.pick_device(1, 2, False) == 1
    with pytest.raises(SystemExit):
        bench.pick_device(2, 4, False)
    assert bench.pick_device(3, 4, True) == 1
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 0)
    with pytest.raises(SystemExit):
        bench.pick_device(0, 1, False)


def test_strong_scaling_split(bench):
    """Config 4: 256 Mi packets split evenly over 1, 2, 4 and 8 ranks in whole
    64 Ki-packet shard blocks (32 Mi per GPU at 8)."""
    for world in (1, 2, 4, 8):
        assert bench.STRONG_TOTAL_PKTS % (world * bench.SHARD_BLOCK) == 0
    assert bench.STRONG_TOTAL_PKTS // 8 == bench.WORKLOADS["udp64"][1]


def test_roofline_traffic_scales_with_batch(bench):
    """The committed PMC bytes (taken at 32 Mi packets) scale per packet to a
    strong-scaling launch's batch."""
    import types
    w = types.SimpleNamespace(name="udp64", n=256 << 20, vbytes=4, bytes_per_pkt=68)
    r = bench.roofline(w, 2.9)
    if r["traffic"] is not None:
        assert abs(r["traffic"] / (w.n * 68) - 1) < 0.01
        assert abs(r["moved"]["frac"] - r["frac"]) < 0.01


def test_frames_len_bounded_by_buffer():
    """The binding refuses a frames_len past the frame buffer (the kernel
    trusts it as the bound of every frame read)."""
    import numpy as np
    from caladan_amd import gclassify as g
    buf = np.zeros(4096, dtype=np.uint8)
    assert g._frames_len(buf, None) == 4096
    assert g._frames_len(buf, 100) == 100
    with pytest.raises(ValueError):
        g._frames_len(buf, 4097)
    with pytest.raises(ValueError):
        g._frames_len(buf, -1)


def test_rxpipe_rows_report_the_median_run(bench, monkeypatch):
    """Each e2e.rx_burst_pipeline row runs tools/rxpipe in three fresh
    processes and reports the median one, with all three rates."""
    import subprocess
    rates = iter([30.0, 10.0, 20.0] * 20)
    calls = []

    def fake_run(cmd, **kw):
        calls.append(cmd)
        line = json.dumps({"burst": int(cmd[1]), "workers": int(cmd[2]), "mpps_one_core": next(rates)})
        return types.SimpleNamespace(returncode=0, stdout=line + "\n", stderr="")

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(os, "access", lambda p, m: True)
    out = bench.rxpipe_bench()
    rows = out["runs"]
    assert out["reps_per_row"] == 3 and len(calls) == 3 * len(rows) and len(rows) >= 10
    for r in rows:
        assert r["mpps_one_core"] == 20.0 and r["mpps_samples"] == [10.0, 20.0, 30.0]
