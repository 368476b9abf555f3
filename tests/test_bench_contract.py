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


def _full_result():
    """A fully populated bench result: round 4's final line (the 23-KB one the
    driver could not parse, tests/golden/bench_full_r04.json), with the
    fields added since filled in with fake numbers."""
    with open(os.path.join(ROOT, "tests", "golden", "bench_full_r04.json")) as f:
        r = json.load(f)
    r["roofline"]["traffic_source"] = "profiles/pmc_udp64_v1.json: committed PMC pass, not this run"
    cpu = r["cpu_baseline"]
    cpu["pinning"] = "1-core cells on CPU 7, all-cores cells on 16 distinct physical cores"
    for m in ("nic_mode", "jenkins_mode"):
        cpu[m]["samples"] = {"1core": [60.0, 61.0, 62.0], "1core_lrpc": [50.0] * 3, "all_cores": [900.0] * 3}
        cpu[m]["spread_1core"] = 0.0328
        cpu[m]["spread_all_cores"] = 0.2406
    r["group_node"] = {"n_gpus": 8, "value": 800000.0, "ms_per_step": 0.33, "counts_check": "ok",
                       "what": "x" * 300, "host_ingress_c": {"rows": ["y" * 100] * 20}}
    return r


def test_compact_line_fits_the_driver(bench):
    """The stdout line stays under 8 KB with every section populated, and
    keeps the contract keys, the roofline and the CPU baseline."""
    full = _full_result()
    assert len(json.dumps(full)) > 16000  # the detail really is large
    line = bench.compact(full)
    n = len(json.dumps(line))
    assert n < bench.LINE_LIMIT, n
    for k in bench.CONTRACT_KEYS:
        assert line[k] == full[k]
    rf = line["roofline"]
    assert rf["frac"] == full["roofline"]["frac"] and "frac_of_ceiling" in rf and "traffic_source" in rf
    cb = line["cpu_baseline"]
    assert cb["value"] == full["cpu_baseline"]["value"] and cb["cores"] == 1 and cb["kind"] == "port"
    assert cb["nic_mode"]["1core_lrpc_mpps"] and cb["jenkins_mode"]["all_cores_mpps"]
    assert line["secondary"]["roofline"]["frac"] == full["secondary"]["roofline"]["frac"]
    assert line["header_split"]["value"] and line["toeplitz"]["value"] and line["group"]["counts_check"] == "ok"
    assert line["group_node"]["n_gpus"] == 8
    e = line["e2e"]
    assert e["udp64"]["zerocopy_mpps"] and e["ingress_integrated_nic"]["frac"]
    for k in ("records_1x1_nic", "records_4x8_nic"):
        assert e["pipeline"][k]["mpps_one_core"] > 0
    assert line["detail"]


def test_compact_line_sheds_sections_past_the_limit(bench):
    """Even an oversized summary is cut below the limit, contract keys kept."""
    full = _full_result()
    full["config"]["workload"] = "w" * 1000
    full["secondary"]["verdict"] = "v" * 3000
    full["cpu_baseline"]["sample"] = "s" * 2500
    line = bench.compact(full)
    assert len(json.dumps(line)) < bench.LINE_LIMIT
    assert all(k in line for k in bench.CONTRACT_KEYS) and "roofline" in line and "cpu_baseline" in line


def test_emit_result_writes_detail(bench, tmp_path, monkeypatch, capsys):
    path = tmp_path / "d" / "detail.json"
    monkeypatch.setattr(bench, "DETAIL_PATH", str(path))
    monkeypatch.setattr(bench, "_JSON_FD", None)
    full = _full_result()
    bench.emit_result(full)
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1 and len(out[0]) < bench.LINE_LIMIT
    assert json.loads(out[0])["value"] == full["value"]
    assert json.loads(path.read_text()) == full


def test_pmc_traffic_is_labelled_and_stale_dropped(bench):
    """roofline.traffic comes from a committed profile, and says so; a
    profile whose kernel time disagrees with this run's is dropped."""
    prof = os.path.join(ROOT, "profiles", "pmc_udp64_v1.json")
    if not os.path.exists(prof):
        pytest.skip("no committed udp64 PMC pass")
    avg_ms = json.load(open(prof))["avg_kernel_ns"] / 1e6
    t, src = bench.pmc_traffic("udp64", 1, avg_ms * 1.02)
    assert t and "committed PMC pass" in src and "pmc_udp64_v1.json" in src
    t2, src2 = bench.pmc_traffic("udp64", 1, avg_ms * 1.5)
    assert t2 is None and "stale" in src2
    assert bench.pmc_traffic("nonexistent", 1, 1.0) == (None, None)
    r = bench.roofline_obj(1e9, avg_ms * 1.5, (t2, src2))
    assert r["traffic"] is None and "stale" in r["traffic_source"]


def test_rank_envs_match_torchrun(bench):
    envs = bench.rank_envs(4, 29999, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and
               e["MASTER_PORT"] == "29999" and e["PATH"] == "/bin" for e in envs)
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]


def test_gpus_n_without_launcher_never_prints_a_one_gpu_line():
    """`bench.py --gpus 2` with no WORLD_SIZE spawns two rank processes; here
    (no GPU) both refuse to start, so it exits non-zero with no line -- never
    an n_gpus 1 line for --gpus 2."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "ranks exited" in r.stderr


def test_pick_cores_distinct_physical_idlest_first(bench):
    """Two SMT siblings per core (c, c + 4); core {1, 5} idlest, then {3, 7}."""
    sib = lambda c: frozenset((c % 4, c % 4 + 4))
    a = {c: 0 for c in range(8)}
    b = {0: 10, 4: 10, 1: 90, 5: 90, 2: 30, 6: 30, 3: 50, 7: 50}
    assert bench.pick_cores(2, list(range(8)), a, b, sib) == [1, 3]
    assert bench.pick_cores(8, list(range(8)), a, b, sib) == [1, 3, 2, 0]
    assert bench.pick_cores(1, [2, 6], a, b, sib) == [2]


def test_oracle_bench_pinned_runs():
    """orc_bench_pinned: the CPU baseline's pinned timer (no GPU)."""
    import numpy as np
    from oracle import orc
    from caladan_amd import gclassify as g
    n, stride, R = 4096, 64, 16
    frames, olf, rss = orc.generate(g.WL_UDP64, n, stride, R)
    t = orc.Tables(R, g.HASH_JENKINS, 0, g.F_RSS_HASH)
    for r in range(R):
        t.runtime_set(r, orc.runtime_ip(r), 8, 8, orc.steer_flows(8, list(range(8))))
    cpu = sorted(os.sched_getaffinity(0))[0]
    s = t.bench(frames, n, stride, threads=1, passes=2, olflags=olf, rss=rss, direct=True, cpus=[cpu])
    s2 = t.bench(frames, n, stride, threads=2, passes=2, olflags=olf, rss=rss, direct=True, cpus=[cpu, -1])
    assert s > 0 and s2 > 0


def _fake_children(calls):
    """subprocess.run standing in for bench.py's children: the group child
    (--group-child N), the CPU child (--cpu-child) and tools/grouppipe."""
    def run(cmd, **kw):
        calls.append(cmd)
        if "--group-child" in cmd:
            n = int(cmd[cmd.index("--group-child") + 1])
            line = {"n_gpus": n, "devices": list(range(n)), "exchange": "rccl", "rccl_ranks": n,
                    "value": 95000.0 * n, "unit": "Mpkt/s", "ms_per_step": 0.35, "counts_check": "ok",
                    "what": "g" * 200}
        elif "--cpu-child" in cmd:
            line = {"value": 60.0, "unit": "Mpkt/s", "cores": 1, "kind": "port", "sample": "s" * 300,
                    "nic_mode": {"1core_mpps": 60.0, "1core_lrpc_mpps": 55.0, "all_cores_mpps": 900.0},
                    "jenkins_mode": {"1core_mpps": 50.0, "1core_lrpc_mpps": 42.0, "all_cores_mpps": 800.0},
                    "streams": {"tcp1500": {"x": "y" * 500}}, "seconds": 25.0}
        else:  # tools/grouppipe
            line = {"rows": [{"mode": "zerocopy", "mpps": 700.0}]}
        return types.SimpleNamespace(returncode=0, stdout="banner\n" + json.dumps(line) + "\n", stderr="")
    return run


def test_n2_line_carries_group_node_and_cpu_baseline(bench, monkeypatch):
    """an N>1 line carries the product's multi-GPU path
    (gcl_group over exactly the line's N GPUs, from a fresh child, with the
    RCCL communicators' own rank count) and the CPU baseline (a CPU-only
    child), and the merged line stays under the driver's 8 KB."""
    import subprocess
    calls = []
    monkeypatch.setattr(subprocess, "run", _fake_children(calls))
    monkeypatch.setattr(os, "access", lambda p, m: True)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    args = types.SimpleNamespace(no_group=False, no_cpu=False, group_node_force=False, allow_shared_gpu=False,
                                 steps=50, warmup=5, cpu_budget=30.0)
    ex = bench.node_extras(args, 2, 190000.0)
    grp = [c for c in calls if "--group-child" in c]
    assert len(grp) == 1 and grp[0][grp[0].index("--group-child") + 1] == "2"  # N GPUs, not all 8
    assert "--allow-shared-gpu" not in grp[0]
    assert any("--cpu-child" in c for c in calls)
    assert ex["group_node"]["n_gpus"] == 2 and ex["group_node"]["rccl_ranks"] == 2
    assert ex["cpu_baseline"]["gpu_over_1core_nic"] == round(190000.0 / 60.0, 1)
    full = _full_result()
    full["n_gpus"] = 2
    full.pop("group_node")
    full.update(ex)
    full["exchange"] = {"gpu_ms_per_step": 0.34, "period_steps": 8, "periods": 7, "backend": "nccl", "ranks": 2}
    line = bench.compact(full)
    assert len(json.dumps(line)) < bench.LINE_LIMIT
    assert line["group_node"]["n_gpus"] == 2 and line["group_node"]["rccl_ranks"] == 2
    assert line["group_node"]["exchange"] == "rccl"
    assert line["cpu_baseline"]["value"] == 60.0 and line["cpu_baseline"]["gpu_over_1core_nic"]
    assert line["exchange"]["ranks"] == 2


def test_group_node_only_at_n_gt_1_unless_forced(bench, monkeypatch):
    """At N=1 the group row covers one GPU already: no group_node child
    unless forced; more GPUs than visible only as a shared-GPU rehearsal."""
    import subprocess
    calls = []
    monkeypatch.setattr(subprocess, "run", _fake_children(calls))
    monkeypatch.setattr(os, "access", lambda p, m: True)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    args = types.SimpleNamespace(no_group=False, no_cpu=True, group_node_force=False, allow_shared_gpu=False,
                                 steps=5, warmup=1, cpu_budget=30.0)
    assert bench.group_node_line(args, 1) is None and not calls
    assert "error" in bench.group_node_line(args, 2)  # 2 asked, 1 visible, no rehearsal flag
    args.allow_shared_gpu = True
    node = bench.group_node_line(args, 2)
    assert "--allow-shared-gpu" in calls[-1] and node["n_gpus"] == 2
    args.group_node_force = True
    assert bench.group_node_line(args, 1)["n_gpus"] == 1


def test_cpu_child_runs_without_gpu():
    """`bench.py --cpu-child` (the N>1 lines' CPU baseline) makes no GPU call:
    it runs here, on a box without one, and prints one cpu_baseline object."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-child", "--cpu-budget", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-500:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    cpu = json.loads(lines[0])
    assert cpu["value"] > 0 and cpu["cores"] == 1 and cpu["kind"] == "port"
    assert cpu["nic_mode"]["1core_lrpc_mpps"] > 0 and "tcp1500" in cpu["streams"]
