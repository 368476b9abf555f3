"""Summarise a round's rocprofv3 outputs (gpurun_out/prof_<round>) into
profiles/: kernel stats per workload, PMC bytes per classify launch corrected
as MI355X_MICROARCH.md §HBM prescribes, and the membench calibration that
justifies the correction.

    python tools/prof_summary.py r01

FETCH_SIZE correction: on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced read.  tools/membench.hip `calib` dispatches of known size
measure the factor for each access pattern this kernel uses: a 2 GiB
coalesced stream and 64-, 128- and 32-byte header reads at a 1536-B stride all
report exactly half a 128-B line per line touched, so hbm_read = 2 x FETCH_SIZE.
WRITE_SIZE reads exactly (calib rw kernels: 8 B per packet).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR_BYTES = 64
PKTS = {"udp64": 32 << 20, "tcp1500": 8 << 20, "mixed": 1 << 20, "ingress_nic": 8 << 20,
        "ingress_ws": 8 << 20}
# per-packet bytes besides the 64-B header and the verdict: the integrated
# ingress shape reads a u64 offset, u8 ol_flags and u32 hash.rss per descriptor
EXTRA = {"ingress_nic": 8 + 1 + 4, "ingress_ws": 8 + 1 + 4}
# which kernel instance is the workload's: the ingress rows run NIC mode (MODE
# 0) on the GENERAL kernel -- classify_pair_kernel<0, ...> since round 3,
# classify_kernel<0, ...> before -- and tools/ingress_run.py launches one row
KNAME = {"ingress_nic": "_kernel<0,", "ingress_ws": "_kernel<0,"}


def is_kernel(wl, name):
    """The workload's classify kernel -- not classify_kernel<3, ...> or
    classify_pair_kernel<3, ...>, the same launch in gcl_access_probe's mode
    (kModeProbe), which the bench times as the kernel's ceiling after its own
    timed steps."""
    n = name.replace(" ", "")
    return KNAME.get(wl, "classify_kernel") in n and "_kernel<3," not in n


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def calib(base):
    names = []
    jl = os.path.join(base, "calib_FETCH_SIZE.jsonl")
    for line in open(jl):
        line = line.strip()
        if line.startswith("{"):
            names.append(json.loads(line))
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rs = [r for r in rows(os.path.join(base, f"calib_{c}", "run_counter_collection.csv"))
              if "read_kernel" in r["Kernel_Name"] or "rw_kernel" in r["Kernel_Name"]]
        # each pattern is dispatched twice (warm-up + timed)
        for i, meta in enumerate(names):
            vals = [float(rs[2 * i]["Counter_Value"]), float(rs[2 * i + 1]["Counter_Value"])]
            d = out.setdefault(meta["pattern"], {"useful_bytes": meta["useful_bytes"]})
            d[c + "_KB"] = sum(vals) / 2
    for p, d in out.items():
        read_bytes = d["useful_bytes"] if not p.startswith("rw_") else d["useful_bytes"] / 72 * 64
        d["read_bytes_requested"] = read_bytes
        d["fetch_reported_over_requested"] = round(d["FETCH_SIZE_KB"] * 1024 / read_bytes, 4)
    return out


def request_bytes(base, tag, wl):
    """Fabric request counts per classify launch (TCC_EA0_RDREQ / _32B,
    TCC_BUBBLE, TCC_EA0_WRREQ / _64B).  rocprof-compute's gfx950 'HBM
    Bandwidth' formula prices reads as 128 x TCC_BUBBLE + 32 x RDREQ_32B + 64 x
    the rest, but on this ROCm 7.2 / gfx950 TCC_BUBBLE reads 0 even for a
    dense 2 GiB stream that is 16.8 M requests for 2.15 GB (tools/halfline.hip,
    profiles/archive/r01_halfline.jsonl): every read request carries a 128-B line, the
    guide's x2.  So the request counts are reported, and the byte totals use
    128 B per read request and the write counters as documented."""
    d1 = os.path.join(base, f"{tag}_REQ", "run_counter_collection.csv")
    d2 = os.path.join(base, f"{tag}_REQ64", "run_counter_collection.csv")
    if not (os.path.exists(d1) and os.path.exists(d2)):
        return None
    per = {}
    for path in (d1, d2):
        launches = {}
        for r in rows(path):
            if is_kernel(wl, r["Kernel_Name"]):
                launches.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"].replace("_sum", "")] = \
                    float(r["Counter_Value"])
        for c in {k for v in launches.values() for k in v}:
            vals = [v[c] for v in launches.values() if c in v]
            per[c] = sum(vals) / len(vals)
    b, rd, r32, wr, w64 = (per["TCC_BUBBLE"], per["TCC_EA0_RDREQ"], per["TCC_EA0_RDREQ_32B"],
                           per["TCC_EA0_WRREQ"], per["TCC_EA0_WRREQ_64B"])
    rbytes = 128 * (rd - r32) + 32 * r32
    wbytes = 64 * w64 + 32 * (wr - w64)
    return {"req_reads": rd, "req_reads_32B": r32, "req_TCC_BUBBLE": b, "req_writes": wr,
            "req_writes_64B": w64, "hbm_read_bytes_from_requests": rbytes,
            "hbm_write_bytes_from_requests": wbytes, "hbm_bytes_from_requests": rbytes + wbytes}


TIMED_DEFAULT = 20  # tools/profile.sh's trace pass: --steps 20 / 20 ingress reps


def timed_dispatches(tdir, wl, tag, bench_json):
    """Average only the TIMED dispatches of the workload's kernel: the last K
    of the trace pass, K = the bench line's `steps` (its timed steps come
    last: placement checks, warmup and settle launch the same kernel before
    them, and --no-group keeps anything after them out of the pass).  The
    whole-run average of run_kernel_stats.csv mixes in the ramp (the first
    ~40 launches run up to 19 % slower), so this is the figure
    the bench line's roofline is checked against."""
    path = os.path.join(tdir, "run_kernel_trace.csv")
    if not os.path.exists(path):
        return None
    line = {}
    if bench_json and os.path.exists(bench_json):
        with open(bench_json) as f:
            txt = [ln for ln in f.read().splitlines() if ln.startswith("{")]
        line = json.loads(txt[-1]) if txt else {}
    k = int(line.get("steps", TIMED_DEFAULT))
    ds = sorted((r for r in rows(path) if is_kernel(wl, r["Kernel_Name"])),
                key=lambda r: int(r["Start_Timestamp"]))
    kept = ds[-k:]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kept]
    avg = sum(durs) / len(durs)
    out = {"workload": wl, "tag": tag, "kernel": kept[0]["Kernel_Name"],
           "dispatches_in_trace": len(ds), "timed_kept": len(kept),
           "kept_dispatch_ids": [int(r["Dispatch_Id"]) for r in kept],
           "kept_positions": [len(ds) - len(kept), len(ds) - 1],
           "avg_ns": round(avg, 1), "min_ns": min(durs), "max_ns": max(durs),
           "whole_trace_avg_ns": round(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                                           for r in ds) / len(ds), 1)}
    rl = line.get("roofline") or {}
    if wl in ("udp64", "tcp1500") and rl.get("bytes_per_pkt"):
        algo = line["config"]["pkts_per_gpu"] * rl["bytes_per_pkt"]
        frac = algo / (avg * 1e-9) / 1e9 / rl["peak"]
        out.update({"algorithmic_bytes_per_launch": algo, "frac_from_timed_dispatches": round(frac, 4),
                    "bench_line_under_rocprof": {"frac": rl.get("frac"), "kernel_ms": rl.get("kernel_ms"),
                                                 "ms_per_step": line.get("ms_per_step")},
                    "frac_rel_diff": round(frac / rl["frac"] - 1, 4) if rl.get("frac") else None})
    return out


def main(rnd):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    if os.path.isdir(os.path.join(base, "calib_FETCH_SIZE")):
        cal = calib(base)
        with open(os.path.join(prof, f"{rnd}_calibration.json"), "w") as f:
            json.dump({"note": __doc__.strip().split("\n\n")[2], "patterns": cal}, f, indent=1)
    for wl, vb in [(w, v) for w in PKTS for v in (1, 2, 4, 8)]:
        tag = f"{wl}_v{vb}"
        tdir = os.path.join(base, f"{tag}_trace")
        if not os.path.isdir(tdir):
            continue
        shutil.copy(os.path.join(tdir, "run_kernel_stats.csv"),
                    os.path.join(prof, f"{rnd}_{tag}_kernel_stats.csv"))
        td = timed_dispatches(tdir, wl, tag, os.path.join(base, f"{tag}_bench.json"))
        if td:
            with open(os.path.join(prof, f"{rnd}_{tag}_timed.json"), "w") as f:
                json.dump(td, f, indent=1)
            print(json.dumps({k: v for k, v in td.items() if k != "kept_dispatch_ids"}))
        if not os.path.isdir(os.path.join(base, f"{tag}_FETCH_SIZE")):
            continue
        st = [r for r in rows(os.path.join(tdir, "run_kernel_stats.csv")) if is_kernel(wl, r["Name"])]
        pm = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            vals = [float(r["Counter_Value"]) for r in
                    rows(os.path.join(base, f"{tag}_{c}", "run_counter_collection.csv"))
                    if is_kernel(wl, r["Kernel_Name"])]
            pm[c] = sum(vals) / len(vals)
        hbm_read = 2.0 * pm["FETCH_SIZE"] * 1024
        hbm_write = pm["WRITE_SIZE"] * 1024
        algo = PKTS[wl] * (HDR_BYTES + EXTRA.get(wl, 0) + vb)
        avg_ns = float(st[0]["AverageNs"])
        out = {
            "workload": wl,
            "verdict_bytes": vb,
            "kernel": st[0]["Name"],
            "calls": int(st[0]["Calls"]),
            "avg_kernel_ns": avg_ns,
            "min_kernel_ns": float(st[0]["MinNs"]),
            "FETCH_SIZE_KB_per_launch": pm["FETCH_SIZE"],
            "WRITE_SIZE_KB_per_launch": pm["WRITE_SIZE"],
            "fetch_correction": 2.0,
            "hbm_read_bytes_per_launch": hbm_read,
            "hbm_write_bytes_per_launch": hbm_write,
            "hbm_bytes_per_launch": hbm_read + hbm_write,
            "algorithmic_bytes_per_launch": algo,
            "traffic_over_algorithmic": round((hbm_read + hbm_write) / algo, 4),
            "hbm_GBs_from_traffic": round((hbm_read + hbm_write) / (avg_ns * 1e-9) / 1e9, 1),
            "algorithmic_GBs": round(algo / (avg_ns * 1e-9) / 1e9, 1),
            "source": f"gpurun_out/prof_{rnd}/{tag}_{{trace,FETCH_SIZE,WRITE_SIZE}} (rocprofv3)",
        }
        req = request_bytes(base, tag, wl)
        if req:
            out.update(req)
            out["traffic_over_algorithmic_from_requests"] = round(req["hbm_bytes_from_requests"] / algo, 4)
            out["requests_per_pkt"] = round((req["req_reads"] + req["req_writes"]) / PKTS[wl], 4)
        with open(os.path.join(prof, f"pmc_{wl}{'' if vb == 8 else f'_v{vb}'}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
