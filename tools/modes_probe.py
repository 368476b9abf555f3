"""Is the udp64 step's bimodal rate (~92 vs ~100 Gpkt/s in one process on
the same buffers, profiles/archive/r02_streams_ab.jsonl) a clock state?  Runs
200-step samples for ~25 s and records, between samples, the current DPM
levels the amdgpu driver exposes read-only in sysfs (pp_dpm_sclk / mclk /
fclk / socclk, the '*' line) and the hwmon power reading.  Reads only.

    python tools/modes_probe.py > gpurun_out/modes.jsonl
"""
import glob
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def card_dir():
    """The sysfs device directory of the GPU this process sees (by PCI bus id)."""
    bus = torch.cuda.get_device_properties(0).pci_bus_id
    for d in glob.glob("/sys/class/drm/card*/device"):
        try:
            if os.path.basename(os.path.realpath(d)).endswith(f"{bus:02x}:00.0"):
                return d
        except OSError:
            pass
    return None


def read_levels(d):
    out = {}
    if d is None:
        return out
    for k in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk"):
        try:
            for line in open(os.path.join(d, k)):
                if "*" in line:
                    out[k[7:]] = line.strip()
        except OSError:
            pass
    for h in glob.glob(os.path.join(d, "hwmon", "hwmon*")):
        for k in ("power1_average", "power1_input"):
            try:
                out[k] = int(open(os.path.join(h, k)).read()) / 1e6
            except (OSError, ValueError):
                pass
    return out


def main(seconds=25.0):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.Workload("udp64", 0, 1, dev)
    st = torch.cuda.current_stream()
    d = card_dir()
    print(json.dumps({"card": d, "placement": w.frames.pair_info}), flush=True)
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            w.step(st.cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"t": round(time.perf_counter() - t_end + seconds, 3),
                          "gpkts": round(w.n * 200 / el / 1e9, 2), **read_levels(d)}), flush=True)


if __name__ == "__main__":
    main()
