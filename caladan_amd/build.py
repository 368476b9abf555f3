"""Build the product shared library libgclassify.so in-tree for gfx950.

hipcc compiles the HIP kernels + C ABI (csrc/gclassify.hip); gcc compiles the
host-side C (csrc/gcl_host.c); hipcc links both into caladan_amd/libgclassify.so.
The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgclassify.so")
OBJ = os.path.join(HERE, "_obj")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GCL_OFFLOAD_ARCH", "gfx950")

SOURCES_HIP = ["gclassify.hip"]
SOURCES_C = ["gcl_host.c", "gcl_pcap.c"]
DEPS = ["gcl_device.h", "../../include/gclassify.h", "../../include/gcl_host.h",
        "../../include/gcl_pcap.h"]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _stale(target, inputs):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(i) > t for i in inputs)


def build(force=False, verbose_resources=False):
    os.makedirs(OBJ, exist_ok=True)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.abspath(__file__)]
    objs = []
    for src in SOURCES_HIP:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        if force or _stale(o, [s] + deps):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-Wall", "-Wno-unused-function", "-c", s, "-o", o]
            if verbose_resources:
                cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            _run(cmd)
        objs.append(o)
    for src in SOURCES_C:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        if force or _stale(o, [s] + deps):
            _run(["gcc", "-std=gnu11", "-O3", "-fPIC", "-Wall", "-Wextra",
                  "-Wno-unused-parameter", "-c", s, "-o", o])
        objs.append(o)
    if force or _stale(OUT, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs + ["-lm"])
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resources="--resources" in sys.argv)
