"""Build the product shared libraries in-tree for gfx950.

hipcc compiles the HIP kernels + C ABI (csrc/gcl_*.hip: the context, the
batch kernels, the persistent rx loop, the transports and allocation, the
generator); gcc compiles the host-side C (csrc/gcl_host.c, csrc/gcl_pcap.c);
hipcc links them into caladan_amd/libgclassify.so.  The multi-GPU group (csrc/gcl_group.hip,
include/gcl_group.h) is its own library, caladan_amd/libgclgroup.so, linked
against libgclassify.so and RCCL, so that a single-GPU dataplane does not
load RCCL.  The .so files are git-ignored but travel to the GPU box with the
gpurun snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgclassify.so")
OUT_GROUP = os.path.join(HERE, "libgclgroup.so")
OBJ = os.path.join(HERE, "_obj")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GCL_OFFLOAD_ARCH", "gfx950")

SOURCES_HIP = ["gcl_ctx.hip", "gcl_batch.hip", "gcl_loop.hip", "gcl_xfer.hip", "gcl_gen.hip"]
SOURCES_C = ["gcl_host.c", "gcl_pcap.c"]
DEPS = ["gcl_device.h", "gcl_kern.h", "gcl_ctx.h", "../../include/gclassify.h", "../../include/gcl_host.h",
        "../../include/gcl_pcap.h"]
SOURCE_GROUP = "gcl_group.hip"
DEPS_GROUP = ["../../include/gclassify.h", "../../include/gcl_group.h"]


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
    objs, cmds = [], []
    for src in SOURCES_HIP:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        if force or _stale(o, [s] + deps):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-Wall", "-Wno-unused-function", "-c", s, "-o", o]
            if verbose_resources:
                cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            cmds.append(cmd)
        objs.append(o)
    # the translation units are independent: compile them side by side
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(cmds), 4) or 1) as ex:
        list(ex.map(_run, cmds))
    for src in SOURCES_C:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        if force or _stale(o, [s] + deps):
            _run(["gcc", "-std=gnu11", "-O3", "-fPIC", "-Wall", "-Wextra",
                  "-Wno-unused-parameter", "-c", s, "-o", o])
        objs.append(o)
    if force or _stale(OUT, objs):
        # only the C ABI (gcl_*) is exported; the translation units' shared
        # helpers (namespace gclk) stay internal to the library
        vs = os.path.join(OBJ, "exports.map")
        with open(vs, "w") as f:
            f.write("{ global: gcl_*; local: *; };\n")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs +
             ["-lm", "-Wl,--version-script=" + vs])
    build_group(force)
    return OUT


def build_group(force=False):
    """libgclgroup.so: the multi-GPU group over libgclassify.so + RCCL."""
    s = os.path.join(CSRC, SOURCE_GROUP)
    o = os.path.join(OBJ, SOURCE_GROUP + ".o")
    deps = [s, os.path.abspath(__file__)] + [os.path.join(CSRC, d) for d in DEPS_GROUP]
    if force or _stale(o, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
              "-c", s, "-o", o])
    if force or _stale(OUT_GROUP, [o, OUT]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT_GROUP, o,
              "-L" + HERE, "-lgclassify", "-L/opt/rocm/lib", "-lrccl",
              "-Wl,-rpath,$ORIGIN", "-Wl,--no-undefined"])
    return OUT_GROUP


SANITIZE_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                  "-fno-omit-frame-pointer", "-static-libasan", "-g", "-O1"]


def build_sanitized(out_dir=None):
    """Host-only CPU build of the C that parses untrusted input -- the pcap
    loader (csrc/gcl_pcap.c), the verdict post-pass (csrc/gcl_host.c) and the
    oracle's classifier (oracle/orc.c, test infrastructure) -- under ASan +
    UBSan, linked into the fuzz driver tests/fuzz/host_fuzz.c.  No HIP code is
    compiled: GPU code is never built with sanitizers here.  Returns the
    driver's path."""
    out_dir = out_dir or os.path.join(ROOT, "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "host_fuzz")
    srcs = [os.path.join(ROOT, "tests", "fuzz", "host_fuzz.c"), os.path.join(CSRC, "gcl_host.c"),
            os.path.join(CSRC, "gcl_pcap.c"), os.path.join(ROOT, "oracle", "orc.c")]
    if _stale(exe, srcs + [os.path.join(CSRC, d) for d in DEPS]):
        _run(["gcc", "-std=gnu11", "-Wall", "-Wno-unused-parameter", *SANITIZE_FLAGS,
              "-o", exe, *srcs, "-lm", "-lpthread"])
    return exe


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        print(build_sanitized())
    else:
        build(force="--force" in sys.argv, verbose_resources="--resources" in sys.argv)
