"""Build the in-tree HIP library (gfx950) — used by __graft_entry__.build().

hipcc is driven directly (no CMake): the product is one shared library,
fast-livo-noted_amd/lib/liblivo_hip.so, exporting the C ABI of include/livo.h.
"""
from __future__ import annotations

import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "liblivo_hip.so")
OBJ_DIR = os.path.join(HERE, "build")

ARCH = os.environ.get("LIVO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: no FMA contraction, the reference runs x86-64 SSE2 (no FMA);
# f32 division / sqrt stay correctly rounded (HIP default, stated explicitly).
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
          "-Wall", "-Wno-unused-function"]
DEVICE = ["--offload-arch=" + ARCH, "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics"]

SOURCES = [
    ("livo_kernels.hip", True),
    ("ivox_kernels.hip", True),
    ("frontend_kernels.hip", True),
    ("vio_kernels.hip", True),
    ("ikd_incr_kernels.hip", True),
    ("prims.hip", True),
    ("livo_capi.cpp", False),
    ("map_build.cpp", False),
]


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError("build step failed: " + os.path.basename(cmd[-1]))
    return r


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(ROOT, "include", "livo.h")] + \
        [os.path.join(HERE, "host", f) for f in os.listdir(os.path.join(HERE, "host"))]
    newest = max(os.path.getmtime(d) for d in deps)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        return LIB
    objs, cmds = [], []
    for src, is_dev in SOURCES:
        obj = os.path.join(OBJ_DIR, src + ".o")
        cmd = [HIPCC] + COMMON + (DEVICE + ["-x", "hip"] if is_dev else ["-D__HIP_PLATFORM_AMD__"]) + \
              ["-c", "-o", obj, os.path.join(CSRC, src)]
        if not is_dev:
            cmd.insert(1, "-pthread")
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(obj)
    # one compiler process per source (a few CPUs: each hipcc holds ~1 GB)
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        list(ex.map(_run, cmds))
    cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-pthread", "-o", LIB + ".tmp"] + objs
    _run(cmd)
    os.replace(LIB + ".tmp", LIB)
    build_facade_demo(verbose)
    build_checks(verbose)
    return LIB


HOST = os.path.join(HERE, "host")
FACADE_DEMO = os.path.join(LIB_DIR, "facade_demo")


def build_facade_demo(verbose: bool = False) -> str:
    """The C++ facade (host/laser_mapping_gpu.hpp) driven by host/facade_demo.cpp, linked to the C ABI."""
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"), "-I" + HOST,
           os.path.join(HOST, "facade_demo.cpp"), "-L" + LIB_DIR, "-llivo_hip", "-Wl,-rpath,$ORIGIN",
           "-o", FACADE_DEMO]
    if verbose:
        print(" ".join(cmd))
    _run(cmd)
    return FACADE_DEMO




WAVE_CHECK = os.path.join(LIB_DIR, "wave_nth_check")


def build_checks(verbose: bool = False) -> str:
    """Device unit checks run by the -m gpu tests (built here, on the CPU, like the library)."""
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=" + ARCH, "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"),
           "-I" + CSRC, os.path.join(ROOT, "tests", "native", "wave_nth_check.hip"), "-o", WAVE_CHECK]
    if verbose:
        print(" ".join(cmd))
    _run(cmd)
    return WAVE_CHECK


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
