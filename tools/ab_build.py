"""Build variant libraries for on-GPU A/B runs (LIVO_LIB selects one).

usage: python tools/ab_build.py NAME [-DMACRO=VALUE ...] [ENV=VALUE ...]
Writes fast-livo-noted_amd/lib/variants/NAME.so: every device source compiled
with the extra -D flags (the tuning macros of livo_internal.h and the kernel
files), linked with the host objects of the regular build.  Run A/B on one box, e.g.
  LIVO_LIB=fast-livo-noted_amd/lib/variants/NAME.so python bench.py
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import build as B  # noqa: E402


def main(name, *flags):
    B.build()
    vdir = os.path.join(B.LIB_DIR, "variants")
    os.makedirs(vdir, exist_ok=True)
    objs = []
    for src, dev in B.SOURCES:
        if not dev:
            objs.append(os.path.join(B.OBJ_DIR, src + ".o"))
            continue
        obj = os.path.join(vdir, name + "." + src + ".o")
        B._run([B.HIPCC] + B.COMMON + B.DEVICE + ["-x", "hip"] + list(flags) + ["-c", "-o", obj, os.path.join(B.CSRC, src)])
        objs.append(obj)
    out = os.path.join(vdir, name + ".so")
    B._run([B.HIPCC, "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-pthread", "-o", out] + objs)
    for o in objs:
        if o.startswith(vdir):
            os.remove(o)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
