"""Build variant libraries for on-GPU A/B runs (LIVO_LIB selects one).

usage: python tools/ab_build.py NAME [-DMACRO=VALUE ...] [ENV=VALUE ...]
Writes fast-livo-noted_amd/lib/variants/NAME.so: livo_kernels.hip compiled with
the extra -D flags (the tuning macros of livo_internal.h / livo_kernels.hip),
linked with the host objects of the regular build.  Run A/B on one box, e.g.
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
    obj = os.path.join(vdir, name + ".o")
    cmd = [B.HIPCC] + B.COMMON + B.DEVICE + ["-x", "hip"] + list(flags) + \
        ["-c", "-o", obj, os.path.join(B.CSRC, "livo_kernels.hip")]
    B._run(cmd)
    host = [os.path.join(B.OBJ_DIR, s + ".o") for s, dev in B.SOURCES if not dev]
    out = os.path.join(vdir, name + ".so")
    B._run([B.HIPCC, "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-pthread", "-o", out, obj] + host)
    os.remove(obj)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
