"""Build variant libraries for on-GPU A/B runs (LIVO_LIB selects one).

usage: python tools/ab_build.py NAME [-DMACRO=VALUE ...] [ENV=VALUE ...]
Writes fast-livo-noted_amd/lib/variants/NAME.so: every source compiled with
the extra -D flags (the tuning macros of livo_internal.h and the kernel files).  Run A/B on one box, e.g.
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
        obj = os.path.join(vdir, name + "." + src + ".o")
        if not dev:
            # host objects too: some macros (LIVO_EVAL_BLOCK) size host-side buffers
            B._run([B.HIPCC, "-pthread"] + B.COMMON + ["-D__HIP_PLATFORM_AMD__"] + list(flags) +
                   ["-c", "-o", obj, os.path.join(B.CSRC, src)])
            objs.append(obj)
            continue
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
