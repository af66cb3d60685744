"""Drop-in regime (one scan per call, the reference's boundary hands host points
every frame, laser_mapping.cpp:129-131): host time per call of livo_scan_upload,
livo_iekf_update and livo_scan_release, cold (first pass: buffer allocation)
and warm (later passes: released buffers reused).

usage: python tools/dropin_probe.py [passes] [scans]
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))


def main():
    import livo_amd
    from livo_amd import synth
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(ns)]
    states = [synth.make_state(s) for s in range(ns)]
    pinned = [np.ascontiguousarray(s[:, :3], np.float32) for s in scans]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        for mode in ("pageable", "page-locked"):
            arrs = scans if mode == "pageable" else pinned
            if mode == "page-locked":
                for a in pinned:
                    ctx.host_register(a)
            for p in range(passes):
                tu = tk = tr = 0.0
                ctx.sync()
                t0 = time.perf_counter()
                for k in range(ns):
                    t1 = time.perf_counter()
                    sid = ctx.scan_upload(arrs[k])
                    t2 = time.perf_counter()
                    ctx.iekf_update(sid, states[k])
                    t3 = time.perf_counter()
                    ctx.scan_release(sid)
                    t4 = time.perf_counter()
                    tu += t2 - t1
                    tk += t3 - t2
                    tr += t4 - t3
                ctx.sync()
                el = time.perf_counter() - t0
                print(f"{mode:11s} pass {p}: {el / ns * 1e3:.3f} ms/scan  upload {tu / ns * 1e3:.3f}  update "
                      f"{tk / ns * 1e3:.3f}  release {tr / ns * 1e3:.3f}", flush=True)
            if mode == "page-locked":
                for a in pinned:
                    ctx.host_unregister(a)


if __name__ == "__main__":
    main()
