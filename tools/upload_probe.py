"""Scan upload timings (development tool): livo_scan_upload_batch_async of 8 x
100k-point scans (1M map), pageable and page-locked, alone and inside the
pipelined farm, with the host time of each call.

    python tools/upload_probe.py [steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    m = synth.cached_map(1_000_000)
    align = "--unaligned" not in sys.argv
    scans = [np.ascontiguousarray(synth.make_scan(100_000, s)[0][:, :3], np.float32) for s in range(32)]
    if align:
        scans = [livo_amd.page_aligned_copy(x) for x in scans]
    print("page-aligned arrays" if align else "arrays as numpy allocates them")
    states = [synth.make_state(s) for s in range(32)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        for pinned in (False, True):
            if pinned:
                for x in scans:
                    ctx.host_register(x)
            for rep in range(3):
                ctx.sync()
                t0 = time.perf_counter()
                ids = ctx.scan_upload_batch_async(scans[:8])
                t1 = time.perf_counter()
                ctx.sync()
                t2 = time.perf_counter()
                for sid in ids:
                    ctx.scan_release(sid)
                print(f"{'pinned' if pinned else 'pageable':8s} rep {rep}: batch upload host {1e3 * (t1 - t0):.3f} ms, "
                      f"to device done {1e3 * (t2 - t0):.3f} ms")
            # the farm: uploads two batches ahead
            for warm, n in ((True, 4), (False, steps)):
                ctx.sync()
                t0 = time.perf_counter()
                pend, ahead, nxt = [], [], 0
                t_up = t_wait = t_sub = 0.0
                for k in range(n):
                    while len(ahead) < 2 and nxt < n:
                        ta = time.perf_counter()
                        ahead.append((nxt, ctx.scan_upload_batch_async(scans[8 * (nxt % 4): 8 * (nxt % 4) + 8])))
                        t_up += time.perf_counter() - ta
                        nxt += 1
                    if len(pend) == 2:
                        t, ids = pend.pop(0)
                        ta = time.perf_counter()
                        ctx.iekf_update_batch_wait(t, 8)
                        t_wait += time.perf_counter() - ta
                        for sid in ids:
                            ctx.scan_release(sid)
                    b, ids = ahead.pop(0)
                    ta = time.perf_counter()
                    pend.append((ctx.iekf_update_batch_submit(ids, states[8 * (b % 4): 8 * (b % 4) + 8]), ids))
                    t_sub += time.perf_counter() - ta
                for t, ids in pend:
                    ctx.iekf_update_batch_wait(t, 8)
                    for sid in ids:
                        ctx.scan_release(sid)
                ctx.sync()
                el = time.perf_counter() - t0
                if not warm:
                    print(f"farm with uploads ({'pinned' if pinned else 'pageable'}): {1e3 * el / n:.4f} ms/step "
                          f"({8 * n / el:.0f} updates/s); host per step: uploads {1e3 * t_up / n:.4f}, submits "
                          f"{1e3 * t_sub / n:.4f}, waits {1e3 * t_wait / n:.4f} ms")
            if pinned:
                for x in scans:
                    ctx.host_unregister(x)


if __name__ == "__main__":
    main()
