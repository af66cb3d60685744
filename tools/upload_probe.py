"""Scan upload timings (development tool): livo_scan_upload vs livo_scan_upload_async
on 100k-point scans (1M map), alone and inside the pipelined farm.

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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(32)]
    states = [synth.make_state(s) for s in range(32)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        for mode in ("sync", "async"):
            up = ctx.scan_upload if mode == "sync" else ctx.scan_upload_async
            for rep in range(3):
                ctx.sync()
                t0 = time.perf_counter()
                ids = [up(x) for x in scans[:8]]
                t1 = time.perf_counter()
                ctx.sync()
                t2 = time.perf_counter()
                for sid in ids:
                    ctx.scan_release(sid)
                t3 = time.perf_counter()
                print(f"{mode:5s} rep {rep}: 8 uploads host {1e3 * (t1 - t0):.3f} ms, to device done "
                      f"{1e3 * (t2 - t0):.3f} ms, releases {1e3 * (t3 - t2):.3f} ms")
        # the farm: resident scans, then with the uploads inside
        res = [ctx.scan_upload(x) for x in scans[:16]]
        batches = [(res[:8], states[:8]), (res[8:16], states[8:16])]
        for k in range(4):
            ctx.iekf_update_batch(*batches[k % 2])
        ctx.sync()
        t0 = time.perf_counter()
        pend = []
        for k in range(steps):
            if len(pend) == 2:
                ctx.iekf_update_batch_wait(pend.pop(0), 8)
            pend.append(ctx.iekf_update_batch_submit(*batches[k % 2]))
        for t in pend:
            ctx.iekf_update_batch_wait(t, 8)
        ctx.sync()
        t_res = time.perf_counter() - t0
        for sid in res:
            ctx.scan_release(sid)
        t0 = time.perf_counter()
        pend, ahead, nxt = [], [], 0
        t_up = t_wait = t_rel = 0.0
        for k in range(steps):
            while len(ahead) < 2 and nxt < steps:
                ta = time.perf_counter()
                ahead.append((nxt, [ctx.scan_upload_async(x) for x in scans[8 * (nxt % 4): 8 * (nxt % 4) + 8]]))
                t_up += time.perf_counter() - ta
                nxt += 1
            if len(pend) == 2:
                t, ids = pend.pop(0)
                ta = time.perf_counter()
                ctx.iekf_update_batch_wait(t, 8)
                tb = time.perf_counter()
                for sid in ids:
                    ctx.scan_release(sid)
                t_wait += tb - ta
                t_rel += time.perf_counter() - tb
            b, ids = ahead.pop(0)
            pend.append((ctx.iekf_update_batch_submit(ids, states[8 * (b % 4): 8 * (b % 4) + 8]), ids))
        for t, ids in pend:
            ctx.iekf_update_batch_wait(t, 8)
            for sid in ids:
                ctx.scan_release(sid)
        ctx.sync()
        t_upl = time.perf_counter() - t0
        print(f"farm resident: {1e3 * t_res / steps:.4f} ms/step ({8 * steps / t_res:.0f} updates/s)")
        print(f"farm with uploads: {1e3 * t_upl / steps:.4f} ms/step ({8 * steps / t_upl:.0f} updates/s); host: "
              f"uploads {1e3 * t_up / steps:.4f}, waits {1e3 * t_wait / steps:.4f}, releases "
              f"{1e3 * t_rel / steps:.4f} ms/step")


if __name__ == "__main__":
    main()
