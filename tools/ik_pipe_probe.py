"""IKFoM farm probe (development tool): synchronous batches vs two batches in
flight (livo_ikfom_update_batch_submit / _wait) on 8 x 100k scans, host times.

    python tools/ik_pipe_probe.py [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    m = synth.cached_map(1_000_000)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(synth.make_scan(100_000, s)[0]) for s in range(16)]
        sts = [synth.make_ikfom_state(s) for s in range(16)]
        sets = [(sids[:8], sts[:8]), (sids[8:], sts[8:])]
        for _ in range(2):
            ctx.ikfom_update_batch(*sets[0])
        ctx.sync()
        t0 = time.perf_counter()
        for k in range(steps):
            ctx.ikfom_update_batch(*sets[k % 2])
        ctx.sync()
        print(f"sync: {1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step")
        for rep in range(2):
            ctx.sync()
            t0 = time.perf_counter()
            pend, ts, tw = [], 0.0, 0.0
            for k in range(steps):
                if len(pend) == 2:
                    a = time.perf_counter()
                    ctx.ikfom_update_batch_wait(pend.pop(0), 8)
                    tw += time.perf_counter() - a
                a = time.perf_counter()
                pend.append(ctx.ikfom_update_batch_submit(*sets[k % 2]))
                ts += time.perf_counter() - a
            for t in pend:
                ctx.ikfom_update_batch_wait(t, 8)
            ctx.sync()
            el = time.perf_counter() - t0
            print(f"pipelined rep {rep}: {1e3 * el / steps:.3f} ms/step; host submit {1e3 * ts / steps:.3f}, "
                  f"wait {1e3 * tw / steps:.3f} ms/step")


if __name__ == "__main__":
    main()
