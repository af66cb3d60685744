"""Upper-bound probe for batch pipelining: K host threads, each with its own
context (own map replica, own streams) and 8 scans, run the bench's headline
batch back to back; the device then holds K batches in flight.  Prints the
aggregate scan updates/s per K.  An experiment, not the product path.
usage: python tools/pipeline_probe.py [K ...]
"""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    ks = [int(x) for x in sys.argv[1:]] or [1, 2]
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(8)]
    st0 = [synth.make_state(s) for s in range(8)]
    ctxs = []
    for _ in range(max(ks)):
        ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
        ctx.map_build(m)
        sids = [ctx.scan_upload(s) for s in scans]
        init = (livo_amd.State * 8)(*[livo_amd.state_to_c(s) for s in st0])
        work = (livo_amd.State * 8)()
        ctxs.append((ctx, sids, init, work))

    def run(ci, steps, out):
        ctx, sids, init, work = ctxs[ci]
        for _ in range(steps):
            C.memmove(work, init, C.sizeof(init))
            ctx.iekf_update_batch(sids, work, raw=True)
        out[ci] = steps

    for k in ks:
        for ci in range(k):  # warm-up
            run(ci, 3, {})
        steps = 60
        out = {}
        th = [threading.Thread(target=run, args=(ci, steps, out)) for ci in range(k)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t
        print(f"K={k}: {k * steps * 8 / dt:.1f} scan updates/s ({dt / steps * 1e3:.3f} ms per round of K batches)",
              flush=True)
    for ctx, *_ in ctxs:
        ctx.close()


if __name__ == "__main__":
    main()
