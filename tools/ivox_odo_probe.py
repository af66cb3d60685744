"""iVox single-scan regime (the reference's shipped default: one scan per frame,
map_incremental after every scan): per-call times of livo_iekf_update and
livo_map_incremental, per iVox search kind.

usage: python tools/ivox_odo_probe.py [kinds] [scans]     kinds: comma list of auto,wave,team,thread
Each kind runs on a fresh context (map built, 2 passes over the scans: the
first warms the allocations, the second is timed).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))


def run(kind, m, scans, st0):
    import livo_amd
    if kind == "auto":
        os.environ.pop("LIVO_IVOX_KIND", None)
    else:
        os.environ["LIVO_IVOX_KIND"] = kind
    with livo_amd.Context(0, t_LI=livo_amd.synth.T_LI, max_iterations=4) as ctx:
        ctx.set_backend(livo_amd.BACKEND_IVOX)
        ctx.ivox_init()
        ctx.ivox_add_points(m)
        rows = []
        for rep in range(2):
            sids = [ctx.scan_upload(sc) for sc in scans]
            ctx.sync()
            t_upd = t_inc = 0.0
            t0 = time.perf_counter()
            for sid, s in zip(sids, st0):
                t1 = time.perf_counter()
                st, _ = ctx.iekf_update(sid, s)
                t2 = time.perf_counter()
                ctx.map_incremental(sid, st, filter_size_map=0.5)
                t3 = time.perf_counter()
                t_upd += t2 - t1
                t_inc += t3 - t2
            ctx.sync()
            el = time.perf_counter() - t0
            for sid in sids:
                ctx.scan_release(sid)
            rows.append((el, t_upd, t_inc))
        el, t_upd, t_inc = rows[-1]
        n = len(scans)
        print(f"kind {kind:6s}: {el / n * 1e3:.3f} ms/scan  iekf {t_upd / n * 1e3:.3f}  map_incremental "
              f"{t_inc / n * 1e3:.3f}  (cold pass {rows[0][0] / n * 1e3:.3f} ms/scan)", flush=True)


def main():
    import livo_amd
    from livo_amd import synth
    livo_amd.synth = synth
    kinds = (sys.argv[1] if len(sys.argv) > 1 else "auto,wave,team").split(",")
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(ns)]
    st0 = [synth.make_state(s) for s in range(ns)]
    for k in kinds:
        run(k, m, scans, st0)


if __name__ == "__main__":
    main()
