"""iVox single-scan regime (the reference's shipped default: one scan per frame,
map_incremental after every scan): per-call times of livo_iekf_update and
livo_map_incremental, per iVox search kind.

usage: python tools/ivox_odo_probe.py [kinds] [scans] [map]   kinds: comma list of auto,wave,team,thread
                                                              map: dense (default) | room
Each kind runs on a fresh context (map built, 2 passes over the scans: the
first warms the allocations, the second is timed).  room: the map bench.py's
ivox.odometry.mapped_room uses (the first scan voxel-downsampled at 0.5 m, grown
by 31 mapping scans at their true poses, each updated then merged).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))


def build_room(ctx, ns):
    import numpy as np
    from livo_amd import synth
    seeds = list(range(1000, 1032))
    mscans = [synth.make_scan(100_000, s)[0] for s in seeds]
    R0, p0, _ = synth.true_pose(seeds[0])
    w0 = (mscans[0].astype(np.float64) @ synth.R_LI.T + synth.T_LI) @ R0.T + p0
    _, first = np.unique(np.floor(w0 / 0.5).astype(np.int64), axis=0, return_index=True)
    ctx.ivox_add_points(np.ascontiguousarray(w0[np.sort(first)], dtype=np.float32))
    for sd, sc in zip(seeds[1:], mscans[1:]):
        sid = ctx.scan_upload(sc)
        stm, _ = ctx.iekf_update(sid, synth.make_state(sd, rot_deg=0.0, trans_m=0.0))
        ctx.map_incremental(sid, stm, filter_size_map=0.5)
        ctx.scan_release(sid)
    print("room map:", ctx.ivox_info(), flush=True)


def run(kind, m, scans, st0):
    import livo_amd
    if kind == "auto":
        os.environ.pop("LIVO_IVOX_KIND", None)
    else:
        os.environ["LIVO_IVOX_KIND"] = kind
    with livo_amd.Context(0, t_LI=livo_amd.synth.T_LI, max_iterations=4) as ctx:
        ctx.set_backend(livo_amd.BACKEND_IVOX)
        ctx.ivox_init()
        if m is None:
            build_room(ctx, len(scans))
        else:
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
    room = len(sys.argv) > 3 and sys.argv[3] == "room"
    m = None if room else synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(ns)]
    st0 = [synth.make_state(s) for s in range(ns)]
    for k in kinds:
        run(k, m, scans, st0)


if __name__ == "__main__":
    main()
