"""Per-frame device pipeline lab (raw frame -> preprocess -> IEKF (iVox) -> map_incremental).

usage: python tools/pipeline_lab.py [scan_points] [frames] [map_points]
Host-timed stages per frame; run under `rocprofv3 --kernel-trace --stats` for
the kernel breakdown.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))


def main(N=100_000, F=8, M=1_000_000):
    import livo_amd
    from livo_amd import synth
    N, F, M = int(N), int(F), int(M)
    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    ctx.set_backend(livo_amd.BACKEND_IVOX)
    ctx.ivox_init()
    ctx.ivox_add_points(synth.cached_map(M))
    raws = [synth.make_raw_scan(N, s) for s in range(F)]
    sts = [synth.make_state(s) for s in range(F)]
    prev = None
    for rep in range(3):
        acc = [0.0, 0.0, 0.0]
        for (raw, poses, Re, pe), s in zip(raws, sts):
            t1 = time.perf_counter()
            sid, _, down = ctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.5)
            t2 = time.perf_counter()
            if prev is not None:
                ctx.scan_inherit_neighbors(sid, prev)
                ctx.scan_release(prev)
            st, stats = ctx.iekf_update(sid, s)
            t3 = time.perf_counter()
            ctx.map_incremental(sid, st, filter_size_map=0.5)
            t4 = time.perf_counter()
            acc[0] += t2 - t1
            acc[1] += t3 - t2
            acc[2] += t4 - t3
            prev = sid
        print(f"rep {rep}: preprocess {acc[0] / F * 1e3:.3f} ms, iekf {acc[1] / F * 1e3:.3f} ms "
              f"({len(down)} pts, {stats['iterations']} evals), map_incremental {acc[2] / F * 1e3:.3f} ms")
    ctx.scan_release(prev)
    ctx.close()


if __name__ == "__main__":
    main(*sys.argv[1:])
