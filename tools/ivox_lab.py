"""iVox k-NN lab: device time of the batched first search on config-2 shapes.

usage: python tools/ivox_lab.py [map_points] [scan_points] [batch] [resolution]
Prints the first-evaluation k-NN time (HIP events, profiling level 2), the
other stages, and the ivox_knn call rate; for A/B runs of kernel variants
(LIVO_LIB points at an alternative build).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402


def main(M=1_000_000, N=100_000, B=8, res=0.2):
    import livo_amd
    from livo_amd import synth
    M, N, B, res = int(M), int(N), int(B), float(res)
    m = synth.cached_map(M)
    scans = [synth.make_scan(N, s)[0] for s in range(B)]
    st0 = [synth.make_state(s) for s in range(B)]
    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    ctx.set_backend(livo_amd.BACKEND_IVOX)
    ctx.ivox_init(resolution=res)
    ctx.ivox_add_points(m)
    info = ctx.ivox_info()
    sids = [ctx.scan_upload(s) for s in scans]
    init = (livo_amd.State * B)(*[livo_amd.state_to_c(s) for s in st0])
    work = (livo_amd.State * B)()
    for _ in range(3):
        C.memmove(work, init, C.sizeof(init))
        ctx.iekf_update_batch(sids, work, raw=True)
    ctx.set_profiling(2)
    acc = np.zeros(3)
    R = 10
    for _ in range(R):
        C.memmove(work, init, C.sizeof(init))
        ctx.iekf_update_batch(sids, work, raw=True)
        t = ctx.last_timings()
        acc += [t["knn_ms"], t["rematch_knn_ms"], t["plane_ms"]]
    ctx.set_profiling(0)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(R):
        C.memmove(work, init, C.sizeof(init))
        ctx.iekf_update_batch(sids, work, raw=True)
    ctx.sync()
    el = (time.perf_counter() - t0) / R
    q = np.concatenate([((s.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(np.float32)
                        for s, st in zip(scans, st0)])
    ctx.ivox_knn(q[:1000])
    t0 = time.perf_counter()
    _, _, cnt = ctx.ivox_knn(q)
    tk = time.perf_counter() - t0
    print(f"map {M} pts, {info['num_grids']} grids (max {info['max_grid_points']}), {B}x{N} scans, res {res}")
    print(f"knn_first {acc[0] / R:.3f} ms  rematch(sum) {acc[1] / R:.3f} ms  plane+solve(sum) {acc[2] / R:.3f} ms")
    print(f"batch {el * 1e3:.3f} ms = {B / el:.1f} scan updates/s")
    print(f"ivox_knn host call over {len(q)} queries: {tk * 1e3:.1f} ms (incl. transfers); found 5: "
          f"{(cnt == 5).mean():.3f}, none: {(cnt == -1).mean():.3f}")
    ctx.close()


if __name__ == "__main__":
    main(*sys.argv[1:])
