"""The IEKF on the incremental map (bench.py's ikd leg, sequential odometry):
per scan the update's evaluation times (profiling level 2) and, with the
LIVO_EVAL_PROF build (LIVO_LIB=.../evprof.so), the search statistics and the
flagged-query reasons of its evaluations.
usage: python tools/dyn_probe.py [--scans 8] [--passes 2]
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=8)
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(a.scans)]
    st0 = [synth.make_state(s) for s in range(a.scans)]
    prof = "evprof" in os.environ.get("LIVO_LIB", "")
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        L = ctx._L
        if prof:
            L.livo_debug_eval_stats.argtypes = [C.c_void_p]
            L.livo_debug_amb_reason.argtypes = [C.c_void_p]
            sbuf = (C.c_ulonglong * 24)()
            abuf = (C.c_ulonglong * 8)()
        for p in range(a.passes):
            for k in range(a.scans):
                sid = ctx.scan_upload(scans[k])
                ctx.set_profiling(2)
                if prof:
                    L.livo_debug_eval_stats(sbuf)
                    L.livo_debug_amb_reason(abuf)
                t = time.perf_counter()
                st, stats = ctx.iekf_update(sid, st0[k])
                dt = time.perf_counter() - t
                tm = ctx.last_timings()
                ctx.set_profiling(0)
                line = (f"pass {p} scan {k}: update {dt * 1e3:.3f} ms host, evals " +
                        " ".join(f"{x:.3f}" for x in tm["eval_ms"][:tm["n_evals"]]) +
                        f"  searched {tm['eval_searched'][:tm['n_evals']]}  pts/query "
                        f"{tm['knn_points'] / max(tm['knn_queries'], 1):.1f}  replays {tm['knn_replays']}")
                if prof:
                    L.livo_debug_eval_stats(sbuf)
                    L.livo_debug_amb_reason(abuf)
                    r = sbuf[16:24]
                    lanes = max(r[0], 1)
                    line += (f"  | first: ball-cert {r[1] / lanes:.3f} cell-run {r[2] / lanes:.3f} "
                             f"ball/lane {r[3] / lanes:.1f} cell/lane {r[5] / lanes:.1f}  flagged: unc {abuf[0]} "
                             f"C1 {abuf[1]} C1= {abuf[4]} gap {abuf[2]} eqx {abuf[3]}")
                print(line, flush=True)
                t = time.perf_counter()
                _, cnt = ctx.map_incremental(sid, st, filter_size_map=0.5)
                print(f"   map_incremental {(time.perf_counter() - t) * 1e3:.3f} ms  {cnt}", flush=True)
                ctx.scan_release(sid)


if __name__ == "__main__":
    main()
