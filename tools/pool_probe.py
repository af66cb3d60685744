"""First-evaluation time per batch of the bench's distinct-scan pool, cold and warm.

For every batch of the pool (seeds b*8 .. b*8+7, as bench.py's rank 0) the
batch runs twice back to back with per-evaluation events (profiling level 2):
the first run meets the batch's map regions and scan buffers cold, the second
warm.  Cold >> warm: capacity (cache / TLB); cold ~ warm but batches differ:
the scans' own load (poses, distances to the surfaces).
usage: python tools/pool_probe.py [--batches 23] [--map-points 1000000]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))

import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=23)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--map-points", type=int, default=1_000_000)
    a = ap.parse_args()
    m = synth.cached_map(a.map_points)
    n = a.batches * a.batch
    scans = bench.gen_scans(100_000, range(n), min(16, bench.host_threads()))
    st0 = [synth.make_state(s) for s in range(n)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(s) for s in scans]
        ctx.set_profiling(2)
        work = (livo_amd.State * a.batch)()
        rows = []
        for b in range(a.batches):
            ini = (livo_amd.State * a.batch)(*[livo_amd.state_to_c(s) for s in st0[b * a.batch:(b + 1) * a.batch]])
            out = []
            for rep in range(3):
                C.memmove(work, ini, C.sizeof(ini))
                _, stats = ctx.iekf_update_batch(sids[b * a.batch:(b + 1) * a.batch], work, raw=True)
                tm = ctx.last_timings()
                out.append((tm["knn_ms"], tm["knn_points"] / max(tm["knn_queries"], 1),
                            tm["rematch_knn_ms"], sum(s.iterations for s in stats) / a.batch, tm["knn_replays"],
                            tm["plane_ms"]))
            rows.append(out)
            print(f"batch {b:2d}: first cold {out[0][0]:.4f} warm {out[1][0]:.4f} {out[2][0]:.4f} ms  "
                  f"pts/query {out[0][1]:.1f}  rematch {out[2][2]:.4f}  no-search {out[2][5]:.4f}  "
                  f"evals/scan {out[0][3]:.2f}  replays {out[2][4]}", flush=True)
        cold = sum(r[0][0] for r in rows) / len(rows)
        warm = sum(r[2][0] for r in rows) / len(rows)
        print(f"mean first evaluation: cold {cold:.4f} ms, warm {warm:.4f} ms")


if __name__ == "__main__":
    main()
