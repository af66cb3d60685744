"""The bench's batch of scan updates, for rocprofv3 --pmc passes (bench.py pmc_traffic).

Same map, scans, states and batch as bench.py's headline (synthetic, seeded);
a warm-up batch, then three batches: the profiled dispatches of the
first-evaluation k-NN kernel are those of the bench's roofline unit.
--config5: the bench's config-5 leg instead (10M-point map, 8 scans per batch,
each the device VoxelGrid at leaf 0.05 of a raw still frame).
usage: python tools/knn_probe.py [--scan-points N] [--map-points M] [--batch B] [--steps K] [--config5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))

import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scan-points", type=int, default=100_000)
    ap.add_argument("--map-points", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-iter", type=int, default=4)
    ap.add_argument("--seed0", type=int, default=0, help="first scan seed")
    ap.add_argument("--config5", action="store_true")
    ap.add_argument("--fresh", action="store_true", help="every batch other scans (the bench's distinct-scan pool)")
    a = ap.parse_args()
    if a.config5:
        m = synth.cached_map(10_000_000)
    else:
        m = synth.cached_map(a.map_points)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=a.max_iter) as ctx:
        ctx.map_build(m)
        del m
        seeds = [a.seed0 + s for s in range(a.batch)]
        if a.config5:  # bench.py's config5 leg: scan seeds 1000 + j
            sids = []
            for s in seeds:
                raw, poses, Re, pe = synth.make_config5_frame(1000 + s)
                sids.append(ctx.scan_preprocess(raw, poses, Re, pe, leaf_size=synth.CONFIG5_LEAF)[0])
            st0 = [synth.make_state(1000 + s) for s in seeds]
        elif a.fresh:
            nb = 1 + a.steps
            seeds = [a.seed0 + s for s in range(nb * a.batch)]
            sids = [ctx.scan_upload(synth.make_scan(a.scan_points, s)[0]) for s in seeds]
            st0 = [synth.make_state(s) for s in seeds]
            for b in range(nb):
                ctx.iekf_update_batch(sids[b * a.batch:(b + 1) * a.batch], st0[b * a.batch:(b + 1) * a.batch])
            print("probe done", flush=True)
            return
        else:
            sids = [ctx.scan_upload(synth.make_scan(a.scan_points, s)[0]) for s in seeds]
            st0 = [synth.make_state(s) for s in seeds]
        for _ in range(1 + a.steps):
            ctx.iekf_update_batch(sids, st0)
    print("probe done", flush=True)


if __name__ == "__main__":
    main()
