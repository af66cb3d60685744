"""The bench's batch of scan updates, for rocprofv3 --pmc passes (bench.py pmc_traffic).

Same map, scans, states and batch as bench.py's headline (synthetic, seeded);
a warm-up batch, then three batches: the profiled dispatches of the
first-evaluation k-NN kernel are those of the bench's roofline unit.
usage: python tools/knn_probe.py [--scan-points N] [--map-points M] [--batch B] [--steps K]
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
    a = ap.parse_args()
    m = synth.cached_map(a.map_points)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=a.max_iter) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(synth.make_scan(a.scan_points, s)[0]) for s in range(a.batch)]
        st0 = [synth.make_state(s) for s in range(a.batch)]
        for _ in range(1 + a.steps):
            ctx.iekf_update_batch(sids, st0)
    print("probe done", flush=True)


if __name__ == "__main__":
    main()
