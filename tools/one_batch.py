"""One synchronous batch of 8 x 100k scans vs the 1M map (development tool: a
first look at a failing launch, e.g. under AMD_LOG_LEVEL)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402

m = synth.cached_map(1_000_000)
with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
    ctx.map_build(m)
    sids = [ctx.scan_upload(synth.make_scan(100_000, s)[0]) for s in range(8)]
    outs, stats = ctx.iekf_update_batch(sids, [synth.make_state(s) for s in range(8)])
    print("iterations", [s["iterations"] for s in stats])
