"""Block timeline of the fused evaluation kernel (k_iekf_eval) for one batch.

Build the profiling variant first:  python tools/ab_build.py evprof -DLIVO_EVAL_PROF
then on the GPU box:
    LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so LIVO_STREAM_GROUPS=1 python tools/eval_timeline.py [--config5]
Thread 0 of every block records s_memtime (shader cycles) at its start and at
its end; per evaluation this prints the span, block durations (median / mean /
p90 / max), the mean number of blocks in flight (sum of durations / span) and
how much of the span is left after 90% of the blocks have ended (the tail).
One stream group, so blockIdx is unique within a launch.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402

MAX_EVALS, TL_BLOCKS = 16, 4096  # LIVO_MAX_EVALS, kTlBlocks


def main():
    config5 = "--config5" in sys.argv
    seed0 = int(sys.argv[sys.argv.index("--seed0") + 1]) if "--seed0" in sys.argv else 0  # first scan seed (config 2)
    m = synth.cached_map(10_000_000 if config5 else 1_000_000)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        if config5:
            sids = []
            for s in range(8):
                raw, poses, Re, pe = synth.make_config5_frame(1000 + s)
                sids.append(ctx.scan_preprocess(raw, poses, Re, pe, leaf_size=synth.CONFIG5_LEAF)[0])
            st0 = [synth.make_state(1000 + s) for s in range(8)]
        else:
            sids = [ctx.scan_upload(synth.make_scan(100_000, seed0 + s)[0]) for s in range(8)]
            st0 = [synth.make_state(seed0 + s) for s in range(8)]
        L = ctx._L
        L.livo_debug_eval_timeline.argtypes = [C.c_void_p, C.c_int64]
        buf = np.zeros((MAX_EVALS, TL_BLOCKS, 2), np.uint64)
        for _ in range(3):
            ctx.iekf_update_batch(sids, st0)
        ctx.set_profiling(2)
        ctx.iekf_update_batch(sids, st0)
        tm = ctx.last_timings()
        assert L.livo_debug_eval_timeline(buf.ctypes.data, buf.nbytes) == 0
    ms = tm.get("eval_ms", [])
    for e in range(MAX_EVALS):
        t = buf[e]
        ok = t[:, 1] > 0
        if not ok.any():
            continue
        st, en = t[ok, 0].astype(np.int64), t[ok, 1].astype(np.int64)
        t0 = st.min()
        span = en.max() - t0
        dur = en - st
        end_sorted = np.sort(en - t0)
        p90_end = end_sorted[int(0.9 * (len(end_sorted) - 1))]
        clk = f"  {span / (ms[e] * 1e3):.0f} cycles/us by the events" if e < len(ms) and ms[e] > 0 else ""
        print(f"eval {e}: blocks {ok.sum()}  span {span / 1e3:.1f} kcyc{clk}  block dur median "
              f"{np.median(dur) / 1e3:.1f} mean {dur.mean() / 1e3:.1f} p90 {np.percentile(dur, 90) / 1e3:.1f} "
              f"max {dur.max() / 1e3:.1f} kcyc  in flight {dur.sum() / span:.0f}  tail after 90% of blocks "
              f"{(span - p90_end) / span:.2f} of the span  last start {(st.max() - t0) / span:.2f}")
        if "--top" in sys.argv:  # the longest blocks: launch index, start and duration
            idx = np.nonzero(ok)[0]
            for k in np.argsort(-dur)[:8]:
                print(f"    block {idx[k]}: start {(st[k] - t0) / 1e3:.1f} dur {dur[k] / 1e3:.1f} kcyc")


if __name__ == "__main__":
    main()
