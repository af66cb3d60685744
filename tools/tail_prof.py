"""Tail and solve phases of the fused evaluation (tools/ab_build.py tailprof -DLIVO_TAIL_PROF):
only the scan's last block takes marks (a few atomics per evaluation), so the
kernel runs unperturbed, unlike the per-block phase marks of LIVO_EVAL_PROF.

    LIVO_LIB=fast-livo-noted_amd/lib/variants/tailprof.so python tools/tail_prof.py [--groups N]
Prints the s_memtime clock, the per-evaluation windows of 10 synchronous
batches (8 x 100k scans, 1M map) and, per evaluation kind, the last block's
reduction / solve / slot write and the solve's phases (us at the measured clock).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    m = synth.cached_map(1_000_000)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(synth.make_scan(100_000, s)[0]) for s in range(8)]
        st0 = [synth.make_state(s) for s in range(8)]
        L = ctx._L
        mhz = C.c_double(0.0)
        L.livo_debug_clock.argtypes = [C.c_void_p]
        assert L.livo_debug_clock(C.byref(mhz)) == 0
        L.livo_debug_tail_prof.argtypes = [C.c_void_p]
        tbuf = (C.c_ulonglong * 72)()
        ctx.iekf_update_batch(sids, st0)
        ctx.set_profiling(2)
        wins = []
        for _ in range(5):
            ctx.iekf_update_batch(sids, st0)
            wins.append(ctx.last_timings()["eval_ms"])
        ctx.set_profiling(0)
        L.livo_debug_tail_prof(tbuf)  # reset
        steps = 10
        for _ in range(steps):
            ctx.iekf_update_batch(sids, st0)
        assert L.livo_debug_tail_prof(tbuf) == 0
    us = 1.0 / mhz.value
    print(f"s_memtime clock {mhz.value:.0f} MHz")
    n = min(len(w) for w in wins)
    print("per-evaluation windows (us, mean of 5 synchronous batches, max over groups):",
          [round(1e3 * sum(w[e] for w in wins) / len(wins), 1) for e in range(n)])
    # factored path (cov_ok): C, T = C L, Q + LDL^T, w / u (incl. the wait for vec), y, sol; LU path: C, M, LU, ...
    names = ("C", "T|M", "Q+LDL|LU", "w,u|Minv+w", "y|K6", "sol|G6+sol", "boxplus+ctrl", "stores+cov")
    for s, name in ((2, "first-search"), (1, "rematch"), (0, "no-search")):
        r = tbuf[8 * s: 8 * s + 8]
        nb, nl = max(r[0], 1), max(r[5], 1)
        print(f"{name:12s}: bfly+ticket {r[1] / nb * us:6.2f} us/block; last block ({r[5]}): partial reduction "
              f"{r[2] / nl * us:6.2f}  solve {r[3] / nl * us:6.2f}  slot write {r[4] / nl * us:6.2f} us")
        ph = tbuf[24 + 16 * s: 24 + 16 * s + 16]
        print("    solve: " + "  ".join(f"{k} {v / nl * us:.2f}" for k, v in zip(names, ph)) + " us")
        if ph[8] or ph[9]:  # LIVO_TAIL_TWICE: the same T / Q code timed cold (first pass) and warm (second)
            print(f"    I-cache probe: T cold {ph[8] / nl * us:.2f} warm {ph[1] / nl * us:.2f} us;  Q cold "
                  f"{ph[9] / nl * us:.2f} us")


if __name__ == "__main__":
    main()
