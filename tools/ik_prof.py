"""Phase marks of k_solve_ik (the IKFoM solve) on the bench's 8-scan batch.

Build the profiling variant first:  python tools/ab_build.py ikprof -DLIVO_SOLVE_PROF
then on the GPU box:  LIVO_LIB=fast-livo-noted_amd/lib/variants/ikprof.so python tools/ik_prof.py
Marks (lane 0 of the wave that passes them, s_memtime): 0 start, 1 partials merged
per wave, 2 waves merged; on the last wave beside them (ik_prep) 3 boxminus + P copy,
4 SO3/S2 corrections, 5 (P/R)^-1; then 6 P_temp^-1, 7 K_h/K_x,
8 dx_, boxplus and control, 9 covariance (stopping evaluations only).
Development tool, not the product.
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
        L = ctx._L
        L.livo_debug_solve_prof.argtypes = [C.c_void_p]
        buf = (C.c_ulonglong * (256 * 16))()
        ik0 = [synth.make_ikfom_state(s) for s in range(8)]
        for rep in range(3):
            ctx.ikfom_update_batch(sids, [dict(x) for x in ik0])
            assert L.livo_debug_solve_prof(buf) == 0
            for b in range(8):
                r = buf[16 * b: 16 * b + 16]
                marks = [r[k] for k in range(10)]
                if not marks[0] or marks[0] == 2**64 - 1:
                    continue
                off = {k: marks[k] - marks[0] for k in range(1, 10) if marks[k] and marks[k] >= marks[0]
                       and marks[k] - marks[0] < 10**7}
                print(f"rep {rep} block {b}: cycles from mark 0: {off}")


if __name__ == "__main__":
    main()
