"""Per-phase block time of the fused evaluation kernel (k_iekf_eval) on the bench's batch.

Build the profiling variant first:  python tools/ab_build.py evprof -DLIVO_EVAL_PROF
then on the GPU box:  LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so python tools/eval_prof.py [--config5]
Phases (thread 0 of each block, s_memtime cycles): 1 build_tile, 2 search + tie replay,
3 plane pass (hshare_point), 4 block reduction + ticket (+ the last block's solve).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import livo_amd  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    config5 = "--config5" in sys.argv  # 10M map, the bench's VoxelGrid scans
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
        L.livo_debug_eval_prof.argtypes = [C.c_void_p]
        buf = (C.c_ulonglong * 24)()
        ctx.iekf_update_batch(sids, st0)
        ctx.set_profiling(2)
        ctx.iekf_update_batch(sids, st0)
        t = ctx.last_timings()
        print("per-evaluation windows (ms, events, max over groups):", [round(x, 4) for x in t["eval_ms"]])
        ctx.set_profiling(0)
        L.livo_debug_eval_stats.argtypes = [C.c_void_p]
        sbuf = (C.c_ulonglong * 24)()
        L.livo_debug_amb_reason.argtypes = [C.c_void_p]
        abuf = (C.c_ulonglong * 8)()
        mhz = C.c_double(0.0)
        L.livo_debug_clock.argtypes = [C.c_void_p]
        if L.livo_debug_clock(C.byref(mhz)) == 0:
            print(f"s_memtime clock: {mhz.value:.0f} MHz (vs s_memrealtime)")
        L.livo_debug_tail_prof.argtypes = [C.c_void_p]
        tbuf = (C.c_ulonglong * 72)()
        L.livo_debug_tail_prof(tbuf)
        L.livo_debug_eval_prof(buf)  # reset after the warm-up
        L.livo_debug_eval_stats(sbuf)
        L.livo_debug_amb_reason(abuf)
        steps = 10
        for _ in range(steps):
            ctx.iekf_update_batch(sids, st0)
        assert L.livo_debug_eval_prof(buf) == 0
        assert L.livo_debug_eval_stats(sbuf) == 0
        assert L.livo_debug_amb_reason(abuf) == 0
        assert L.livo_debug_tail_prof(tbuf) == 0
        # the reduction's tail (thread 0 s_memtime cycles): every block's butterfly + partial store +
        # ticket; the scan's last block: the partials' reduction, the solve, the host slot write
        for s, name in ((2, "first-search evals"), (1, "rematch evals"), (0, "no-search evals")):
            r = tbuf[8 * s: 8 * s + 8]
            nb, nl = max(r[0], 1), max(r[5], 1)
            print(f"{name} tail: blocks {r[0]}  bfly+ticket {r[1] / nb / 1e3:.2f} kcyc/block  last blocks {r[5]}: "
                  f"reduce {r[2] / nl / 1e3:.2f}  solve {r[3] / nl / 1e3:.2f}  slot write {r[4] / nl / 1e3:.2f} kcyc")
            ph = tbuf[24 + 16 * s: 24 + 16 * s + 8]
            names = ("P+C", "M+vec", "LU", "Minv+w", "K6", "G6+sol", "boxplus+ctrl", "cov")
            print(f"    solve phases (kcyc per last block): " +
                  "  ".join(f"{n} {v / nl / 1e3:.2f}" for n, v in zip(names, ph)))
        print(f"flagged queries per batch: uncertified {abuf[0] / steps:.2f}  C1 near-tie {abuf[1] / steps:.2f}  "
              f"C1 exact tie {abuf[4] / steps:.2f}  C2 gap {abuf[2] / steps:.2f}  C2 equal x {abuf[3] / steps:.2f}")
        for s, name in ((2, "first-search evals"), (1, "rematch evals")):
            r = sbuf[8 * s: 8 * s + 8]
            lanes, waves = max(r[0], 1), max(r[7], 1)
            print(f"{name} search: lanes {r[0]}  ball-certified {r[1] / lanes:.3f}  cell-run lanes {r[2] / lanes:.3f}  "
                  f"ball entries/lane {r[3] / lanes:.1f} (wave max {r[4] / waves:.1f})  "
                  f"cell entries/lane {r[5] / lanes:.1f} (wave max {r[6] / waves:.1f})")
        for s, name in ((2, "first-search evals"), (1, "rematch evals"), (0, "no-search evals")):
            row = buf[8 * s: 8 * s + 8]
            nb = max(row[0], 1)
            # cell-run path: ph1 loads + slot control, ph5 vrun search, ph6 lq_finish (record),
            # ph2 tie replay + barrier, ph3 plane pass, ph4 reduction + ticket (+ solve); slot 7:
            # lanes not certified inside the cube (a count, per block)
            print(f"{name}: blocks {row[0]}  per block (kcycles): " +
                  "  ".join(f"ph{k} {row[k] / nb / 1e3:.2f}" for k in (1, 5, 6, 2, 3, 4)) +
                  f"  uncertified lanes/block {row[7] / nb:.2f}")


if __name__ == "__main__":
    main()
