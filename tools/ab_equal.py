"""Bitwise A/B of two library builds on the same inputs (development tool).

    LIVO_LIB=<lib.so> python tools/ab_equal.py dump OUT.npz [--ikfom]
    python tools/ab_equal.py compare A.npz B.npz

dump: config 2 (1M map, 16 scans of 100k points, max_iteration 4): two
synchronous batches of 8, then the same 16 scans as two pipelined batches
(submit / submit / wait / wait); with --ikfom also the IKFoM batch of the first
8.  Every state (rot, pos, cov, ...) and every statistic goes into the npz.
compare: exits non-zero unless every array is bitwise equal.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))


def _flat(prefix, d, out):
    for k, v in d.items():
        if isinstance(v, dict):
            _flat(prefix + k + ".", v, out)
        else:
            out[prefix + k] = np.asarray(v)


def dump(path, ikfom=False):
    import livo_amd
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, s)[0] for s in range(16)]
    st0 = [synth.make_state(s) for s in range(16)]
    res = {}
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(b) for b in scans]
        for h in range(2):
            outs, stats = ctx.iekf_update_batch(sids[8 * h: 8 * h + 8], st0[8 * h: 8 * h + 8])
            for b in range(8):
                _flat(f"sync.{8 * h + b}.state.", outs[b], res)
                _flat(f"sync.{8 * h + b}.stats.", stats[b], res)
        t0 = ctx.iekf_update_batch_submit(sids[:8], st0[:8])
        t1 = ctx.iekf_update_batch_submit(sids[8:], st0[8:])
        for h, t in enumerate((t0, t1)):
            outs, stats = ctx.iekf_update_batch_wait(t, 8)
            for b in range(8):
                _flat(f"pipe.{8 * h + b}.state.", outs[b], res)
                _flat(f"pipe.{8 * h + b}.stats.", stats[b], res)
        if ikfom:
            ist = [synth.make_ikfom_state(s) for s in range(8)] if hasattr(synth, "make_ikfom_state") else None
            if ist is not None:
                outs, stats = ctx.ikfom_update_batch(sids[:8], ist)
                for b in range(8):
                    _flat(f"ikfom.{b}.state.", outs[b], res)
                    _flat(f"ikfom.{b}.stats.", stats[b], res)
    np.savez(path, **res)
    print(f"dumped {len(res)} arrays to {path}")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if k not in B.files or A[k].shape != B[k].shape or
           A[k].tobytes() != B[k].tobytes()]
    missing = [k for k in B.files if k not in A.files]
    # the pipelined batches must equal the synchronous ones inside each file too
    inner = [k for k in A.files if k.startswith("pipe.") and A[k].tobytes() != A["sync." + k[5:]].tobytes()]
    print(f"{len(A.files)} arrays: {len(bad)} differ between the builds, {len(missing)} missing, "
          f"{len(inner)} pipelined != synchronous")
    for k in (bad + inner)[:20]:
        print("  differs:", k)
    return 0 if not (bad or missing or inner) else 1


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], "--ikfom" in sys.argv)
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
