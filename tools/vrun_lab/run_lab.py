"""Drive the vertex-run lab on the GPU box: time the variants, check they agree."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "fast-livo-noted_amd")]
from livo_amd import synth  # noqa: E402

L = C.CDLL(os.path.join(HERE, "libvrun_lab.so"))
L.lab_build.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_int]
L.lab_queries.argtypes = [C.c_void_p, C.c_int64]
L.lab_run.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
L.lab_run.restype = C.c_double
P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731


def queries(nscans, npts):
    qs = []
    for sid in range(nscans):
        body, _, _ = synth.make_scan(npts, sid)
        st = synth.make_state(sid)
        lo = body.min(0)
        cb = np.floor((body - lo) * 4).astype(np.int64)
        key = np.zeros(len(body), np.int64)
        for bit in range(20):
            for ax in range(3):
                key |= ((cb[:, ax] >> bit) & 1) << (3 * bit + ax)
        body = body[np.argsort(key, kind="stable")]
        qs.append(((body.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(np.float32))
    return np.ascontiguousarray(np.concatenate(qs))


def main():
    mpts = int(os.environ.get("LAB_MAP", "1000000"))
    m = np.ascontiguousarray(synth.cached_map(mpts).astype(np.float32))
    q = queries(int(os.environ.get("LAB_SCANS", "8")), int(os.environ.get("LAB_SCANPTS", "100000")))
    for spec in os.environ.get("LAB_PPC", "v14").split(","):
        mode, ppc = (1 if spec[0] == "c" else 0), float(spec[1:])
        assert L.lab_build(P(m), len(m), ppc, mode) == 0
        L.lab_queries(P(q), len(q))
        n = len(q)
        ref = None
        for v in [int(x) for x in os.environ.get("LAB_VARIANTS", "0,1,2").split(",")]:
            idx = np.zeros((5, n), np.int32); d = np.zeros((5, n), np.float32); fl = np.zeros(n, np.int32)
            st = np.zeros(2, np.int64)
            ms = L.lab_run(v, 10, P(idx), P(d), P(fl), P(st))
            extra = ""
            if ref is None:
                ref = (idx.copy(), fl.copy())
            else:
                bad = ((idx != ref[0]).any(0) & (fl == 0) & (ref[1] == 0)).sum()
                extra = f"mismatch(certified)={bad}"
            print(f"{spec} V{v}: {ms:.4f} ms ({n / ms / 1e3:.0f} Mq/s) scanned/q {st[0] / n:.1f} "
                  f"uncertified {st[1] / n:.4f} {extra}", flush=True)


if __name__ == "__main__":
    main()
