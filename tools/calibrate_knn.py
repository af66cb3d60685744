"""CPU-timing calibration of the oracle's k-NN against the reference's own ikd-Tree timing.

BASELINE.md ("Measured in the survey container") records the reference
`include/ikd-Tree/ikd_Tree.cpp` k=5 `Nearest_Search` (`:350-380,843-986`),
single thread, on synthetic planar maps in this container class (8-core
Xeon): 100k map / 10k queries 2.9-4.1 us, 1M / 100k 4.8-5.7 us, 10M / 200k
6.8 us per query.  That build needs PCL and Eigen headers, which the image
lacks; a rebuild on stand-in headers is not allowed here, so the reference is
not re-timed.  This script times the oracle's restatement (`oracle/`,
`KD_TREE::Build` + `Nearest_Search`) single-threaded on maps and queries of the
same sizes (the repo's synthetic room and Avia scans, moved to the world frame
by the true pose) and writes the ratio oracle / reference per size.

It ties the bench's `cpu_baseline` (kind "port") to the reference's CPU speed;
it pins no parity (different inputs, different run).  Output:
tests/golden/knn_calibration.json.  Run here (not on the GPU box):
    python tools/calibrate_knn.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import oracle  # noqa: E402
from livo_amd import synth  # noqa: E402

# BASELINE.md survey table: (map points, queries, reference us/query low, high)
SURVEY = [(100_000, 10_000, 2.9, 4.1), (1_000_000, 100_000, 4.8, 5.7), (10_000_000, 200_000, 6.8, 6.8)]


def queries(n: int) -> np.ndarray:
    out = []
    sid = 0
    while sum(len(q) for q in out) < n:
        body, R, p = synth.make_scan(min(n, 100_000), sid)
        out.append((body.astype(np.float64) @ (R @ synth.R_LI).T + (R @ synth.T_LI + p)).astype(np.float32))
        sid += 1
    return np.ascontiguousarray(np.concatenate(out)[:n])


def main():
    rows = []
    for m_pts, nq, lo, hi in SURVEY:
        if "--quick" in sys.argv and m_pts > 1_000_000:
            continue
        m = synth.cached_map(m_pts)
        t = time.perf_counter()
        tree = oracle.Tree(m)
        build_s = time.perf_counter() - t
        q = queries(nq)
        times = []
        for k in range(3 + 5):  # 3 warm-ups, median of 5 (each run = all nq queries)
            t = time.perf_counter()
            tree.knn(q, 5, threads=1)
            if k >= 3:
                times.append(time.perf_counter() - t)
        us = float(np.median(times)) / nq * 1e6
        ref = 0.5 * (lo + hi)
        rows.append({"map_points": m_pts, "queries": nq, "oracle_us_per_query": round(us, 3),
                     "reference_us_per_query": [lo, hi], "ratio_oracle_over_reference": round(us / ref, 3),
                     "oracle_build_s": round(build_s, 3)})
        print(rows[-1], flush=True)
        del tree
    out = {"what": "oracle k=5 Nearest_Search vs the reference ikd_Tree.cpp, single thread, us per query",
           "reference_source": "BASELINE.md 'Measured in the survey container' (ikd_Tree.cpp -O3, g++ 11.4)",
           "oracle_source": "oracle/livo_oracle.cpp (this container, g++ -O3), tools/calibrate_knn.py",
           "pins_parity": False,
           "note": "same container class, same sizes, different synthetic inputs: a timing calibration only",
           "rows": rows}
    path = os.path.join(ROOT, "tests", "golden", "knn_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


if __name__ == "__main__":
    main()
