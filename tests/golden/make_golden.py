"""Generate tests/golden/config1_small.npz (committed fixture).

The reference has no golden vectors for this path and cannot be built here
(SURVEY.md §4, §8c), so this fixture is produced by the CPU restatement
(oracle/livo_oracle.cpp) on deterministic synthetic inputs, and stores the
inputs themselves so that it does not depend on the generator staying
unchanged.  It pins the oracle (tests/test_oracle.py::test_oracle_matches_golden)
and the HIP path (tests/test_gpu_bench_mode.py::test_golden_fixture) against
regressions.

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "fast-livo-noted_amd"), os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402
from livo_amd import synth  # noqa: E402


def main():
    m = synth.make_map(20_000)
    scan, _, _ = synth.make_scan(2_000, 0)
    st = synth.make_state(0)
    tree = oracle.Tree(m)
    r = tree.h_share(scan, st["rot"], st["pos"], np.eye(3), synth.T_LI, True)
    max_iter = 4
    out, stats = tree.iekf_update(scan, st, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=max_iter)
    np.savez_compressed(
        os.path.join(HERE, "config1_small.npz"),
        map=m, scan=scan, t_LI=synth.T_LI, max_iter=np.int32(max_iter),
        **{"state_" + k: v for k, v in st.items()},
        nn_idx=r["cache"]["idx"], nn_d=r["cache"]["d"], normvec=r["normvec"], sel=r["sel"],
        HTH=r["HTH"], HTL=r["HTL"], effct=np.int64(r["effct"]), visits=np.int64(r["visits"]),
        iterations=np.int32(stats["iterations"]), knn_passes=np.int32(stats["knn_passes"]),
        effct_feat_num=np.array(stats["effct_feat_num"], np.int64), solution=stats["solution"],
        out_rot=out["rot"], out_pos=out["pos"], out_cov=out["cov"])
    print("wrote", os.path.join(HERE, "config1_small.npz"), "effct", r["effct"], "iters", stats["iterations"])


if __name__ == "__main__":
    main()
