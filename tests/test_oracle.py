"""CPU tests of the oracle (oracle/livo_oracle.cpp) — the checker the GPU path is held to.

Parity status: "parity unpinned" — the reference ships no tests or golden
vectors for this path and cannot be built here (PCL/Eigen headers absent), so
the restatement is pinned against independent implementations instead:
  * exact brute-force k-NN (same float distance, same PointType_CMP order);
  * LAPACK xGELSY (column-pivoting QR least squares) for esti_plane;
  * numpy float64 for the Jacobian / normal equations and the IEKF algebra;
and against its own committed golden fixtures (tests/golden/) for regressions.
"""
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _synth():
    from livo_amd import synth
    return synth


@pytest.mark.parametrize("kind", ["uniform", "planar"])
def test_knn_matches_bruteforce(built, kind):
    import oracle
    rng = np.random.default_rng(11)
    if kind == "uniform":
        m = rng.uniform(-10, 10, size=(20_000, 3)).astype(np.float32)
        q = rng.uniform(-11, 11, size=(3_000, 3)).astype(np.float32)
    else:
        m = _synth().make_map(20_000)
        q = (m[rng.choice(len(m), 3_000)] + rng.normal(0, 0.05, size=(3_000, 3))).astype(np.float32)
    idx, d, vis = oracle.Tree(m).knn(q, 5)
    bi, bd = oracle.knn_brute(m, q, 5)
    assert np.array_equal(idx, bi)
    assert np.array_equal(d, bd)
    assert np.all(vis >= 1)


def test_knn_small_maps_and_order(built):
    import oracle
    rng = np.random.default_rng(5)
    for M in range(1, 12):
        m = rng.normal(size=(M, 3)).astype(np.float32)
        q = rng.normal(size=(50, 3)).astype(np.float32)
        idx, d, _ = oracle.Tree(m).knn(q, 5)
        bi, bd = oracle.knn_brute(m, q, 5)
        assert np.array_equal(idx, bi) and np.array_equal(d, bd)
        assert np.all(idx[:, min(M, 5):] == -1)
        assert np.all(np.diff(d[:, :min(M, 5)], axis=1) >= 0)


def test_knn_ties_break_on_x(built):
    """PointType_CMP (ikd_Tree.h:57-60): equal distances order by x."""
    import oracle
    m = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1], [2, 0, 0]], np.float32)
    idx, d, _ = oracle.Tree(m).knn(np.zeros((1, 3), np.float32), 5)
    assert np.all(d[0] == 1.0)
    xs = m[idx[0], 0]
    assert np.all(np.diff(xs) >= 0)


def _plane_cases(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = rng.uniform(-20, 20, size=3)
        c[2] = rng.uniform(-1.5, 2.5)
        nrm = rng.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        u = np.cross(nrm, [1, 0, 0] if abs(nrm[0]) < 0.9 else [0, 1, 0])
        u /= np.linalg.norm(u)
        v = np.cross(nrm, u)
        ab = rng.uniform(-0.2, 0.2, size=(5, 2))
        pts = c + ab[:, :1] * u + ab[:, 1:] * v + rng.normal(0, 0.005, size=(5, 1)) * nrm
        out.append(pts.astype(np.float32))
    return out


def test_esti_plane_vs_lapack_gelsy(built):
    """The float col-pivot Householder LS fit agrees with LAPACK sgelsy."""
    import oracle
    import scipy.linalg as sl
    worst = 0.0
    for pts in _plane_cases(400):
        ok, pabcd = oracle.esti_plane(pts, 0.1)
        x_ref = sl.lstsq(pts, -np.ones(5, np.float32), lapack_driver="gelsy")[0].astype(np.float64)
        x = pabcd[:3].astype(np.float64) / pabcd[3]
        n_ref = x_ref / np.linalg.norm(x_ref)
        worst = max(worst, np.abs(n_ref - pabcd[:3]).max())
        # residual test (common_lib.h:693-699) agrees with a float64 evaluation
        r64 = np.abs(pts.astype(np.float64) @ (x_ref / np.linalg.norm(x_ref)) + 1 / np.linalg.norm(x_ref))
        if r64.max() < 0.09:
            assert ok
        if r64.max() > 0.11:
            assert not ok
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) < 5e-3
    assert worst < 5e-3


def test_esti_plane_degenerate(built):
    import oracle
    # 5 identical points: rank 1 -> one pivot; must not crash, must reject or give finite output
    pts = np.tile(np.array([[3.0, 4.0, 5.0]], np.float32), (5, 1))
    ok, pabcd = oracle.esti_plane(pts, 0.1)
    assert np.all(np.isfinite(pabcd))
    # exact plane z = 2 (x = (0, 0, -0.5)) is recovered
    rng = np.random.default_rng(1)
    pts = np.c_[rng.uniform(-1, 1, size=(5, 2)), np.full(5, 2.0)].astype(np.float32)
    ok, pabcd = oracle.esti_plane(pts, 0.1)
    assert ok
    assert abs(pabcd[2] + 1.0) < 1e-6 and abs(pabcd[3] - 2.0) < 1e-5  # x = (0, 0, -0.5)


def _numpy_hshare(body, rot, pos, t_LI, nv, sel, lpc=0.001):
    keep = sel.astype(bool)
    pb = body[keep].astype(np.float64)
    n = nv[keep, :3].astype(np.float64)
    pd2 = nv[keep, 3].astype(np.float64)
    pI = pb + t_LI
    A = np.cross(pI, n @ rot)  # [p_I]x (R^T n)
    H = np.c_[A, n]
    HTH = H.T @ H / lpc
    HTL = H.T @ (-pd2) / lpc
    return HTH, HTL


def test_h_share_normal_equations_vs_numpy(tree100k):
    synth = _synth()
    body, _, _ = synth.make_scan(8_000, 4)
    st = synth.make_state(4)
    r = tree100k.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True)
    HTH, HTL = _numpy_hshare(body, st["rot"], st["pos"], synth.T_LI, r["normvec"], r["sel"])
    assert r["effct"] == int(r["sel"].sum()) > 7_000
    assert np.allclose(r["HTH"][:6, :6], HTH, rtol=1e-10, atol=1e-6)
    assert np.allclose(r["HTL"][:6], HTL, rtol=1e-10, atol=1e-8)
    assert np.all(r["HTH"][6:] == 0) and np.all(r["HTL"][6:] == 0)
    # every accepted residual passes the gates of laser_mapping.cpp:535,552
    pd2 = r["normvec"][r["sel"].astype(bool), 3]
    assert np.all(np.abs(pd2) <= 2.0)
    # neighbours of accepted points pass the sqdis[4] <= 5 gate
    assert np.all(r["cache"]["d"][r["sel"].astype(bool), 4] <= 5.0)


def _boxplus(st, d):
    synth = _synth()
    out = dict(st)
    out["rot"] = st["rot"] @ synth.so3_exp(d[:3])
    out["pos"] = st["pos"] + d[3:6]
    return out


def test_iekf_first_step_vs_numpy(tree100k):
    """One IEKF evaluation (laser_mapping.cpp:187-193) against numpy float64."""
    synth = _synth()
    body, _, _ = synth.make_scan(6_000, 5)
    st = synth.make_state(5)
    r = tree100k.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True)
    H18 = np.zeros((18, 18))
    H18[:9, :9] = r["HTH"]
    K1 = np.linalg.inv(H18 + np.linalg.inv(st["cov"]))
    sol = K1[:, :9] @ r["HTL"]  # vec = prior - state = 0 on the first evaluation
    _, stats = tree100k.iekf_update(body, st, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=0)
    assert stats["iterations"] == 1
    assert np.allclose(stats["solution"][0], sol, rtol=1e-9, atol=1e-14)


def test_iekf_control_flow(tree100k):
    """Iteration / rematch bookkeeping of laser_mapping.cpp:178-238."""
    synth = _synth()
    body, _, _ = synth.make_scan(4_000, 6)
    st = synth.make_state(6)
    for mi in range(0, 7):
        _, s = tree100k.iekf_update(body, st, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=mi)
        assert 1 <= s["iterations"] <= mi + 1
        assert 1 <= s["knn_passes"] <= 3
        if s["rematch_num"] < 2:
            assert s["iterations"] == mi + 1  # stopped by iterCount == NUM_MAX_ITERATIONS - 1
    # a scan that starts at the truth converges at the first evaluation
    R, p, _ = synth.true_pose(6)
    truth = dict(st)
    truth["rot"], truth["pos"] = R, p
    _, s = tree100k.iekf_update(body, truth, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4)
    assert s["converged"] == 1


def test_iekf_reduces_pose_error(tree100k):
    synth = _synth()
    body, _, _ = synth.make_scan(10_000, 7)
    st = synth.make_state(7, rot_deg=0.3, trans_m=0.03)
    R, p, _ = synth.true_pose(7)
    out, _ = tree100k.iekf_update(body, st, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4)
    assert np.linalg.norm(out["pos"] - p) < np.linalg.norm(st["pos"] - p)
    # covariance shrinks and stays symmetric-ish after (I - G) P
    assert np.trace(out["cov"]) < np.trace(st["cov"])


# ------------------------------------------------------------ golden -----
def _golden_path():
    return os.path.join(GOLDEN, "config1_small.npz")


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, "config1_small.npz")), reason="golden fixture missing")
def test_oracle_matches_golden(built):
    import oracle
    g = np.load(_golden_path(), allow_pickle=False)
    tree = oracle.Tree(g["map"])
    st = {k[6:]: g[k] for k in g.files if k.startswith("state_")}
    r = tree.h_share(g["scan"], st["rot"], st["pos"], np.eye(3), g["t_LI"], True)
    assert np.array_equal(r["cache"]["idx"], g["nn_idx"])
    assert np.array_equal(r["cache"]["d"], g["nn_d"])
    assert np.array_equal(r["normvec"], g["normvec"])
    assert np.array_equal(r["sel"], g["sel"])
    assert np.array_equal(r["HTH"], g["HTH"]) and np.array_equal(r["HTL"], g["HTL"])
    out, stats = tree.iekf_update(g["scan"], st, R_LI=np.eye(3), t_LI=g["t_LI"], max_iter=int(g["max_iter"]))
    assert stats["iterations"] == int(g["iterations"])
    assert np.array_equal(stats["solution"], g["solution"])
    assert np.array_equal(out["rot"], g["out_rot"]) and np.array_equal(out["pos"], g["out_pos"])


# ---------------------------------------------------------------- IKFoM ----
# The IKFoM formulation: MTK manifold pieces, then the
# first update checked against an independent numpy restatement.

def _hat(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _so3_exp(v):
    th = np.linalg.norm(v)
    if th < 1e-15:
        return np.eye(3)
    K = _hat(v / th)
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def test_mtk_A_matrix_is_left_jacobian():
    import oracle
    rng = np.random.default_rng(3)
    for _ in range(5):
        v = rng.normal(size=3) * 0.7
        A = oracle.mtk(2, v, [0.0]).reshape(3, 3)
        d = rng.normal(size=3) * 1e-6
        lhs = _so3_exp(v + d) @ _so3_exp(v).T          # Exp(v + d) Exp(v)^-1 = Exp(A d)
        w = np.array([lhs[2, 1] - lhs[1, 2], lhs[0, 2] - lhs[2, 0], lhs[1, 0] - lhs[0, 1]]) / 2
        assert np.allclose(w, A @ d, rtol=0, atol=1e-11)
    assert np.allclose(oracle.mtk(2, [0.0, 0.0, 0.0], [0.0]).reshape(3, 3), np.eye(3))


def test_mtk_s2_roundtrip_and_length():
    import oracle
    from livo_amd import synth
    rng = np.random.default_rng(4)
    for _ in range(20):
        g = rng.normal(size=3)
        g = g / np.linalg.norm(g) * synth.S2_LEN
        d = rng.normal(size=2) * 0.3
        g2 = oracle.mtk(0, g, d)
        assert abs(np.linalg.norm(g2) - synth.S2_LEN) < 1e-12
        assert np.allclose(oracle.mtk(1, g2, g), d, rtol=0, atol=1e-12)


def test_ikfom_state_boxplus_boxminus_roundtrip():
    import oracle
    from livo_amd import synth
    st = synth.make_ikfom_state(2)
    dx = np.random.default_rng(5).normal(size=23) * 0.05
    assert np.allclose(oracle.mtk(3, st, dx), dx, rtol=0, atol=1e-12)


def _ikfom_dx0_numpy(tree, map_xyz, body, st, lpc=0.001):
    """First-evaluation dx of the IKFoM update in numpy (x = x_propagated: dx_new = 0,
    dx = P_inv[:, :12] H^T h, information form), from the oracle's k-NN and plane fit."""
    import oracle
    from livo_amd import synth
    R = synth.quat_to_rot(st["rot"])
    pI = body.astype(np.float64) + st["offset_T"]
    world = (pI @ R.T + st["pos"]).astype(np.float32)
    idx, d, _ = tree.knn(world)
    rows, hs = [], []
    for i in range(len(body)):
        if d[i, 4] > 5.0:
            continue
        ok, pa = oracle.esti_plane(map_xyz[idx[i]])
        if not ok:
            continue
        pd2 = np.float32(pa[0] * world[i, 0] + pa[1] * world[i, 1] + pa[2] * world[i, 2] + pa[3])
        s = 1 - 0.9 * abs(float(pd2)) / math.sqrt(np.linalg.norm(body[i].astype(np.float64)))
        if not (np.float32(s) > 0.9 and abs(float(pd2)) <= 2.0):
            continue
        n = pa[:3].astype(np.float64)
        C = R.T @ n
        A = _hat(pI[i]) @ C
        B = _hat(body[i].astype(np.float64)) @ C   # offset_R = identity
        rows.append(np.concatenate([n, A, B, C]))
        hs.append(-float(pd2))
    H, h = np.array(rows).reshape(-1, 12), np.array(hs)
    Pt = np.linalg.inv(st["cov"] / lpc)
    Pt[:12, :12] += H.T @ H
    Pinv = np.linalg.inv(Pt)
    return Pinv[:, :12] @ (H.T @ h), len(rows)


def test_ikfom_first_update_matches_numpy(tree100k, map100k):
    from livo_amd import synth
    body, _, _ = synth.make_scan(4000, 7)
    st = synth.make_ikfom_state(7)
    _, stats = tree100k.ikfom_update(body, st, max_iter=0)
    dx, m = _ikfom_dx0_numpy(tree100k, map100k, body, st)
    assert stats["effct_feat_num"][0] == m
    assert np.linalg.norm(stats["dx"][0] - dx) <= 1e-8 * np.linalg.norm(dx)


def test_ikfom_update_reduces_pose_error(tree100k):
    from livo_amd import synth
    body, _, _ = synth.make_scan(8000, 9)
    st0 = synth.make_ikfom_state(9)
    Rt, pt, _ = synth.true_pose(9)
    st, stats = tree100k.ikfom_update(body, st0, max_iter=4)
    assert 1 <= stats["iterations"] <= 5 and stats["knn_passes"] >= 1
    err0 = np.linalg.norm(st0["pos"] - pt)
    err1 = np.linalg.norm(st["pos"] - pt)
    assert err1 < 0.2 * err0
    Rerr = synth.quat_to_rot(st["rot"]).T @ Rt
    assert math.degrees(math.acos(min(1.0, (np.trace(Rerr) - 1) / 2))) < 0.2
    assert abs(np.linalg.norm(st["grav"]) - synth.S2_LEN) < 1e-9
    assert np.all(np.linalg.eigvalsh((st["cov"] + st["cov"].T) / 2) > 0)
    assert np.all(np.diag(st["cov"])[:6] < np.diag(st0["cov"])[:6])


def test_ikfom_few_points_measurement_space_branch(tree100k, map100k):
    """Fewer than 23 effective points: the reference switches to the
    measurement-space gain (esekfom.hpp:1701-1736), the same update as the
    information form up to rounding."""
    from livo_amd import synth
    body, _, _ = synth.make_scan(4000, 3)
    st0 = synth.make_ikfom_state(3)
    few = body[:12]
    _, stats = tree100k.ikfom_update(few, st0, max_iter=0)
    dx, m = _ikfom_dx0_numpy(tree100k, map100k, few, st0)
    assert 0 < m < 23 and stats["effct_feat_num"][0] == m
    assert np.linalg.norm(stats["dx"][0] - dx) <= 1e-8 * np.linalg.norm(dx)
