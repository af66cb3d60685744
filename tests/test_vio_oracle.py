"""CPU tests of the VIO photometric-update restatement (oracle/livo_oracle.cpp,
VIO section; SURVEY.md §8f row 4: LidarSelector::UpdateState / ComputeJ,
src/lidar_selection.cpp:748-978).

Parity status: "parity unpinned" against the reference itself (OpenCV, vikit,
Sophus, Eigen, ROS absent; no fixtures).  Pinned against an independent numpy
restatement of the same update (float32 weights / residual sums, float64
Jacobians and algebra), and by its behaviour: on synthetic frames whose
reference patches were sampled at the true pose, the update converges to it.
"""
import numpy as np


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _exp(v):
    n = np.linalg.norm(v)
    if n <= 1e-5:
        return np.eye(3)
    K = _skew(v / n)
    return np.eye(3) + np.sin(n) * K + (1 - np.cos(n)) * K @ K


def _log(R):
    tr = np.trace(R)
    th = 0.0 if tr > 3 - 1e-6 else np.arccos(0.5 * (tr - 1))
    k = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return 0.5 * k if abs(th) < 0.001 else 0.5 * th / np.sin(th) * k


def _vio_np(fr, st, max_iter=4, cov_img=10.0):
    from livo_amd import synth
    img = fr["image"].astype(np.float32)
    H_, W = img.shape
    cam, ps = fr["cam"], fr["patch_size"]
    pst, ph = ps * ps, ps // 2
    Rci, Pci = fr["Rci"], fr["Pci"]
    Pic = -Rci.T @ Pci
    Jdphi_dR, Jdp_dR = Rci, -Rci @ _skew(Pic)
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    prior = {k: np.array(v, copy=True) for k, v in st.items()}
    G = np.zeros((18, 18))

    def minus(a, b):
        return np.concatenate([_log(b["rot"].T @ a["rot"]), a["pos"] - b["pos"], a["vel"] - b["vel"],
                               a["bias_g"] - b["bias_g"], a["bias_a"] - b["bias_a"], a["gravity"] - b["gravity"]])

    def update_state(level, total):
        nonlocal G
        old = {k: v.copy() for k, v in st.items()}
        last = np.float32(total)
        for it in range(max_iter):
            Rcw = Rci @ st["rot"].T
            Pcw = -Rcw @ st["pos"] + Pci
            rows, zs = [], []
            err = np.float32(0)
            for i in range(len(fr["pos"])):
                scale = 1 << (level + int(fr["levels"][i]))
                pf = Rcw @ fr["pos"][i] + Pcw
                pc = synth._world2cam(cam, pf[None])[0]
                Jdpi = np.array([[cam["fx"] / pf[2], 0, -cam["fx"] * pf[0] / pf[2] ** 2],
                                 [0, cam["fy"] / pf[2], -cam["fy"] * pf[1] / pf[2] ** 2]])
                ui = int(np.floor(np.float32(pc[0] / scale)) * scale)
                vi = int(np.floor(np.float32(pc[1] / scale)) * scale)
                su = np.float32((np.float32(pc[0]) - ui) / scale)
                sv = np.float32((np.float32(pc[1]) - vi) / scale)
                w = [np.float32((1.0 - su) * (1.0 - sv)), np.float32(su * (1.0 - sv)), np.float32((1.0 - su) * sv),
                     np.float32(su * sv)]
                P = fr["patches"][i]
                pe = np.float32(0)
                for x in range(ps):
                    for y in range(ps):
                        r0, c0 = vi + x * scale - ph * scale, ui - ph * scale + y * scale

                        def I(dr, dc):
                            return img[r0 + dr, c0 + dc]
                        s = scale
                        bl = lambda a, b, c, d: ((w[0] * a + w[1] * b) + w[2] * c) + w[3] * d  # noqa: E731
                        du = np.float32(0.5) * (bl(I(0, s), I(0, 2 * s), I(s, s), I(s, 2 * s)) -
                                                bl(I(0, -s), I(0, 0), I(s, -s), I(s, 0)))
                        dv = np.float32(0.5) * (bl(I(s, 0), I(s, s), I(2 * s, 0), I(2 * s, s)) -
                                                bl(I(-s, 0), I(-s, s), I(0, 0), I(0, s)))
                        J = np.array([du, dv], np.float64) * (1.0 / scale)
                        Jdphi = J @ Jdpi @ _skew(pf)
                        Jdp = -J @ Jdpi
                        rows.append(np.concatenate([Jdphi @ Jdphi_dR + Jdp @ Jdp_dR, Jdp @ Rcw]))
                        res = float(bl(I(0, 0), I(0, s), I(s, 0), I(s, s)) - P[pst * level + x * ps + y])
                        zs.append(res)
                        pe = np.float32(float(pe) + res * res)
                err = np.float32(err + pe)
            err = np.float32(err / np.float32(len(zs)))
            if err <= last:
                old = {k: v.copy() for k, v in st.items()}
                last = err
                Hs, z = np.array(rows), np.array(zs)
                HTH = np.zeros((18, 18))
                HTH[:6, :6] = Hs.T @ Hs
                K1 = np.linalg.inv(HTH + np.linalg.inv(st["cov"] / cov_img))
                G = np.zeros((18, 18))
                G[:, :6] = K1[:, :6] @ HTH[:6, :6]
                vec = minus(prior, st)
                sol = -K1[:, :6] @ (Hs.T @ z) + vec - G[:, :6] @ vec[:6]
                st["rot"] = st["rot"] @ _exp(sol[:3])
                for k, sl in (("pos", 3), ("vel", 6), ("bias_g", 9), ("bias_a", 12), ("gravity", 15)):
                    st[k] = st[k] + sol[sl:sl + 3]
                if np.linalg.norm(sol[:3]) * 57.3 < 0.001 and np.linalg.norm(sol[3:6]) * 100 < 0.001:
                    break
            else:
                st.update({k: v.copy() for k, v in old.items()})
                break
        return last

    err0 = np.float32(1e10)
    now = err0
    for level in (2, 1, 0):
        now = update_state(level, err0)
    if now < err0:
        st["cov"] = st["cov"] - G @ st["cov"]
    return st


def test_vio_update_matches_numpy(built):
    import oracle
    from livo_amd import synth
    fr, st, truth = synth.make_vio_frame(150, 1)
    got, stats, err = oracle.vio_update(fr, st)
    exp = _vio_np(fr, st)
    assert np.allclose(got["pos"], exp["pos"], rtol=0, atol=1e-9)
    assert np.allclose(got["rot"], exp["rot"], rtol=0, atol=1e-9)
    assert np.allclose(got["cov"], exp["cov"], rtol=0, atol=1e-12)
    assert stats["cov_updated"] == 1 and stats["out_of_frame"] == 0


def test_vio_update_converges_to_truth(built):
    import oracle
    from livo_amd import synth
    for fid in (0, 2):
        fr, st, truth = synth.make_vio_frame(1500, fid)
        got, stats, err = oracle.vio_update(fr, st)
        assert np.linalg.norm(got["pos"] - truth["pos"]) < 0.1 * np.linalg.norm(st["pos"] - truth["pos"])
        assert np.linalg.norm(_log(got["rot"].T @ truth["rot"])) < 0.1 * np.linalg.norm(_log(st["rot"].T @ truth["rot"]))
        assert sum(stats["updates"]) >= 3 and np.all(err >= 0)


def test_vio_no_points_is_a_no_op(built):
    import oracle
    from livo_amd import synth
    fr, st, _ = synth.make_vio_frame(10, 3)
    for k in ("pos", "levels", "patches"):
        fr[k] = fr[k][:0]
    got, stats, _ = oracle.vio_update(fr, st)
    assert np.array_equal(got["pos"], st["pos"]) and stats["iterations"] == [0, 0, 0]
