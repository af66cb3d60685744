"""CPU tests of the scan front-end restatement (oracle/livo_oracle.cpp, scan
front-end section).

Parity status: "parity unpinned" against the reference itself (ROS/PCL/Eigen
absent; the reference ships no fixtures).  Pinned against independent numpy
restatements of the documented behaviour:
  * UndistortPcl's backward walk (IMU_Processing.cpp:340-378), including the
    first point being re-compensated by every remaining IMU segment (the inner
    loop breaks at begin() without stepping) and points at or before the first
    pose untouched;
  * PCL VoxelGrid::applyFilter: leaf indices, voxel order (ascending index),
    point counts exact; centroids to float rounding (the reference sums a
    voxel in std::sort's unstable order; numpy here sums in input order).
"""
import numpy as np


def _exp(g, dt):
    n = np.sqrt((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2])
    if n <= 1e-7:
        return np.eye(3)
    r = g / n
    K = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
    a = n * dt
    return np.eye(3) + np.sin(a) * K + ((1 - np.cos(a)) * K) @ K


def _undistort_np(raw, poses, Re, pe, RLI, tLI):
    p = raw.astype(np.float32).copy()
    extR = RLI.T @ Re.T
    ext_t = RLI.T @ tLI
    it = len(p) - 1

    def comp(i, h):
        dt = float(p[i, 4]) / 1000.0 - h[0]
        Ri = h[13:22].reshape(3, 3) @ _exp(h[4:7], dt)
        T = h[10:13] + h[7:10] * dt + 0.5 * h[1:4] * dt * dt - pe
        c = extR @ (Ri @ (RLI @ p[i, :3].astype(np.float64) + tLI) + T) - ext_t
        p[i, :3] = c.astype(np.float32)

    for kp in range(len(poses) - 1, 0, -1):
        h = poses[kp - 1]
        while float(p[it, 4]) / 1000.0 > h[0]:
            comp(it, h)
            if it == 0:
                break
            it -= 1
    return p


def test_undistort_matches_numpy(built):
    import oracle
    from livo_amd import synth
    raw, poses, Re, pe = synth.make_raw_scan(3_000, 1)
    raw[:40, 4] = 0.0  # points at the first pose's time: never compensated
    got = oracle.undistort(raw, poses, Re, pe, t_LI=synth.T_LI)
    exp = _undistort_np(raw, poses, Re, pe, np.eye(3), synth.T_LI)
    assert np.allclose(got, exp, rtol=0, atol=2e-6)
    assert np.array_equal(got[:40], raw[:40])
    assert np.array_equal(got[:, 3:], raw[:, 3:])


def test_undistort_first_point_recompensated(built):
    """A scan whose first point lies after several IMU poses: the reference moves
    it once per remaining segment (its walk breaks at begin() without stepping)."""
    import oracle
    from livo_amd import synth
    raw, poses, Re, pe = synth.make_raw_scan(50, 2)
    raw[:, 4] = np.linspace(30.0, 99.0, 50, dtype=np.float32)
    got = oracle.undistort(raw, poses, Re, pe, t_LI=synth.T_LI)
    exp = _undistort_np(raw, poses, Re, pe, np.eye(3), synth.T_LI)
    assert np.allclose(got, exp, rtol=0, atol=2e-6)
    # point 1 moved once, with the last pose before its time
    h = poses[int(np.searchsorted(poses[:, 0], raw[1, 4] / 1000.0)) - 1]
    dt = float(raw[1, 4]) / 1000.0 - h[0]
    Ri = h[13:22].reshape(3, 3) @ _exp(h[4:7], dt)
    T = h[10:13] + h[7:10] * dt + 0.5 * h[1:4] * dt * dt - pe
    once = Re.T @ (Ri @ (raw[1, :3].astype(np.float64) + synth.T_LI) + T) - synth.T_LI
    assert np.allclose(got[1, :3], once, atol=2e-6)
    # point 0 moved by its segment and every earlier one: not the single move
    h0 = poses[int(np.searchsorted(poses[:, 0], raw[0, 4] / 1000.0)) - 1]
    dt0 = float(raw[0, 4]) / 1000.0 - h0[0]
    R0 = h0[13:22].reshape(3, 3) @ _exp(h0[4:7], dt0)
    T0 = h0[10:13] + h0[7:10] * dt0 + 0.5 * h0[1:4] * dt0 * dt0 - pe
    once0 = Re.T @ (R0 @ (raw[0, :3].astype(np.float64) + synth.T_LI) + T0) - synth.T_LI
    assert np.abs(got[0, :3] - once0).max() > 1e-3


def _voxel_np(raw, leaf):
    leaf = np.float32(leaf)
    inv = np.float32(1.0) / leaf
    mn = raw[:, :3].min(0)
    mx = raw[:, :3].max(0)
    d = ((mx - mn) * inv).astype(np.int64) + 1
    assert np.prod(d) <= 2 ** 31 - 1
    mnb = np.floor(mn * inv).astype(np.int64)
    mxb = np.floor(mx * inv).astype(np.int64)
    div = mxb - mnb + 1
    ijk = (np.floor(raw[:, :3] * inv) - mnb.astype(np.float32)).astype(np.int64)
    idx = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)
    o = np.argsort(idx, kind="stable")
    keys, start, cnt = np.unique(idx[o], return_index=True, return_counts=True)
    out = np.zeros((len(keys), 5), np.float32)
    for k, (s, c) in enumerate(zip(start, cnt)):
        acc = np.zeros(5, np.float32)
        for j in o[s:s + c]:
            acc += raw[j]
        out[k] = acc / np.float32(c)
    return out, cnt


def test_voxel_grid_matches_numpy(built):
    import oracle
    from livo_amd import synth
    raw, _, _, _ = synth.make_raw_scan(6_000, 3)
    for leaf in (0.5, 0.2, 0.05):
        got = oracle.voxel_grid(raw, leaf)
        exp, cnt = _voxel_np(raw, leaf)
        assert got.shape == exp.shape
        assert np.allclose(got, exp, rtol=2e-6, atol=2e-5)
    # leaf too small for 32-bit leaf indices: PCL returns the input unchanged
    big = raw.copy()
    big[0, :3] = [-3000, -3000, -3000]
    big[1, :3] = [3000, 3000, 3000]
    assert np.array_equal(oracle.voxel_grid(big, 0.01), big)
