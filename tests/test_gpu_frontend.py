"""GPU parity of the scan front-end: livo_scan_preprocess
against the oracle's UndistortPcl walk and PCL VoxelGrid restatement.

Bars: de-skewed points within 1e-6 relative (double sin/cos of the device
math library may differ from glibc's in the last ulp before the float
rounding); VoxelGrid voxel set, order and counts exact, centroids to float
rounding (the reference sums a voxel in std::sort's unstable order); the
resident scan it creates is the scan livo_scan_upload makes of the same
points (same device Morton order: IEKF results bit-identical).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fctx(built):
    import livo_amd
    from livo_amd import synth
    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    yield ctx
    ctx.close()


def _close(a, b, rel=1e-6):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= rel * np.maximum(np.abs(b), 1.0))


@pytest.mark.parametrize("n,scan", [(50_000, 0), (1, 1), (777, 2)])
def test_undistort_and_voxel_grid(fctx, n, scan):
    import oracle
    from livo_amd import synth
    raw, poses, Re, pe = synth.make_raw_scan(n, scan)
    sid, und, down = fctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.5)
    try:
        ref = oracle.undistort(raw, poses, Re, pe, t_LI=synth.T_LI)
        assert _close(und, ref)
        assert np.array_equal(und[:, 3:], raw[:, 3:])
        dref = oracle.voxel_grid(und, 0.5)  # from the device's de-skewed points: the filter alone
        assert down.shape == dref.shape
        assert _close(down, dref, 2e-6)
    finally:
        fctx.scan_release(sid)


def test_first_point_and_untouched(fctx):
    import oracle
    from livo_amd import synth
    raw, poses, Re, pe = synth.make_raw_scan(2_000, 3)
    raw[:, 4] = np.linspace(-5.0, 99.0, len(raw), dtype=np.float32)  # the first points precede the first pose
    sid, und, _ = fctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.0)
    fctx.scan_release(sid)
    ref = oracle.undistort(raw, poses, Re, pe, t_LI=synth.T_LI)
    assert _close(und, ref)
    assert np.array_equal(und[raw[:, 4] <= 0], raw[raw[:, 4] <= 0])
    raw2 = raw.copy()
    raw2[:, 4] = np.linspace(40.0, 99.0, len(raw), dtype=np.float32)  # first point after 8 poses
    sid, und2, _ = fctx.scan_preprocess(raw2, poses, Re, pe, leaf_size=0.0)
    fctx.scan_release(sid)
    assert _close(und2, oracle.undistort(raw2, poses, Re, pe, t_LI=synth.T_LI))


@pytest.mark.parametrize("leaf", [0.05, 0.2, 1.0])
def test_voxel_grid_only(fctx, leaf):
    import oracle
    from livo_amd import synth
    raw, _, _, _ = synth.make_raw_scan(30_000, 4)
    sid, und, down = fctx.scan_preprocess(raw, leaf_size=leaf)
    fctx.scan_release(sid)
    assert np.array_equal(und, raw)
    dref = oracle.voxel_grid(raw, leaf)
    assert down.shape == dref.shape
    assert _close(down, dref, 2e-6)


def test_voxel_leaf_too_small_keeps_input(fctx):
    from livo_amd import synth
    raw, _, _, _ = synth.make_raw_scan(1_000, 5)
    raw[0, :3] = [-3000, -3000, -3000]
    raw[1, :3] = [3000, 3000, 3000]
    sid, _, down = fctx.scan_preprocess(raw, leaf_size=0.01)
    fctx.scan_release(sid)
    assert np.array_equal(down, raw)


def test_preprocessed_scan_equals_uploaded(fctx):
    """The resident scan from the device front-end is the scan livo_scan_upload
    makes of the same points: same Morton order, bit-identical IEKF update."""
    from livo_amd import synth
    fctx.map_build(synth.cached_map(200_000))
    raw, poses, Re, pe = synth.make_raw_scan(40_000, 6)
    sid, und, down = fctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.2)
    sid2 = fctx.scan_upload(down[:, :3])
    try:
        st = synth.make_state(6)
        s1, t1 = fctx.iekf_update(sid, st)
        s2, t2 = fctx.iekf_update(sid2, st)
        assert t1["effct_feat_num"] == t2["effct_feat_num"] and t1["iterations"] == t2["iterations"]
        assert np.array_equal(s1["pos"], s2["pos"]) and np.array_equal(s1["rot"], s2["rot"])
        assert np.array_equal(s1["cov"], s2["cov"])
        i1, d1 = fctx.scan_neighbors(sid)
        i2, d2 = fctx.scan_neighbors(sid2)
        assert np.array_equal(i1, i2) and np.array_equal(d1, d2)
    finally:
        fctx.scan_release(sid)
        fctx.scan_release(sid2)


def test_preprocess_edge_cases(fctx):
    import livo_amd
    from livo_amd import synth
    sid, und, down = fctx.scan_preprocess(np.zeros((0, 5), np.float32), leaf_size=0.5)
    assert down.shape == (0, 5)
    fctx.scan_release(sid)
    raw, poses, Re, pe = synth.make_raw_scan(100, 7)
    bad = poses.copy()
    bad[3, 0] = -1.0  # segments must be time-ordered
    with pytest.raises(livo_amd.LivoError):
        fctx.scan_preprocess(raw, bad, Re, pe)
    sid, und, _ = fctx.scan_preprocess(raw, poses[:1], Re, pe, leaf_size=0.0)  # one pose: nothing to undo
    fctx.scan_release(sid)
    assert np.array_equal(und, raw)


@pytest.mark.parametrize("n", [30_000, 0])
def test_frame_to_world(fctx, n):
    """RGBpointBodyToWorld over laserCloudFullRes (laser_mapping.cpp:258-265, 647-660):
    the de-skewed full-resolution frame (feats_undistort, kept on the device by
    livo_scan_preprocess) and the downsampled resident scan (feats_down_body, in the
    caller's point order), at the updated state: bit-exact against the oracle's
    transform of the same body points."""
    import oracle
    from livo_amd import synth
    raw, poses, Re, pe = synth.make_raw_scan(max(n, 1), 4)
    raw = raw[:n]
    sid, und, down = fctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.5)
    try:
        st = synth.make_state(4)
        w = fctx.frame_to_world(st)  # the full-resolution frame
        ref = oracle.to_world(und, st, t_LI=synth.T_LI)
        assert w.shape == (n, 5)
        assert np.array_equal(w.view(np.uint32), ref.view(np.uint32))
        wd = fctx.frame_to_world(st, sid)  # the resident scan (x, y, z only: intensity 0)
        refd = oracle.to_world(down[:, :3], st, t_LI=synth.T_LI)
        assert np.array_equal(wd.view(np.uint32), refd.view(np.uint32))
    finally:
        fctx.scan_release(sid)


@pytest.mark.gpu
def test_failed_preprocess_drops_frame(fctx):
    """A livo_scan_preprocess that fails part-way leaves no frame behind: the
    previous frame's feats_undistort is not readable through
    livo_frame_to_world(-1) any more (its buffer may have been reused), and the
    new one is not published until it has been processed completely."""
    import ctypes as C

    from livo_amd import _ptr, synth
    raw, poses, Re, pe = synth.make_raw_scan(4000, 5)
    sid, _, _ = fctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.5)
    fctx.scan_release(sid)
    st = synth.make_state(5)
    assert fctx.frame_to_world(st).shape == (4000, 5)
    raw2 = np.ascontiguousarray(raw[:3000], np.float32)
    down = np.zeros((1, 5), np.float32)  # too small: LIVO_E_RANGE after the frame was de-skewed
    nd, sid2 = C.c_int64(), C.c_int32()
    rc = fctx._L.livo_scan_preprocess(fctx.h, _ptr(raw2), 3000, _ptr(np.ascontiguousarray(poses, np.float64)),
                                      len(poses), _ptr(np.ascontiguousarray(Re, np.float64).reshape(9)),
                                      _ptr(np.ascontiguousarray(pe, np.float64).reshape(3)), C.c_float(0.5),
                                      C.byref(sid2), None, _ptr(down), 1, C.byref(nd))
    assert rc == -6  # LIVO_E_RANGE
    assert fctx.frame_to_world(st).shape == (0, 5)
