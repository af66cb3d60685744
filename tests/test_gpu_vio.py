"""GPU parity of the VIO photometric update:
livo_vio_update against the oracle's ComputeJ / UpdateState restatement.

Bars: iteration / update counts and the per-level float errors exact (they
steer the reference's control flow: `error <= last_error`, the error is the
float sum of the per-point patch errors in point order, summed the same way
on the device); per-point patch errors bit-exact; state within 1e-9 m / rad
of the oracle (HᵀH is summed in a different order); covariance within 1e-12.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vctx(built):
    import livo_amd
    ctx = livo_amd.Context(0)
    yield ctx
    ctx.close()


def _check(g, r):
    gs, gst, gerr = g
    rs, rst, rerr = r
    assert gst["iterations"] == rst["iterations"] and gst["updates"] == rst["updates"]
    assert gst["cov_updated"] == rst["cov_updated"] and gst["n_meas"] == rst["n_meas"]
    assert np.array_equal(np.float32(gst["last_error"]), np.float32(rst["last_error"]))
    assert np.array_equal(gerr.view(np.uint32), rerr.view(np.uint32))
    assert np.abs(gs["pos"] - rs["pos"]).max() < 1e-9
    assert np.abs(gs["rot"] - rs["rot"]).max() < 1e-9
    assert np.abs(gs["cov"] - rs["cov"]).max() < 1e-12


@pytest.mark.parametrize("n,fid", [(2000, 0), (300, 1), (5000, 2), (1, 3)])
def test_vio_update_parity(vctx, n, fid):
    import oracle
    from livo_amd import synth
    fr, st, truth = synth.make_vio_frame(n, fid)
    g = vctx.vio_update(fr, st)
    r = oracle.vio_update(fr, st)
    _check(g, r)
    if n >= 300:
        assert np.linalg.norm(g[0]["pos"] - truth["pos"]) < 0.2 * np.linalg.norm(st["pos"] - truth["pos"])


def test_vio_prior_and_iterations(vctx):
    import oracle
    from livo_amd import synth
    fr, st, _ = synth.make_vio_frame(1500, 4)
    prior = dict(st)
    prior["pos"] = st["pos"] + np.array([0.01, -0.005, 0.002])
    for it in (0, 1, 2, 10):
        _check(vctx.vio_update(fr, st, prior, max_iter=it), oracle.vio_update(fr, st, prior, max_iter=it))


def test_vio_patch_size_and_cov(vctx):
    import oracle
    from livo_amd import synth
    fr, st, _ = synth.make_vio_frame(800, 5, patch_size=6)
    _check(vctx.vio_update(fr, st, img_point_cov=100.0), oracle.vio_update(fr, st, img_point_cov=100.0))


def test_vio_no_points(vctx):
    from livo_amd import synth
    fr, st, _ = synth.make_vio_frame(10, 6)
    for k in ("pos", "levels", "patches"):
        fr[k] = fr[k][:0]
    s, stats, _ = vctx.vio_update(fr, st)
    assert np.array_equal(s["pos"], st["pos"]) and stats["iterations"] == [0, 0, 0] and stats["cov_updated"] == 0
