"""IKFoM formulation on the GPU against the oracle.

state_ikfom (use-ikfom.hpp:12-21), the legacy h-model
(origin_laserMapping.cpp:916-1048) and update_iterated_dyn_share_modified
(esekfom.hpp:1619-1928).  Bars: iteration / search / convergence control and
effective-point counts exact; per-evaluation dx within 1e-5 of its own norm
for every step, the converged near-zero ones included (a converged step is a
~1e5-fold cancellation in this form, see _compare: both sides form the
h_x^T h_x sums as compensated sums, so their summation orders do not show);
covariance within 1e-9 of the prior's norm.  Fewer than 23 effective points: the reference's
measurement-space gain (:1701-1736) on both sides (the device collects the
effective rows of such scans in point order, k_hshare_ik / k_solve_ik).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-5


def _rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def ctx(built, map100k):
    import livo_amd
    from livo_amd import synth
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as c:
        c.map_build(map100k)
        yield c


def _compare(g, gs, r, rs, st0):
    assert gs["iterations"] == rs["iterations"]
    assert gs["knn_passes"] == rs["knn_passes"]
    assert gs["converged"] == rs["converged"] and gs["t"] == rs["t"]
    assert gs["effct_feat_num"] == rs["effct_feat_num"]
    # per-evaluation dx against its own norm, every step: a converged step
    # (|dx| ~ 1e-4 of the first) is dx = K_h + (K_x - I) dx_new with K_x ~ I,
    # which amplifies the last bits of the h_x^T h_x sums ~1e5-fold; both sides
    # form them as compensated sums (device partials vs the oracle's serial
    # loop round to the same doubles), so the summation order does not show
    for e in range(gs["iterations"]):
        err = np.linalg.norm(gs["dx"][e] - rs["dx"][e])
        own = np.linalg.norm(rs["dx"][e])
        assert err <= REL * max(own, 1e-300), (e, err / max(own, 1e-300))
    upd = np.linalg.norm(r["pos"] - st0["pos"])
    assert np.linalg.norm(g["pos"] - r["pos"]) <= REL * max(upd, 1e-12)
    for k in ("rot", "offset_R"):
        assert np.linalg.norm(g[k] - r[k]) <= REL * max(np.linalg.norm(rs["dx"][:, 3:9]), 1e-12), k
    assert np.linalg.norm(g["grav"] - r["grav"]) <= 1e-9 * np.linalg.norm(r["grav"])
    assert np.linalg.norm(g["cov"] - r["cov"]) <= 1e-9 * np.linalg.norm(st0["cov"])


@pytest.mark.parametrize("max_iter", [4, 2, 1, 0])
def test_ikfom_parity_config1(ctx, tree100k, max_iter):
    from livo_amd import synth
    body, _, _ = synth.make_scan(10_000, 0)
    st0 = synth.make_ikfom_state(0)
    ctx.set_params(max_iterations=max_iter)
    sid = ctx.scan_upload(body)
    try:
        g, gs = ctx.ikfom_update(sid, st0)
    finally:
        ctx.scan_release(sid)
        ctx.set_params(max_iterations=4)
    r, rs = tree100k.ikfom_update(body, st0, max_iter=max_iter)
    _compare(g, gs, r, rs, st0)


def test_ikfom_batch_equals_single(ctx, tree100k):
    from livo_amd import synth
    scans = [synth.make_scan(3000 + 313 * s, s + 10)[0] for s in range(5)]
    states = [synth.make_ikfom_state(s + 10) for s in range(5)]
    sids = [ctx.scan_upload(b) for b in scans]
    try:
        bg, bs = ctx.ikfom_update_batch(sids, states)
        for i, sid in enumerate(sids):
            one, os_ = ctx.ikfom_update(sid, states[i])
            assert all(np.array_equal(one[k], bg[i][k]) for k in one)
            assert os_["iterations"] == bs[i]["iterations"]
        r, rs = tree100k.ikfom_update(scans[2], states[2], max_iter=4)
        _compare(bg[2], bs[2], r, rs, states[2])
    finally:
        for sid in sids:
            ctx.scan_release(sid)


@pytest.mark.parametrize("n", [12, 40])
def test_ikfom_few_points(ctx, tree100k, n):
    """12 points: fewer than 23 effective (the reference's measurement-space gain
    on the device too); 40: the information form."""
    from livo_amd import synth
    body, _, _ = synth.make_scan(4000, 3)
    body = body[:n]
    st0 = synth.make_ikfom_state(3)
    sid = ctx.scan_upload(body)
    try:
        g, gs = ctx.ikfom_update(sid, st0)
    finally:
        ctx.scan_release(sid)
    r, rs = tree100k.ikfom_update(body, st0, max_iter=4)
    _compare(g, gs, r, rs, st0)


def test_ikfom_empty_scan(ctx):
    from livo_amd import synth
    st0 = synth.make_ikfom_state(1)
    sid = ctx.scan_upload(np.zeros((0, 3), np.float32))
    try:
        g, gs = ctx.ikfom_update(sid, st0)
    finally:
        ctx.scan_release(sid)
    assert gs["iterations"] >= 1 and gs["effct_feat_num"][0] == 0


@pytest.mark.slow
def test_ikfom_full_size_1M(built):
    """IKFoM at BASELINE config 2 size: 100k-point scan vs 1M-point map."""
    import livo_amd
    import oracle
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    tree = oracle.Tree(m)
    body, _, _ = synth.make_scan(100_000, 0)
    st0 = synth.make_ikfom_state(0)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as c:
        c.map_build(m)
        sid = c.scan_upload(body)
        g, gs = c.ikfom_update(sid, st0)
    r, rs = tree.ikfom_update(body, st0, max_iter=4, threads=8)
    _compare(g, gs, r, rs, st0)


def test_ikfom_submit_wait_pipelined(ctx):
    """livo_ikfom_update_batch_submit / _wait: two IKFoM batches in flight (their
    slots, jobs and replay lists per lane) give bit for bit the synchronous
    batches' states and statistics; a third submit while both lanes are busy is
    LIVO_E_BUSY; a LaserMapping wait on an IKFoM ticket is LIVO_E_INVALID."""
    import livo_amd
    from livo_amd import synth
    scans = [synth.make_scan(4000 + 211 * s, s + 40)[0] for s in range(10)]
    states = [synth.make_ikfom_state(s + 40) for s in range(10)]
    sids = [ctx.scan_upload(b) for b in scans]
    try:
        ref_a = ctx.ikfom_update_batch(sids[:5], states[:5])
        ref_b = ctx.ikfom_update_batch(sids[5:], states[5:])
        ta = ctx.ikfom_update_batch_submit(sids[:5], states[:5])
        tb = ctx.ikfom_update_batch_submit(sids[5:], states[5:])
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.ikfom_update_batch_submit(sids[:1], states[:1])
        assert e.value.code == -8  # LIVO_E_BUSY
        with pytest.raises(livo_amd.LivoError):
            ctx.iekf_update_batch_wait(ta, 5)
        got_b = ctx.ikfom_update_batch_wait(tb, 5)  # out of order
        got_a = ctx.ikfom_update_batch_wait(ta, 5)
        for got, ref in ((got_a, ref_a), (got_b, ref_b)):
            for i in range(5):
                assert all(np.array_equal(got[0][i][k], ref[0][i][k]) for k in ref[0][i])
                assert got[1][i]["iterations"] == ref[1][i]["iterations"]
                assert np.array_equal(got[1][i]["dx"], ref[1][i]["dx"])
    finally:
        for sid in sids:
            ctx.scan_release(sid)
