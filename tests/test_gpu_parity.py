"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star):
  * k-NN indices / squared distances, world points, plane normals, residuals
    and selection flags: bit-exact (integer/index work, and float work done in
    the reference's operation order on both sides);
  * HTH / HTL (double, different summation order): 1e-9 relative;
  * IEKF state delta per evaluation: 1e-5 relative (north_star tolerance);
    iteration / k-NN-pass / effective-point counts: exact.
Parity vs the reference itself is unpinned (see oracle/livo_oracle.cpp header).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_HTH = 1e-9
REL_STATE = 1e-5


def _synth():
    from livo_amd import synth
    return synth


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = max(np.linalg.norm(b), 1e-300)
    return np.linalg.norm(a - b) / den


@pytest.fixture(scope="module")
def ctx100k(gpu_ctx, map100k):
    gpu_ctx.map_build(map100k)
    return gpu_ctx


def test_map_info(ctx100k):
    info = ctx100k.map_info()
    assert info["num_points"] == 100_000
    assert info["depth"] == 17  # floor(log2(1e5)) + 1
    assert info["num_slots"] == 2 ** 17 - 1
    # ikd-Tree records + leaf map (internal boxes + float4 points)
    assert info["device_bytes"] >= (2 ** 17) * 64 + 100_000 * 16


def test_knn_bit_exact(ctx100k, tree100k, map100k):
    synth = _synth()
    body, _, _ = synth.make_scan(10_000, 0)
    st = synth.make_state(0)
    q = ((body.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(np.float32)
    idx, d = ctx100k.knn(q, 5)
    ridx, rd, _ = tree100k.knn(q, 5)
    assert np.array_equal(idx, ridx)
    assert np.array_equal(d.view(np.uint32), rd.view(np.uint32))
    # ascending, and distances recomputed from the returned indices
    assert np.all(np.diff(d, axis=1) >= 0)
    p = map100k[idx]
    dd = ((q[:, None, 0] - p[..., 0]) ** 2 + (q[:, None, 1] - p[..., 1]) ** 2) + (q[:, None, 2] - p[..., 2]) ** 2
    assert np.array_equal(dd.astype(np.float32), d)


@pytest.mark.parametrize("k", [1, 3, 5])
def test_knn_k(ctx100k, tree100k, k):
    rng = np.random.default_rng(7)
    q = rng.uniform([-32, -22, -2], [32, 22, 3], size=(3000, 3)).astype(np.float32)
    idx, d = ctx100k.knn(q, k)
    ridx, rd, _ = tree100k.knn(q, k)
    assert np.array_equal(idx, ridx) and np.array_equal(d, rd)


def test_knn_edge_maps(built):
    """Tiny maps (fewer points than k), duplicates / exact ties, far queries."""
    import livo_amd
    import oracle
    rng = np.random.default_rng(3)
    with livo_amd.Context(0) as ctx:
        for M in (1, 2, 3, 4, 5, 6, 7, 31, 64, 65):
            m = rng.normal(size=(M, 3)).astype(np.float32)
            ctx.map_build(m)
            q = np.concatenate([rng.normal(size=(200, 3)), [[1e4, 1e4, 1e4], [0, 0, 0]]]).astype(np.float32)
            idx, d = ctx.knn(q, 5)
            ridx, rd, _ = oracle.Tree(m).knn(q, 5)
            assert np.array_equal(idx, ridx), M
            assert np.array_equal(d, rd), M
            assert np.all(idx[:, min(M, 5):] == -1)
        # exact duplicates and equal-distance ties: a lattice
        g = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(3)), -1).reshape(-1, 3).astype(np.float32)
        m = np.concatenate([g, g[:20]])  # 20 exact duplicate points
        ctx.map_build(m)
        q = np.concatenate([g + 0.5, g, rng.uniform(0, 5, size=(300, 3))]).astype(np.float32)
        idx, d = ctx.knn(q, 5)
        ridx, rd, _ = oracle.Tree(m).knn(q, 5)
        assert np.array_equal(idx, ridx)
        assert np.array_equal(d, rd)


def test_knn_empty_map(built):
    import livo_amd
    with livo_amd.Context(0) as ctx:
        ctx.map_build(np.zeros((0, 3), np.float32))
        idx, d = ctx.knn(np.zeros((4, 3), np.float32), 5)
        assert np.all(idx == -1) and np.all(np.isinf(d))


def _hshare_compare(g, r, n, body=None):
    # laserCloudOri / corr_normvect (laser_mapping.cpp:547-561): the effective points in point order
    if body is not None:
        eff = r["sel"] != 0
        assert np.array_equal(g["ori"], np.asarray(body, np.float32)[eff])
        assert np.array_equal(g["corr_normvec"].view(np.uint32), r["normvec"][eff].view(np.uint32))
    assert np.array_equal(g["nn_idx"], r["cache"]["idx"])
    assert np.array_equal(g["nn_d"].view(np.uint32), r["cache"]["d"].view(np.uint32))
    assert np.array_equal(g["normvec"].view(np.uint32), r["normvec"].view(np.uint32))
    assert np.array_equal(g["sel"], r["sel"])
    assert g["effct"] == r["effct"]
    assert _rel(g["HTH"], r["HTH"]) < REL_HTH
    assert _rel(g["HTL"], r["HTL"]) < REL_HTH


def test_h_share_parity(ctx100k, tree100k):
    synth = _synth()
    body, _, _ = synth.make_scan(10_000, 1)
    st = synth.make_state(1)
    sid = ctx100k.scan_upload(body)
    try:
        g = ctx100k.h_share(sid, st, search_en=True)
        r = tree100k.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True)
        world = ((body.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(np.float32)
        assert np.abs(g["world"] - world).max() <= 1e-5
        _hshare_compare(g, r, len(body), body)
        assert g["visits"] == r["visits"]  # identical traversal => identical node visits
        # re-fit at a moved state, reusing the cached neighbours (nearest_search_en = false)
        st2 = dict(st)
        st2["pos"] = st["pos"] + np.array([0.01, -0.02, 0.005])
        g2 = ctx100k.h_share(sid, st2, search_en=False)
        r2 = tree100k.h_share(body, st2["rot"], st2["pos"], np.eye(3), synth.T_LI, False, cache=r["cache"])
        _hshare_compare(g2, r2, len(body), body)
    finally:
        ctx100k.scan_release(sid)


def _iekf_compare(gpu_ctx, tree, body, st0, max_iter, t_LI):
    gpu_ctx.set_params(max_iterations=max_iter)
    sid = gpu_ctx.scan_upload(body)
    try:
        sg, stg = gpu_ctx.iekf_update(sid, st0)
    finally:
        gpu_ctx.scan_release(sid)
    sr, str_ = tree.iekf_update(body, st0, R_LI=np.eye(3), t_LI=t_LI, max_iter=max_iter)
    assert stg["iterations"] == str_["iterations"]
    assert stg["knn_passes"] == str_["knn_passes"]
    assert stg["converged"] == str_["converged"]
    assert stg["effct_feat_num"] == str_["effct_feat_num"]
    for e in range(stg["iterations"]):
        assert _rel(stg["solution"][e], str_["solution"][e]) < REL_STATE, e
    # final state: rotation / position change relative to the update
    dth_g = np.linalg.norm(st0["rot"].T @ sg["rot"] - st0["rot"].T @ sr["rot"])
    assert dth_g < REL_STATE * max(np.linalg.norm(str_["solution"][:, :3]), 1e-12)
    assert _rel(sg["pos"] - st0["pos"], sr["pos"] - st0["pos"]) < REL_STATE
    # covariance: (I - G) P cancels ~6 orders of magnitude in the pose block; the
    # GPU's Woodbury form and the reference's two inversions agree to rounding
    # relative to the prior covariance
    assert np.linalg.norm(sg["cov"] - sr["cov"]) / np.linalg.norm(st0["cov"]) < 1e-9
    return stg


@pytest.mark.parametrize("max_iter", [4, 2, 0, 1, 10])
def test_iekf_parity_config1(ctx100k, tree100k, max_iter):
    synth = _synth()
    body, _, _ = synth.make_scan(10_000, 0)
    st0 = synth.make_state(0)
    _iekf_compare(ctx100k, tree100k, body, st0, max_iter, synth.T_LI)
    ctx100k.set_params(max_iterations=4)


def test_iekf_prior_differs(ctx100k, tree100k):
    """state_propagat != state: the prior term vec = prior ⊟ state is exercised."""
    synth = _synth()
    body, _, _ = synth.make_scan(5_000, 2)
    st0 = synth.make_state(2)
    prior = dict(st0)
    prior["pos"] = st0["pos"] + np.array([0.02, 0.0, -0.01])
    prior["rot"] = st0["rot"] @ synth.so3_exp(np.array([0.002, -0.001, 0.003]))
    prior["vel"] = np.array([0.5, 0.1, 0.0])
    sid = ctx100k.scan_upload(body)
    try:
        sg, stg = ctx100k.iekf_update(sid, st0, prior)
    finally:
        ctx100k.scan_release(sid)
    import oracle
    sr, str_ = tree100k.iekf_update(body, st0, prior, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4)
    assert stg["iterations"] == str_["iterations"]
    for e in range(stg["iterations"]):
        assert _rel(stg["solution"][e], str_["solution"][e]) < REL_STATE
    assert _rel(sg["vel"], sr["vel"]) < REL_STATE


def test_batch_equals_single_and_deterministic(ctx100k):
    synth = _synth()
    sids, states = [], []
    for s in range(4):
        body, _, _ = synth.make_scan(3000 + 517 * s, s)
        sids.append(ctx100k.scan_upload(body))
        states.append(synth.make_state(s))
    try:
        b1, s1 = ctx100k.iekf_update_batch(sids, states)
        b2, s2 = ctx100k.iekf_update_batch(sids, states)
        for a, b in zip(b1, b2):  # run-to-run bitwise reproducible
            assert all(np.array_equal(a[k], b[k]) for k in a)
        for i, sid in enumerate(sids):
            one, st1 = ctx100k.iekf_update(sid, states[i])
            assert all(np.array_equal(one[k], b1[i][k]) for k in one)
            assert st1["effct_feat_num"] == s1[i]["effct_feat_num"]
    finally:
        for sid in sids:
            ctx100k.scan_release(sid)


@pytest.mark.parametrize("n", [0, 1, 5, 255, 257])
def test_ragged_scans(ctx100k, tree100k, n):
    synth = _synth()
    body, _, _ = synth.make_scan(max(n, 1), 3)
    body = body[:n]
    st0 = synth.make_state(3)
    sid = ctx100k.scan_upload(body)
    try:
        g = ctx100k.h_share(sid, st0, True)
        r = tree100k.h_share(body, st0["rot"], st0["pos"], np.eye(3), synth.T_LI, True)
        _hshare_compare(g, r, n, body)
        sg, stg = ctx100k.iekf_update(sid, st0)
        assert stg["iterations"] >= 1
    finally:
        ctx100k.scan_release(sid)


def test_bad_args(ctx100k):
    import livo_amd
    with pytest.raises(livo_amd.LivoError):
        ctx100k.scan_release(12345)
    with pytest.raises(livo_amd.LivoError):
        ctx100k.iekf_update(9999, _synth().make_state(0))


@pytest.mark.slow
def test_config2_full_size_1M(built):
    """100k-point scan vs 1M-point map (BASELINE configs[1]/[2]): full parity."""
    import livo_amd
    import oracle
    synth = _synth()
    m = synth.cached_map(1_000_000)
    tree = oracle.Tree(m)
    body, _, _ = synth.make_scan(100_000, 0)
    st0 = synth.make_state(0)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=2) as ctx:
        ctx.map_build(m)
        assert ctx.map_info()["depth"] == 20
        stg = _iekf_compare(ctx, tree, body, st0, 2, synth.T_LI)  # config 3: 3 IEKF iterations
        assert stg["iterations"] == 3
        stg = _iekf_compare(ctx, tree, body, st0, 4, synth.T_LI)  # config 2
        sid = ctx.scan_upload(body)
        g = ctx.h_share(sid, st0, True)
        r = tree.h_share(body, st0["rot"], st0["pos"], np.eye(3), synth.T_LI, True)
        _hshare_compare(g, r, len(body))
        assert g["visits"] == r["visits"]


@pytest.mark.slow
def test_config5_10M_properties(built):
    """10M-point map, 200k-point scan: size-independent properties + a sampled oracle check."""
    import livo_amd
    import oracle
    synth = _synth()
    m = synth.cached_map(10_000_000)
    body, _, _ = synth.make_scan(200_000, 5)
    st0 = synth.make_state(5)
    with livo_amd.Context(0, t_LI=synth.T_LI) as ctx:
        ctx.map_build(m)
        q = ((body.astype(np.float64) + synth.T_LI) @ st0["rot"].T + st0["pos"]).astype(np.float32)
        idx, d = ctx.knn(q, 5)
        assert np.all(idx >= 0) and np.all(np.diff(d, axis=1) >= 0)
        p = m[idx]
        dd = ((q[:, None, 0] - p[..., 0]) ** 2 + (q[:, None, 1] - p[..., 1]) ** 2) + (q[:, None, 2] - p[..., 2]) ** 2
        assert np.array_equal(dd.astype(np.float32), d)
        tree = oracle.Tree(m)
        sample = np.random.default_rng(0).choice(len(q), 4000, replace=False)
        ridx, rd, _ = tree.knn(q[sample], 5, threads=8)
        assert np.array_equal(idx[sample], ridx) and np.array_equal(d[sample], rd)
        sid = ctx.scan_upload(body)
        sg, stg = ctx.iekf_update(sid, st0)
        assert stg["iterations"] >= 2 and stg["effct_feat_num"][0] > 150_000
        # the full IEKF update against the oracle's at 10M / 200k: counts exact,
        # per-evaluation state delta within the north_star's 1e-5
        sr, str_ = tree.iekf_update(body, st0, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4, threads=8)
        assert stg["iterations"] == str_["iterations"]
        assert stg["knn_passes"] == str_["knn_passes"]
        assert stg["effct_feat_num"] == str_["effct_feat_num"]
        for e in range(stg["iterations"]):
            assert _rel(stg["solution"][e], str_["solution"][e]) < REL_STATE, e
        assert _rel(sg["pos"] - st0["pos"], sr["pos"] - st0["pos"]) < REL_STATE


@pytest.mark.slow
def test_config5_batch_voxelgrid(built):
    """Config 5 as the bench runs it: 8 raw still frames -> the device VoxelGrid
    at leaf 0.05 (~200k points each) -> ONE batched update of the 8 scans on the
    10M-point map (1.6M points: two stream groups by default).  Every scan
    against the oracle's update of the same downsampled points: iterations,
    k-NN passes, effective points exact, per-evaluation state delta within 1e-5."""
    import livo_amd
    import oracle
    synth = _synth()
    m = synth.cached_map(10_000_000)
    frames = [synth.make_config5_frame(1000 + s) for s in range(8)]
    states = [synth.make_state(1000 + s) for s in range(8)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids, downs = [], []
        for raw, poses, Re, pe in frames:
            sid, _, down = ctx.scan_preprocess(raw, poses, Re, pe, leaf_size=synth.CONFIG5_LEAF)
            sids.append(sid)
            downs.append(np.ascontiguousarray(down[:, :3]))
        assert sum(len(d) for d in downs) > 1_200_000  # the two-group default
        outs, stats = ctx.iekf_update_batch(sids, states)
    assert all(150_000 < len(d) < 260_000 for d in downs)
    tree = oracle.Tree(m)
    for s in range(8):
        sr, rs = tree.iekf_update(downs[s], states[s], R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4, threads=8)
        gs = stats[s]
        assert gs["iterations"] == rs["iterations"], s
        assert gs["knn_passes"] == rs["knn_passes"], s
        assert gs["effct_feat_num"] == rs["effct_feat_num"], s
        for e in range(gs["iterations"]):
            assert _rel(gs["solution"][e], rs["solution"][e]) < REL_STATE, (s, e)
        assert _rel(outs[s]["pos"] - states[s]["pos"], sr["pos"] - states[s]["pos"]) < REL_STATE, s


def test_iekf_duplicate_map_replays(built):
    """Every map point duplicated: every k-NN answer hinges on PointType_CMP ties, so the
    fast pass flags the queries and the exact replay (reference heap + visiting order)
    must reproduce the oracle bit for bit, in the full and in the seeded rematch passes."""
    import livo_amd
    import oracle
    synth = _synth()
    base = synth.make_map(30_000)
    m = np.concatenate([base, base[::-1]])
    body, _, _ = synth.make_scan(4_000, 8)
    st0 = synth.make_state(8)
    tree = oracle.Tree(m)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sid = ctx.scan_upload(body)
        g = ctx.h_share(sid, st0, True)
        r = tree.h_share(body, st0["rot"], st0["pos"], np.eye(3), synth.T_LI, True)
        _hshare_compare(g, r, len(body))
        _iekf_compare(ctx, tree, body, st0, 4, synth.T_LI)


@pytest.mark.gpu
@pytest.mark.parametrize("leaf_size", [2, 5, 16, 64])
def test_iekf_leaf_size(built, map100k, tree100k, leaf_size, monkeypatch):
    """The batched IEKF searches the leaf map (LIVO_LEAF_SIZE points per leaf) and
    replays PointType_CMP-ambiguous queries on the ikd-Tree; any leaf size must give
    the oracle's answer."""
    import livo_amd
    synth = _synth()
    monkeypatch.setenv("LIVO_KNN_KIND", "leaf")
    monkeypatch.setenv("LIVO_LEAF_SIZE", str(leaf_size))
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(map100k)
        for scan_id in (3, 4):
            body, _, _ = synth.make_scan(7_777, scan_id)
            st0 = synth.make_state(scan_id)
            _iekf_compare(ctx, tree100k, body, st0, 4, synth.T_LI)


@pytest.mark.gpu
@pytest.mark.parametrize("n_map", [5, 17, 100, 1000])
def test_iekf_small_maps(built, n_map, monkeypatch):
    """Leaf maps of depth 0..6 (a single leaf up to many), IEKF against the oracle."""
    import livo_amd
    import oracle
    synth = _synth()
    monkeypatch.setenv("LIVO_KNN_KIND", "leaf")
    m = synth.make_map(100_000)[:: 100_000 // n_map][:n_map].copy()
    body, _, _ = synth.make_scan(2_000, 6)
    st0 = synth.make_state(6)
    tree = oracle.Tree(m)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sid = ctx.scan_upload(body)
        _, stg = ctx.iekf_update(sid, st0)
    _, str_ = tree.iekf_update(body, st0, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4)
    assert stg["iterations"] == str_["iterations"]
    assert stg["effct_feat_num"] == str_["effct_feat_num"]
    for e in range(stg["iterations"]):
        if np.linalg.norm(str_["solution"][e]) > 0:
            assert _rel(stg["solution"][e], str_["solution"][e]) < REL_STATE, e


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [1, 3, 4])
def test_batch_stream_groups(built, map100k, groups, monkeypatch):
    """A batch split over 1..4 stream groups (LIVO_STREAM_GROUPS) gives the single-scan results."""
    import livo_amd
    synth = _synth()
    monkeypatch.setenv("LIVO_STREAM_GROUPS", str(groups))
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(map100k)
        sids = [ctx.scan_upload(synth.make_scan(2500 + 301 * s, s)[0]) for s in range(5)]
        states = [synth.make_state(s) for s in range(5)]
        b, st = ctx.iekf_update_batch(sids, states)
        for i, sid in enumerate(sids):
            one, st1 = ctx.iekf_update(sid, states[i])
            assert all(np.array_equal(one[k], b[i][k]) for k in one)
            assert st1["iterations"] == st[i]["iterations"]


@pytest.mark.gpu
def test_slot_writeback_equals_copy(built, map100k, monkeypatch):
    """The stopping solve's slot write into the host staging copy (default) and the
    copy after the batch (LIVO_SLOT_WB=0) return the same states and stats, synchronous
    and submitted, an empty scan included."""
    import livo_amd
    synth = _synth()
    out = {}
    for wb in ("1", "0"):
        monkeypatch.setenv("LIVO_SLOT_WB", wb)
        with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
            ctx.map_build(map100k)
            scans = [synth.make_scan(2000 + 500 * s, s)[0] for s in range(6)] + [np.zeros((0, 3), np.float32)]
            sids = [ctx.scan_upload(sc) for sc in scans]
            states = [synth.make_state(s) for s in range(7)]
            b, st = ctx.iekf_update_batch(sids, states)
            t = ctx.iekf_update_batch_submit(sids[:3], states[:3])
            b2, st2 = ctx.iekf_update_batch_wait(t, 3)
            out[wb] = (b, st, b2, st2)
    for x, y in zip(out["1"], out["0"]):
        for u, v in zip(x, y):
            for k in u:
                assert np.asarray(u[k]).tobytes() == np.asarray(v[k]).tobytes(), k  # (bitwise: NaN stats of the empty scan)


@pytest.mark.gpu
def test_profiling_levels(ctx100k):
    """Profiling level 1 times only the batch's first search, level 2 every stage; neither
    changes the results."""
    synth = _synth()
    sids = [ctx100k.scan_upload(synth.make_scan(3000, s)[0]) for s in range(3)]
    states = [synth.make_state(s) for s in range(3)]
    try:
        ref, _ = ctx100k.iekf_update_batch(sids, states)
        for level in (1, 2):
            ctx100k.set_profiling(level)
            out, _ = ctx100k.iekf_update_batch(sids, states)
            t = ctx100k.last_timings()
            ctx100k.set_profiling(0)
            assert t["knn_ms"] > 0 and t["knn_queries"] == 9000
            assert (t["plane_ms"] > 0) == (level == 2)  # plane pass + the solve of its last block
            for a, b in zip(out, ref):
                assert all(np.array_equal(a[k], b[k]) for k in a)
    finally:
        for sid in sids:
            ctx100k.scan_release(sid)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["grid", "tile"])
@pytest.mark.parametrize("cell", [0.0, 0.05, 0.3, 2.0])
def test_iekf_grid(built, map100k, tree100k, cell, kind, monkeypatch):
    """The cell-grid search (LIVO_KNN_KIND=grid, or tile: the same search with a
    wave's cells staged in LDS; LIVO_GRID_CELL metres, 0: chosen from the map)
    certifies the 5 nearest by ring distance and replays the rest on the
    ikd-Tree; any cell size must give the oracle's answer.  0.05 m cells make
    most waves' boxes too large for a tile and 2 m cells too many points: the
    global path."""
    import livo_amd
    synth = _synth()
    monkeypatch.setenv("LIVO_KNN_KIND", kind)
    monkeypatch.setenv("LIVO_GRID_CELL", str(cell))
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(map100k)
        ctx.set_profiling(1)  # fills last_timings (replay count)
        for scan_id in (3, 4):
            body, _, _ = synth.make_scan(7_777, scan_id)
            st0 = synth.make_state(scan_id)
            _iekf_compare(ctx, tree100k, body, st0, 4, synth.T_LI)
            t = ctx.last_timings()
            if cell in (0.0, 0.3):  # the grid answers nearly every query itself
                assert t["knn_replays"] <= 0.05 * t["knn_queries"], t


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["grid", "tile"])
@pytest.mark.parametrize("n_map", [5, 17, 1000])
def test_iekf_grid_small_maps(built, n_map, kind, monkeypatch):
    """Cell grids of a handful of points: lists that never fill are replayed."""
    import livo_amd
    import oracle
    synth = _synth()
    monkeypatch.setenv("LIVO_KNN_KIND", kind)
    m = synth.make_map(100_000)[:: 100_000 // n_map][:n_map].copy()
    body, _, _ = synth.make_scan(2_000, 6)
    st0 = synth.make_state(6)
    tree = oracle.Tree(m)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        _iekf_compare(ctx, tree, body, st0, 4, synth.T_LI)


@pytest.mark.gpu
def test_grid_batch_equals_leaf(built, map100k, monkeypatch):
    """Grid and leaf-map searches give bit-identical batched updates, including a
    scan shifted 30 m off the map (queries beyond the ring limit: replayed)."""
    import livo_amd
    synth = _synth()
    scans = [synth.make_scan(3000 + 211 * s, s)[0] for s in range(6)]
    scans[5] = scans[5] + np.float32(30.0)
    states = [synth.make_state(s) for s in range(6)]
    out = {}
    for kind in ("leaf", "grid", "tile"):
        monkeypatch.setenv("LIVO_KNN_KIND", kind)
        with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
            ctx.map_build(map100k)
            sids = [ctx.scan_upload(b) for b in scans]
            out[kind] = ctx.iekf_update_batch(sids, states)
            out[kind + "_nn"] = [ctx.scan_neighbors(sid) for sid in sids]
    for kind in ("grid", "tile"):
        for i in range(6):
            a, b = out["leaf"][0][i], out[kind][0][i]
            assert all(np.array_equal(a[k], b[k]) for k in a), (kind, i)
            assert out["leaf"][1][i]["iterations"] == out[kind][1][i]["iterations"]
            np.testing.assert_array_equal(out["leaf_nn"][i][0], out[kind + "_nn"][i][0])
            np.testing.assert_array_equal(out["leaf_nn"][i][1], out[kind + "_nn"][i][1])


def _tie_map(seed=7, n_base=20_000, n_q=2_000):
    """Dyadic map + queries where each query has 2 or 4 map points at exactly the
    same float distance (mirror pairs q +- v, q +- v' with v' = v with x, y swapped)."""
    rng = np.random.default_rng(seed)
    g = 2.0 ** -8
    base = rng.integers(0, 16 * 256, size=(n_base, 3)) * g
    q = rng.integers(256, 15 * 256, size=(n_q, 3)) * g
    v = rng.integers(1, 4, size=(n_q, 3)) * rng.choice([-1, 1], size=(n_q, 3)) * g
    v[:, 1] = np.sign(v[:, 1]) * ((np.abs(v[:, 0]) / g) % 3 + 1) * g  # |vx| != |vy|: distinct x
    vp = v[:, [1, 0, 2]]
    four = np.arange(n_q) % 2 == 0
    extra = [q + v, q - v, (q + vp)[four], (q - vp)[four]]
    m = np.concatenate([base] + extra).astype(np.float32)
    return m, q.astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["leaf", "grid", "tile"])
def test_exact_ties_resolved_in_kernel(built, kind, monkeypatch):
    """Exact distance ties inside the 5-NN list (distinct x) are ordered by
    PointType_CMP's x rule in the batched search itself, without the replay; the
    neighbour cache must equal the reference heap's Nearest_Search order."""
    import livo_amd
    import oracle
    m, q = _tie_map()
    monkeypatch.setenv("LIVO_KNN_KIND", kind)
    st0 = {"rot": np.eye(3), "pos": np.zeros(3), "vel": np.zeros(3), "bias_g": np.zeros(3),
           "bias_a": np.zeros(3), "gravity": np.array([0.0, 0.0, -9.81]), "cov": np.eye(18) * 1e-3}
    with livo_amd.Context(0, t_LI=[0.0, 0.0, 0.0], max_iterations=0) as ctx:
        ctx.map_build(m)
        ctx.set_profiling(1)
        sid = ctx.scan_upload(q)
        ctx.iekf_update(sid, st0)  # one evaluation: the search at the identity pose
        replays = ctx.last_timings()["knn_replays"]
        idx_g, d_g = ctx.scan_neighbors(sid)
    idx_r, d_r, _ = oracle.Tree(m).knn(q, 5)
    np.testing.assert_array_equal(d_g, d_r)
    np.testing.assert_array_equal(idx_g, idx_r)
    assert replays <= 0.01 * len(q), replays


def test_ball_runs_chunked_build(built, monkeypatch):
    """The ball runs built in anchor chunks (LIVO_BR_CHUNK forces ~8 of them on
    the 1M map) hold the runs of the one-pass build: same entry count, and a
    batch of scans on either map gives bit for bit the same updates (a run
    read at its chunk's place must equal the same run of the one-pass array)."""
    import livo_amd
    synth = _synth()
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(50_000, 700 + s)[0] for s in range(4)]
    states = [synth.make_state(700 + s) for s in range(4)]
    res = {}
    for chunk in (None, 1 << 23):
        if chunk is None:
            monkeypatch.delenv("LIVO_BR_CHUNK", raising=False)
        else:
            monkeypatch.setenv("LIVO_BR_CHUNK", str(chunk))
        with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
            ctx.map_build(m)
            info = ctx.map_info()
            sids = [ctx.scan_upload(b) for b in scans]
            res[chunk] = (info, ctx.iekf_update_batch(sids, states))
    i0, i1 = res[None][0], res[1 << 23][0]
    assert i0["ball_chunks"] == 1 and i1["ball_chunks"] >= 4, (i0, i1)
    assert i0["ball_entries"] == i1["ball_entries"] > 0
    for k in range(4):
        a = (res[None][1][0][k], res[None][1][1][k])
        b = (res[1 << 23][1][0][k], res[1 << 23][1][1][k])
        for f in ("rot", "pos", "cov"):
            assert np.array_equal(np.asarray(a[0][f]), np.asarray(b[0][f])), (k, f)
        assert np.array_equal(np.asarray(a[1]["solution"]), np.asarray(b[1]["solution"])), k
