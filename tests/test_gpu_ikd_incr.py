"""GPU parity of the ikd-Tree incremental map (the
USE_ikdtree branch of map_incremental, laser_mapping.cpp:383-384, i.e.
KD_TREE::Add_Points with downsampling, ikd_Tree.cpp:382-457, and
Delete_Point_Boxes, :501-521): livo_map_add_points / livo_map_incremental /
livo_map_delete_boxes against the oracle's restatement (pinned in
tests/test_ikd_incr_oracle.py).

Bars: the map after every call (ids and coordinates, bit for bit) and the
call's counts (Add_Points' return value, points kept, points deleted, centre
ties) exact; k-NN of the updated map (indices, squared distances and order)
bit-exact; IEKF updates on the updated map: counts exact, state delta 1e-5
relative (north_star tolerance).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
f32 = np.float32
REL_STATE = 1e-5
KEYS = ("events", "added", "deleted", "ambiguous")


@pytest.fixture(scope="module")
def ictx(built):
    import livo_amd
    from livo_amd import synth
    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    yield ctx
    ctx.close()


def _world(body, st):
    from livo_amd import synth
    return ((body.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(f32)


def _pair(ctx, m):
    import oracle
    ctx.map_build(m)
    return oracle.DynMap(m)


def _same_map(ctx, dm):
    gx, gi = ctx.map_dump()
    rx, ri = dm.dump()
    assert np.array_equal(gi, ri)
    assert np.array_equal(gx.view(np.uint32), rx.view(np.uint32))


def _same_add(g, r):
    assert {k: g[k] for k in KEYS} == r, (g, r)


@pytest.mark.parametrize("ds", [0.5, 0.3])
def test_add_points_room(ictx, ds):
    from livo_amd import synth
    m = synth.make_map(200_000)
    dm = _pair(ictx, m)
    for sid in (0, 1):
        body, _, _ = synth.make_scan(20_000, sid)
        W = _world(body, synth.make_state(sid))
        g = ictx.map_add_points(W, ds)
        _same_add(g, dm.add_points(W, ds))
        assert g["map_points"] == len(dm.dump()[1]) == ictx.map_info()["num_points"]
        _same_map(ictx, dm)


def test_add_points_box_faces_duplicates_and_ties(ictx):
    """Points within ulps of box faces (the in-order pass), duplicates, centre ties, no-downsample adds."""
    from livo_amd import synth
    rng = np.random.default_rng(31)
    deferred = amb = 0
    for ds in (0.5, 0.3):
        pairs, far = synth.centre_tie_points(ds)
        m = np.concatenate([rng.uniform(-6, 6, (3000, 3)), synth.boundary_points(rng, ds, 600, span=12), pairs])
        m = np.concatenate([m, m[:20]]).astype(f32)
        dm = _pair(ictx, m)
        for rep in range(4):
            W = np.concatenate([rng.uniform(-6, 6, (800, 3)), synth.boundary_points(rng, ds, 400, span=12),
                                m[rng.choice(len(m), 40)], far]).astype(f32)
            W = W[rng.permutation(len(W))]
            down = rep != 2
            g = ictx.map_add_points(W, ds, downsample=down)
            _same_add(g, dm.add_points(W, ds, downsample=down))
            deferred += g["deferred"]
            amb += g["ambiguous"]
            _same_map(ictx, dm)
    assert deferred > 0 and amb > 0  # both special paths ran


def test_add_points_empty_and_tiny_maps(ictx):
    rng = np.random.default_rng(5)
    for M in (0, 1, 4):
        m = rng.uniform(-1, 1, (M, 3)).astype(f32)
        dm = _pair(ictx, m)
        for _ in range(3):
            W = rng.uniform(-2, 2, (50, 3)).astype(f32)
            _same_add(ictx.map_add_points(W, 0.5), dm.add_points(W, 0.5))
            _same_map(ictx, dm)
        q = rng.uniform(-3, 3, (100, 3)).astype(f32)
        gi, gd = ictx.knn(q)
        ri, rd = dm.knn(q)
        assert np.array_equal(gi, ri) and np.array_equal(gd, rd)


def test_knn_after_add_and_delete(ictx):
    from livo_amd import synth
    rng = np.random.default_rng(9)
    m = synth.make_map(100_000)
    dm = _pair(ictx, m)
    body, _, _ = synth.make_scan(20_000, 3)
    W = _world(body, synth.make_state(3))
    ictx.map_add_points(W, 0.3)
    dm.add_points(W, 0.3)
    boxes = np.array([[-5, -5, -2, 0, 0, 3], [10, 10, -2, 12, 12, 3]], f32)
    assert ictx.map_delete_boxes(boxes) == dm.delete_boxes(boxes)
    _same_map(ictx, dm)
    P, _ = dm.dump()
    q = np.concatenate([W[:5000], P[:2000], rng.uniform([-32, -22, -2], [32, 22, 3], (3000, 3))]).astype(f32)
    gi, gd = ictx.knn(q)
    ri, rd = dm.knn(q)
    assert np.array_equal(gi, ri)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))


def test_iekf_on_updated_map(ictx):
    from livo_amd import synth
    m = synth.make_map(100_000)
    dm = _pair(ictx, m)
    body0, _, _ = synth.make_scan(20_000, 0)
    W = _world(body0, synth.make_state(0))
    ictx.map_add_points(W, 0.5)
    dm.add_points(W, 0.5)
    body, _, _ = synth.make_scan(10_000, 1)
    st = synth.make_state(1)
    sid = ictx.scan_upload(body)
    gs, gst = ictx.iekf_update(sid, st)
    rs, rst = dm.iekf_update(body, st, t_LI=synth.T_LI, max_iter=4)
    assert gst["iterations"] == rst["iterations"] and gst["effct_feat_num"] == rst["effct_feat_num"]
    for e in range(gst["iterations"]):
        rel = np.linalg.norm(gst["solution"][e] - rst["solution"][e]) / np.linalg.norm(rst["solution"][e])
        assert rel < REL_STATE, (e, rel)
    # the batched loop (4 stream groups) on the same map gives the same updates
    sids = [sid] + [ictx.scan_upload(synth.make_scan(10_000, k)[0]) for k in (2, 3, 4)]
    sts = [st] + [synth.make_state(k) for k in (2, 3, 4)]
    _, bst = ictx.iekf_update_batch(sids, sts)
    assert bst[0]["iterations"] == gst["iterations"] and np.array_equal(bst[0]["solution"], gst["solution"])
    for s in sids:
        ictx.scan_release(s)


def test_odometry_with_ikd_map_incremental(ictx):
    """LaserMapping::Run with USE_ikdtree: per scan the IEKF update, then map_incremental
    (Add_Points of feats_down_world at the updated state)."""
    from livo_amd import synth
    m = synth.make_map(100_000)
    dm = _pair(ictx, m)
    for k in range(4):
        body, _, _ = synth.make_scan(20_000, 10 + k)
        st0 = synth.make_state(10 + k)
        sid = ictx.scan_upload(body)
        gs, gst = ictx.iekf_update(sid, st0)
        rs, rst = dm.iekf_update(body, st0, t_LI=synth.T_LI, max_iter=4)
        assert gst["iterations"] == rst["iterations"] and gst["effct_feat_num"] == rst["effct_feat_num"]
        assert np.linalg.norm(gs["pos"] - rs["pos"]) <= REL_STATE * max(np.linalg.norm(rs["pos"] - st0["pos"]), 1e-9)
        # both maps take the points at the GPU's updated state
        cat, g = ictx.map_incremental(sid, gs, filter_size_map=0.3)
        assert np.all(cat == 1)
        _same_add(g, dm.map_incremental(body, gs, t_LI=synth.T_LI, filter_size_map=0.3))
        _same_map(ictx, dm)
        ictx.scan_release(sid)


def test_add_points_crowded_boxes(ictx):
    """Boxes with hundreds of new points (the wave-per-box pass), exact duplicates among them
    (equal distances: the later point wins, ikd_Tree.cpp:405-411) and stored points inside."""
    rng = np.random.default_rng(77)
    m = rng.uniform(0, 1, (50, 3)).astype(f32)
    dm = _pair(ictx, m)
    for rep in range(3):
        W = rng.uniform(0, 1, (3000, 3)).astype(f32)
        W = np.concatenate([W, W[rng.choice(3000, 500)], np.full((40, 3), 0.25, f32)])
        W = W[rng.permutation(len(W))]
        _same_add(ictx.map_add_points(W, 0.5), dm.add_points(W, 0.5))
        _same_map(ictx, dm)


@pytest.mark.parametrize("mode", ["runs", "rebase_every_change", "cell_walk"])
def test_iekf_search_records_on_updated_map(built, monkeypatch, mode):
    """The fused IEKF search on the incremental map: with the runs of the base
    point set (deleted base points marked, points added since in the delta
    grid), with a rebase of the runs at every change (LIVO_DYN_REBASE tiny),
    and with the cell walk (the default; the runs are LIVO_DYN_RUNS=1).  One evaluation (max_iteration
    0: one search at the initial state) after each change: every point's
    neighbour record (indices and squared distances, in order) equals the
    oracle's k-NN of the world points on the updated map, bit for bit."""
    import livo_amd
    import oracle
    from livo_amd import synth
    monkeypatch.setenv("LIVO_DYN_RUNS", "0" if mode == "cell_walk" else "1")  # (the runs are opt-in)
    if mode == "rebase_every_change":
        monkeypatch.setenv("LIVO_DYN_REBASE", "1e-9")
    m = synth.make_map(200_000)
    dm = oracle.DynMap(m)
    rng = np.random.default_rng(77)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=0) as ctx:
        ctx.map_build(m)
        for k in range(4):
            body, _, _ = synth.make_scan(20_000, 40 + k)
            W = _world(body, synth.make_state(40 + k))
            _same_add(ctx.map_add_points(W, 0.3), dm.add_points(W, 0.3))
            if k == 1:
                c = rng.uniform([-20, -12, 0], [20, 12, 2], (3, 3))
                boxes = np.concatenate([c, c + 3.0], axis=1).astype(f32)
                assert ctx.map_delete_boxes(boxes) == dm.delete_boxes(boxes)
            q_body, _, _ = synth.make_scan(15_000, 60 + k)
            st = synth.make_state(60 + k)
            sid = ctx.scan_upload(q_body)
            _, gst = ctx.iekf_update(sid, st)
            _, rst = dm.iekf_update(q_body, st, t_LI=synth.T_LI, max_iter=0)
            assert gst["iterations"] == rst["iterations"] == 1
            assert gst["effct_feat_num"] == rst["effct_feat_num"]
            gi, gd = ctx.scan_neighbors(sid)
            ri, rd = dm.knn(oracle.to_world(q_body, st, np.eye(3), synth.T_LI)[:, :3])
            assert np.array_equal(gi, ri), (mode, k, int((gi != ri).any(axis=1).sum()))
            assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))
            ctx.scan_release(sid)


def test_odometry_with_rebases(built, monkeypatch):
    """The odometry loop of test_odometry_with_ikd_map_incremental with the runs
    rebuilt after every map change (LIVO_DYN_REBASE tiny): same updates as the oracle."""
    import livo_amd
    import oracle
    from livo_amd import synth
    monkeypatch.setenv("LIVO_DYN_RUNS", "1")
    monkeypatch.setenv("LIVO_DYN_REBASE", "1e-9")
    m = synth.make_map(100_000)
    dm = oracle.DynMap(m)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        for k in range(3):
            body, _, _ = synth.make_scan(20_000, 20 + k)
            st0 = synth.make_state(20 + k)
            sid = ctx.scan_upload(body)
            gs, gst = ctx.iekf_update(sid, st0)
            rs, rst = dm.iekf_update(body, st0, t_LI=synth.T_LI, max_iter=4)
            assert gst["iterations"] == rst["iterations"] and gst["effct_feat_num"] == rst["effct_feat_num"]
            for e in range(gst["iterations"]):
                rel = np.linalg.norm(gst["solution"][e] - rst["solution"][e]) / np.linalg.norm(rst["solution"][e])
                assert rel < REL_STATE, (k, e, rel)
            _same_add(ctx.map_incremental(sid, gs, filter_size_map=0.3)[1],
                      dm.map_incremental(body, gs, t_LI=synth.T_LI, filter_size_map=0.3))
            _same_map(ctx, dm)
            ctx.scan_release(sid)


def test_grid_merge_equals_sort(built, monkeypatch):
    """The grid rebuild after a change merges the added ids into the old grid
    (dyn_rebuild_merge) instead of sorting every id: over adds, a no-downsample
    add, box deletions and map_incremental, the map, its k-NN and the IEKF's
    neighbour records equal those with LIVO_DYN_MERGE=0 (a sort at every
    change) bit for bit, and the merge path ran."""
    import livo_amd
    from livo_amd import synth
    m = synth.make_map(100_000)
    rng = np.random.default_rng(12)
    q = rng.uniform([-32, -22, -2], [32, 22, 3], (4000, 3)).astype(f32)
    out = {}
    for merge in ("1", "0"):
        monkeypatch.setenv("LIVO_DYN_MERGE", merge)
        rec = []
        with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=0) as ctx:
            ctx.map_build(m)
            for k in range(5):
                body, _, _ = synth.make_scan(20_000, 70 + k)
                st = synth.make_state(70 + k)
                if k == 3:
                    sid = ctx.scan_upload(body)
                    rec.append(ctx.map_incremental(sid, st, filter_size_map=0.5)[1])
                    ctx.scan_release(sid)
                else:
                    rec.append(ctx.map_add_points(_world(body, st), 0.5, downsample=k != 2))
                if k == 1:
                    boxes = np.array([[-5, -5, -2, 0, 0, 3], [10, 10, -2, 12, 12, 3]], f32)
                    rec.append(ctx.map_delete_boxes(boxes))
                rec.append(ctx.map_dump())
                rec.append(ctx.knn(q))
                sid = ctx.scan_upload(synth.make_scan(15_000, 80 + k)[0])
                ctx.iekf_update(sid, synth.make_state(80 + k))
                rec.append(ctx.scan_neighbors(sid))
                ctx.scan_release(sid)
            out[merge] = (rec, ctx.map_rebuilds())
    (a, ra), (b, rb) = out["1"], out["0"]
    assert ra[1] >= 4 and rb[1] == 0, (ra, rb)
    assert ra[2] == rb[2] == 0 and ra[3] >= 1 and rb[3] == 0
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, tuple):
            for u, v in zip(x, y):
                assert np.array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
        else:
            assert x == y


def test_add_points_wrapped_box_key_clash(ictx):
    """The box keys sort as 30-bit keys (10 bits per axis, wrapped): boxes 1024
    boxes apart share a wrapped key, the batch is redone with the 64-bit keys,
    and the result equals the oracle's."""
    rng = np.random.default_rng(21)
    ds = 0.05
    m = rng.uniform(0, 2, (400, 3)).astype(f32)
    dm = _pair(ictx, m)
    base = rng.uniform(0, 2, (300, 3))
    W = np.concatenate([base, base[:40] + [1024 * ds, 0, 0], base[40:80] + [1024 * ds, 1024 * ds, 1024 * ds]])
    W = W[rng.permutation(len(W))].astype(f32)
    r0 = ictx.map_rebuilds()[2]
    _same_add(ictx.map_add_points(W, ds), dm.add_points(W, ds))
    _same_map(ictx, dm)
    assert ictx.map_rebuilds()[2] == r0 + 1
    W2 = rng.uniform(0, 2, (300, 3)).astype(f32)  # no clash: no redo
    _same_add(ictx.map_add_points(W2, ds), dm.add_points(W2, ds))
    _same_map(ictx, dm)
    assert ictx.map_rebuilds()[2] == r0 + 1


def test_add_points_wrapped_box_key_clash_fused(ictx):
    """The same clash on a call that takes the fused pass (the map has changed
    already, so the merged rebuild runs inside Add_Points' stream pass and
    refills the table with its bound's size): the 64-bit-key redo must read the
    grid's own table, so the map equals the oracle's, the redo ran and the
    fused rebuild ran in it."""
    rng = np.random.default_rng(22)
    ds = 0.05
    m = rng.uniform(0, 2, (400, 3)).astype(f32)
    dm = _pair(ictx, m)
    fused = False
    for _ in range(4):  # no clash; until the merged rebuild runs inside Add_Points' pass
        r0 = ictx.map_rebuilds()
        W1 = rng.uniform(0, 2, (200, 3)).astype(f32)
        _same_add(ictx.map_add_points(W1, ds), dm.add_points(W1, ds))
        _same_map(ictx, dm)
        if ictx.map_rebuilds()[3] == r0[3] + 1:
            fused = True
            break
    assert fused
    base = rng.uniform(0, 2, (120, 3))
    W = np.concatenate([base, base[:40] + [1024 * ds, 0, 0], base[40:80] + [1024 * ds, 1024 * ds, 1024 * ds]])
    W = W[rng.permutation(len(W))].astype(f32)
    r0 = ictx.map_rebuilds()
    _same_add(ictx.map_add_points(W, ds), dm.add_points(W, ds))
    _same_map(ictx, dm)
    r1 = ictx.map_rebuilds()
    assert r1[2] == r0[2] + 1  # redone with the 64-bit keys
    assert r1[3] == r0[3] + 1  # and the redo's merged rebuild ran in its pass
    for _ in range(2):  # later adds read the grid's table after the redo
        W3 = rng.uniform(0, 2, (150, 3)).astype(f32)
        _same_add(ictx.map_add_points(W3, ds), dm.add_points(W3, ds))
        _same_map(ictx, dm)
    q = rng.uniform(0, 2, (500, 3)).astype(f32)
    gi, gd = ictx.knn(q)
    ri, rd = dm.knn(q)
    assert np.array_equal(gi, ri)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))


def test_add_points_large_multi_tile(built):
    """Scans of 60k points into a 400k-point map: the one-launch scans span more
    than one 64-tile look-back window (k_scan_boxes ~118 tiles, the merged
    rebuild's survivor ranks ~196), the crowded boxes take whole waves and the
    kept list passes the LDS ranking's 2,048 (the in-order compaction): counts
    and the map bit for bit the oracle's after every call, the merge path ran."""
    import livo_amd
    import oracle
    from livo_amd import synth
    m = synth.make_map(400_000)
    dm = oracle.DynMap(m)
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        for k in range(3):
            body, _, _ = synth.make_scan(60_000, 90 + k)
            W = _world(body, synth.make_state(90 + k))
            _same_add(ctx.map_add_points(W, 0.5), dm.add_points(W, 0.5))
            _same_map(ctx, dm)
        assert ctx.map_rebuilds()[1] >= 2 and ctx.map_rebuilds()[3] >= 1  # merged, and inside Add_Points' pass
