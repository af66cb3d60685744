"""GPU parity of the iVox backend and map_incremental.

The HIP path (through the C ABI) against the CPU oracle's IVox restatement
(oracle/livo_oracle.cpp, iVox section; pinned in tests/test_ivox_oracle.py):
  * GetClosestPoint: neighbour ids, squared distances AND their order (the
    order libstdc++'s nth_element leaves, which esti_plane's row order
    depends on), and the no-candidate case: bit-exact;
  * AddPoints: every grid's points, in insertion order: exact;
  * h_share / IEKF / map_incremental with the iVox backend: same bars as the
    ikd-Tree path (tests/test_gpu_parity.py): normals, flags, categories
    bit-exact, state delta 1e-5 relative, counts exact.
"""
import collections

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
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def ivctx(built):
    import livo_amd
    from livo_amd import synth
    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    ctx.set_backend(livo_amd.BACKEND_IVOX)
    yield ctx
    ctx.close()


def _pair(ctx, m, **kw):
    import oracle
    ctx.ivox_init(**kw)
    iv = oracle.Ivox(**kw)
    if m is not None and len(m):
        ctx.ivox_add_points(m)
        iv.add_points(m)
    return iv


def _world(body, st):
    synth = _synth()
    return ((body.astype(np.float64) + synth.T_LI) @ st["rot"].T + st["pos"]).astype(np.float32)


def _knn_equal(ctx, iv, q, max_num=5, max_range=5.0):
    gi, gd, gc = ctx.ivox_knn(q, max_num, max_range)
    ri, rd, _, rc = iv.knn(q, max_num, max_range)
    assert np.array_equal(gc, rc)
    assert np.array_equal(gi, ri)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))
    return gc


def test_ivox_knn_bit_exact_room(ivctx):
    synth = _synth()
    iv = _pair(ivctx, synth.make_map(300_000))
    info = ivctx.ivox_info()
    ri = iv.info()
    assert info["num_points"] == ri["num_points"] == 300_000
    assert info["num_grids"] == ri["num_grids"]
    body, _, _ = synth.make_scan(20_000, 3)
    q = _world(body, synth.make_state(3))
    cnt = _knn_equal(ivctx, iv, q)
    assert (cnt == 5).mean() > 0.5 and (cnt == -1).sum() >= 0
    rng = np.random.default_rng(1)
    far = rng.uniform(-100, 100, size=(2000, 3)).astype(np.float32)  # mostly nothing found
    cnt = _knn_equal(ivctx, iv, far)
    assert (cnt == -1).mean() > 0.5


@pytest.mark.parametrize("nearby,res,max_num,rng_m", [(0, 0.2, 5, 5.0), (6, 0.5, 3, 5.0), (26, 0.2, 5, 0.15),
                                                      (18, 1.0, 1, 5.0)])
def test_ivox_knn_options(ivctx, nearby, res, max_num, rng_m):
    rng = np.random.default_rng(nearby)
    m = rng.uniform(-4, 4, size=(60_000, 3)).astype(np.float32)
    iv = _pair(ivctx, m, resolution=res, nearby_type=nearby)
    q = rng.uniform(-4.5, 4.5, size=(8000, 3)).astype(np.float32)
    _knn_equal(ivctx, iv, q, max_num, rng_m)


def test_ivox_ties_and_dense_grids(ivctx):
    """Exact distance ties (duplicates, lattices) — the order is nth_element's —
    and grids far beyond the private candidate array (the overflow pass)."""
    rng = np.random.default_rng(4)
    lattice = (np.stack(np.meshgrid(*[np.arange(-10, 11)] * 3), -1).reshape(-1, 3) * 0.05).astype(np.float32)
    dense = np.repeat(rng.uniform(-0.05, 0.05, size=(300, 3)).astype(np.float32), 3, axis=0)  # one grid, dups
    m = np.concatenate([lattice, lattice[::7], dense, rng.uniform(-1, 1, size=(5000, 3)).astype(np.float32)])
    iv = _pair(ivctx, m)
    assert ivctx.ivox_info()["max_grid_points"] > 64
    q = np.concatenate([lattice[::5] + np.float32(0.025), lattice[::11], rng.uniform(-0.6, 0.6, size=(3000, 3))])
    _knn_equal(ivctx, iv, q.astype(np.float32))


def _dump_by_grid(xyz, ids, keys):
    g = collections.defaultdict(list)
    for p, i, k in zip(xyz, ids, map(tuple, keys)):
        g[k].append((int(i), tuple(p.tolist())))
    return g


def _oracle_by_grid(iv):
    xyz, ids, gof, keys = iv.dump()
    g = collections.defaultdict(list)
    for p, i, go in zip(xyz, ids, gof):
        g[tuple(keys[go])].append((int(i), tuple(p.tolist())))
    return g


def test_ivox_add_points_batches_match_oracle(ivctx):
    rng = np.random.default_rng(8)
    import oracle
    ivctx.ivox_init(resolution=0.3, nearby_type=18)
    iv = oracle.Ivox(resolution=0.3, nearby_type=18)
    for n in (1, 0, 777, 5000, 1, 20000, 3):
        pts = rng.normal(0, 2, size=(n, 3)).astype(np.float32)
        ivctx.ivox_add_points(pts)
        iv.add_points(pts)
    assert _dump_by_grid(*ivctx.ivox_dump()) == _oracle_by_grid(iv)
    assert ivctx.ivox_info()["ids_issued"] == iv.info()["ids_issued"]


@pytest.mark.parametrize("cap", [1, 7, 50, 200, 10_000])
def test_ivox_lru_eviction_matches_oracle(ivctx, cap):
    """IVox::AddPoints' LRU grid cache at capacity (ivox3d.h:256-281): batches
    that evict (untouched old grids: one device pass; grids the batch touches
    before or after an eviction: split at the eviction), including capacity 1
    (a new grid evicts itself).  Grids, their points, ids and the
    most-recently-used order equal the oracle's after every batch."""
    import oracle
    rng = np.random.default_rng(11 + cap)
    ivctx.ivox_init(resolution=0.5, nearby_type=6, capacity=cap)
    iv = oracle.Ivox(resolution=0.5, nearby_type=6, capacity=cap)
    near = rng.uniform(-2, 2, size=(3000, 3)).astype(np.float32)   # revisits grids
    far = rng.uniform(-40, 40, size=(3000, 3)).astype(np.float32)  # mostly new grids
    for pts in (near[:400], far[:1500], near[400:1000], far[1500:1501], near[1000:], far[1501:]):
        ivctx.ivox_add_points(pts)
        iv.add_points(pts)
        gx, gi, gk = ivctx.ivox_dump()
        rx, ri, rg, rk = iv.dump()
        assert np.array_equal(gi, ri)
        assert np.array_equal(gx.view(np.uint32), rx.view(np.uint32))
        assert np.array_equal(gk, rk[rg])
        assert ivctx.ivox_info()["num_grids"] == iv.info()["num_grids"]
    assert ivctx.ivox_info()["ids_issued"] == iv.info()["ids_issued"]
    # the searches see the evicted map
    q = rng.uniform(-3, 3, size=(2000, 3)).astype(np.float32)
    _knn_equal(ivctx, iv, q, max_range=5.0)


def test_ivox_lru_eviction_runs(ivctx):
    """A batch whose evictions run far past the capacity (a sweep of 2000 new
    grids at capacity 64), touching old grids just before they would be the
    LRU victim and re-touching grids evicted a few creations earlier: the
    device takes the longest prefix whose victims the prefix leaves untouched
    per pass (ivox3d.h:263-275), so the pass count stays near N / C, not one
    per eviction; grids, ids and order equal the oracle's after the batch."""
    import oracle
    cap = 64
    rng = np.random.default_rng(64)
    ivctx.ivox_init(resolution=1.0, nearby_type=6, capacity=cap)
    iv = oracle.Ivox(resolution=1.0, nearby_type=6, capacity=cap)
    a = np.stack([np.arange(cap - 1) + 0.5, np.full(cap - 1, 0.5), np.full(cap - 1, 0.5)], 1).astype(np.float32)
    ivctx.ivox_add_points(a)
    iv.add_points(a)
    pts = []
    retouch = 0
    for j in range(2000):
        pts.append((j + 0.5, 50.5, 0.5))                 # a new grid (one more eviction)
        if j % 4 == 1 and j < 120:                       # an old grid, newest first: touched before its turn
            pts.append((cap - 2 - j // 4 + 0.25, 0.5, 0.5))
        if j % 50 == 25:                                 # a sweep grid evicted or about to be
            pts.append((j - rng.integers(50, 90) + 0.5, 50.25, 0.5))
            retouch += 1
    b = np.asarray(pts, np.float32)
    before = ivctx.ivox_info()["add_passes"]
    ivctx.ivox_add_points(b)
    iv.add_points(b)
    passes = ivctx.ivox_info()["add_passes"] - before
    print(f"add_passes {passes}")
    gx, gi, gk = ivctx.ivox_dump()
    rx, ri, rg, rk = iv.dump()
    assert np.array_equal(gi, ri)
    assert np.array_equal(gx.view(np.uint32), rx.view(np.uint32))
    assert np.array_equal(gk, rk[rg])
    assert ivctx.ivox_info()["num_grids"] == iv.info()["num_grids"]
    assert passes <= 2 * 2000 // cap + 2 * retouch + 4, passes
    q = np.concatenate([rng.uniform(0, 2000, size=(500, 1)), np.full((500, 1), 50.5), np.full((500, 1), 0.5)], 1)
    _knn_equal(ivctx, iv, q.astype(np.float32), max_range=5.0)


def _hs_equal(g, r):
    assert np.array_equal(g["nn_idx"], r["cache"]["idx"])
    assert np.array_equal(g["nn_d"].view(np.uint32), r["cache"]["d"].view(np.uint32))
    assert np.array_equal(g["normvec"].view(np.uint32), r["normvec"].view(np.uint32))
    assert np.array_equal(g["sel"], r["sel"])
    assert g["effct"] == r["effct"]
    assert _rel(g["HTH"], r["HTH"]) < REL_HTH
    assert _rel(g["HTL"], r["HTL"]) < REL_HTH


def test_ivox_h_share_parity(ivctx):
    import oracle
    synth = _synth()
    iv = _pair(ivctx, synth.make_map(1_000_000))
    body, _, _ = synth.make_scan(20_000, 5)
    st = synth.make_state(5)
    sid = ivctx.scan_upload(body)
    try:
        cache = oracle.new_cache(len(body))
        g = ivctx.h_share(sid, st, search_en=True)
        r = iv.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True, cache)
        _hs_equal(g, r)
        assert g["effct"] > 5000
        st2 = dict(st)
        st2["pos"] = st["pos"] + np.array([0.02, 0.01, -0.01])
        g2 = ivctx.h_share(sid, st2, search_en=False)
        r2 = iv.h_share(body, st2["rot"], st2["pos"], np.eye(3), synth.T_LI, False, r["cache"])
        _hs_equal(g2, r2)
    finally:
        ivctx.scan_release(sid)


def _iekf_check(stg, sg, str_, sr, st0):
    assert stg["iterations"] == str_["iterations"]
    assert stg["knn_passes"] == str_["knn_passes"]
    assert stg["converged"] == str_["converged"]
    assert stg["effct_feat_num"] == str_["effct_feat_num"]
    for e in range(stg["iterations"]):
        assert _rel(stg["solution"][e], str_["solution"][e]) < REL_STATE, e
    assert _rel(sg["pos"] - st0["pos"], sr["pos"] - st0["pos"]) < REL_STATE
    assert np.linalg.norm(sg["cov"] - sr["cov"]) / np.linalg.norm(st0["cov"]) < 1e-9


@pytest.mark.parametrize("max_iter", [4, 2, 0])
def test_ivox_iekf_parity(ivctx, max_iter):
    import oracle
    synth = _synth()
    iv = _pair(ivctx, synth.make_map(1_000_000))
    ivctx.set_params(max_iterations=max_iter)
    try:
        for scan in (6, 7):
            body, _, _ = synth.make_scan(30_000, scan)
            st0 = synth.make_state(scan)
            sid = ivctx.scan_upload(body)
            try:
                sg, stg = ivctx.iekf_update(sid, st0)
            finally:
                ivctx.scan_release(sid)
            sr, str_ = iv.iekf_update(body, st0, oracle.new_cache(len(body)), t_LI=synth.T_LI, max_iter=max_iter)
            _iekf_check(stg, sg, str_, sr, st0)
    finally:
        ivctx.set_params(max_iterations=4)


def test_ivox_batch_equals_single(ivctx):
    synth = _synth()
    _pair(ivctx, synth.make_map(300_000))
    bodies = [synth.make_scan(n, 10 + k)[0] for k, n in enumerate((9_000, 1, 0, 12_345, 700))]
    sts = [synth.make_state(10 + k) for k in range(len(bodies))]
    # fresh uploads for the batch: a point with no candidate keeps its cached
    # neighbours (ivox3d.h:165-167), so a second update of the same scan differs
    sids = [ivctx.scan_upload(b) for b in bodies]
    sids2 = [ivctx.scan_upload(b) for b in bodies]
    try:
        singles = [ivctx.iekf_update(s, st) for s, st in zip(sids, sts)]
        batch_states, batch_stats = ivctx.iekf_update_batch(sids2, sts)
        for (s1, t1), s2, t2 in zip(singles, batch_states, batch_stats):
            assert t1["iterations"] == t2["iterations"] and t1["effct_feat_num"] == t2["effct_feat_num"]
            assert np.array_equal(s1["pos"], s2["pos"]) and np.array_equal(s1["rot"], s2["rot"])
    finally:
        for s in sids + sids2:
            ivctx.scan_release(s)


def test_map_incremental_and_odometry_sequence(ivctx):
    """First scan -> AddPoints(body) (laser_mapping.cpp:145-150); every later scan:
    Nearest_Points carried over by index, the IEKF update, map_incremental;
    states, categories and the whole map compared after every scan."""
    import oracle
    synth = _synth()
    ivctx.ivox_init()
    iv = oracle.Ivox()
    base = synth.make_map(200_000)
    ivctx.ivox_add_points(base)
    iv.add_points(base)
    first, _, _ = synth.make_scan(8_000, 20)
    ivctx.ivox_add_points(first)
    iv.add_points(first)
    prev_sid, cache = None, oracle.new_cache(0)
    for k, n in enumerate((10_000, 7_000, 12_000, 12_000)):
        body, _, _ = synth.make_scan(n, 21 + k)
        st0 = synth.make_state(21 + k)
        sid = ivctx.scan_upload(body)
        if prev_sid is not None:
            ivctx.scan_inherit_neighbors(sid, prev_sid)
            ivctx.scan_release(prev_sid)
        cache = oracle.resize_cache(cache, n)
        sg, stg = ivctx.iekf_update(sid, st0)
        sr, str_ = iv.iekf_update(body, st0, cache, t_LI=synth.T_LI)
        _iekf_check(stg, sg, str_, sr, st0)
        gi, _ = ivctx.scan_neighbors(sid)
        assert np.array_equal(gi, cache["idx"])
        # map_incremental at the (oracle's) updated state: identical inputs on both sides
        cat_g, cnt_g = ivctx.map_incremental(sid, sr, filter_size_map=0.5)
        cat_r, cnt_r = iv.map_incremental(body, sr, cache, t_LI=synth.T_LI, filter_size_map=0.5)
        assert np.array_equal(cat_g, cat_r) and cnt_g == cnt_r
        assert cnt_g["added"] > 0
        prev_sid = sid
    ivctx.scan_release(prev_sid)
    assert ivctx.ivox_info()["num_points"] == iv.info()["num_points"]
    assert _dump_by_grid(*ivctx.ivox_dump()) == _oracle_by_grid(iv)


def test_map_incremental_not_inited_adds_all(ivctx):
    import oracle
    synth = _synth()
    iv = _pair(ivctx, synth.make_map(100_000))
    body, _, _ = synth.make_scan(3_000, 30)
    st = synth.make_state(30)
    sid = ivctx.scan_upload(body)
    try:
        ivctx.h_share(sid, st, search_en=True)
        cat, cnt = ivctx.map_incremental(sid, st, ekf_inited=False)
        assert np.all(cat == 1) and cnt == {"added": 3000, "no_downsample": 0}
        cache = oracle.new_cache(len(body))
        iv.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True, cache)
        iv.map_incremental(body, st, cache, t_LI=synth.T_LI, ekf_inited=False)
        assert _dump_by_grid(*ivctx.ivox_dump()) == _oracle_by_grid(iv)
    finally:
        ivctx.scan_release(sid)


def test_ivox_backend_args(ivctx):
    import livo_amd
    with pytest.raises(livo_amd.LivoError):
        ivctx.ivox_init(nearby_type=5)
    with pytest.raises(livo_amd.LivoError):
        ivctx.set_backend(7)
    ivctx.ivox_init()
    with pytest.raises(livo_amd.LivoError):
        ivctx.ivox_knn(np.zeros((1, 3), np.float32), max_num=6)
    # IKFoM runs on the ikd-Tree h-model only
    synth = _synth()
    sid = ivctx.scan_upload(synth.make_scan(100, 0)[0])
    try:
        with pytest.raises(livo_amd.LivoError):
            ivctx.ikfom_update(sid, synth.make_ikfom_state(0))
    finally:
        ivctx.scan_release(sid)


def test_ivox_batch_overflow_groups(ivctx):
    """Coarse grids (1 m: every query outgrows the private candidate array), a
    batch split over concurrent stream groups: each group's overflow pass has
    its own scratch; the batch equals single updates and the oracle."""
    import oracle
    synth = _synth()
    iv = _pair(ivctx, synth.make_map(300_000), resolution=1.0)
    assert ivctx.ivox_info()["max_grid_points"] > 128
    bodies = [synth.make_scan(4_000, 40 + k)[0] for k in range(6)]
    sts = [synth.make_state(40 + k) for k in range(6)]
    sids = [ivctx.scan_upload(b) for b in bodies]
    sids2 = [ivctx.scan_upload(b) for b in bodies]
    try:
        bs, bst = ivctx.iekf_update_batch(sids, sts)
        for k in (0, 5):
            s1, t1 = ivctx.iekf_update(sids2[k], sts[k])
            assert t1["effct_feat_num"] == bst[k]["effct_feat_num"]
            assert np.array_equal(s1["pos"], bs[k]["pos"])
            sr, tr = iv.iekf_update(bodies[k], sts[k], oracle.new_cache(len(bodies[k])), t_LI=synth.T_LI)
            _iekf_check(t1, s1, tr, sr, sts[k])
    finally:
        for s in sids + sids2:
            ivctx.scan_release(s)


def test_wave_nth_matches_libstdcxx(built):
    """The wave-parallel std::nth_element of the wave-cooperative iVox search
    (csrc/wave_select.h) against libstdc++ on the host, element for element:
    20000 cases of 1..256 elements, many ties, nonzero first."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fast-livo-noted_amd", "lib",
                       "wave_nth_check")
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


@pytest.mark.parametrize("kind", ["wave", "thread", "team"])
def test_ivox_kernel_kinds_agree(ivctx, kind, monkeypatch):
    """Every search kernel (wave or team chosen per launch by size; LIVO_IVOX_KIND
    forces one) gives the oracle's answer, in batch IEKF updates too."""
    import oracle
    synth = _synth()
    monkeypatch.setenv("LIVO_IVOX_KIND", kind)
    m = synth.make_map(200_000)
    iv = _pair(ivctx, m)
    rng = np.random.default_rng(3)
    q = (m[rng.choice(len(m), 30_000)] + rng.normal(0, 0.1, (30_000, 3))).astype(np.float32)
    _knn_equal(ivctx, iv, q)
    body, _, _ = synth.make_scan(20_000, 50)
    st0 = synth.make_state(50)
    sid = ivctx.scan_upload(body)
    try:
        sg, stg = ivctx.iekf_update(sid, st0)
    finally:
        ivctx.scan_release(sid)
    sr, str_ = iv.iekf_update(body, st0, oracle.new_cache(len(body)), t_LI=synth.T_LI)
    _iekf_check(stg, sg, str_, sr, st0)
