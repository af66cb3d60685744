"""CPU tests of the iVox restatement (oracle/livo_oracle.cpp, section iVox) and of
the device's std::nth_element restatement (fast-livo-noted_amd/csrc/stl_select.h).

Parity status of the iVox backend: the reference ships no tests or fixtures
for it and cannot be built here (glog/PCL/Eigen absent), so the
restatement is pinned against independent numpy restatements of each
documented behaviour:
  * the candidate SET of GetClosestPoint (ivox3d.h:132-204) = the max_num
    smallest in-range points of the nearby grids, nearest first (continuous
    random data, so no ties);
  * AddPoints' LRU grid cache with eviction at capacity (ivox3d.h:256-281)
    against an OrderedDict restatement, point order included;
  * map_incremental's add / no-downsample / skip decision
    (laser_mapping.cpp:329-389) against numpy float32 arithmetic.
The ORDER of the candidates is libstdc++'s std::nth_element's, which the
oracle calls directly; the device restates it (stl_select.h), checked here
element for element against libstdc++ on 300k random arrays and Musser's
median-of-3 killer sequences (the heap-select branch).
"""
import collections
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_nth_element_restatement_matches_libstdcxx(tmp_path):
    exe = tmp_path / "sel_check"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "fast-livo-noted_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "sel_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe), "300000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 mismatches" in out.stdout


def _round_half_away(x):
    return np.where(x >= 0, np.floor(x + np.float32(0.5)), -np.floor(-x + np.float32(0.5)))


NEAR18 = [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, -1), (0, 0, 1), (1, 1, 0), (-1, 1, 0),
          (1, -1, 0), (-1, -1, 0), (1, 0, 1), (-1, 0, 1), (1, 0, -1), (-1, 0, -1), (0, 1, 1), (0, -1, 1),
          (0, 1, -1), (0, -1, -1)]


def _keys(p, res):
    inv = np.float32(1.0 / res)
    return _round_half_away(p.astype(np.float32) * inv).astype(np.int64)


@pytest.mark.parametrize("res", [0.2, 0.5])
def test_ivox_knn_set_matches_numpy(built, res):
    import oracle
    rng = np.random.default_rng(5)
    m = rng.uniform(-3, 3, size=(30_000, 3)).astype(np.float32)
    q = rng.uniform(-3.2, 3.2, size=(2_000, 3)).astype(np.float32)
    iv = oracle.Ivox(resolution=res, nearby_type=18)
    iv.add_points(m)
    idx, d, xyz, cnt = iv.knn(q, 5, 5.0)
    mk = _keys(m, res)
    grid = collections.defaultdict(list)
    for i, k in enumerate(map(tuple, mk)):
        grid[k].append(i)
    qk = _keys(q, res)
    for i in range(q.shape[0]):
        cand = []
        for dl in NEAR18:
            cand += grid.get((qk[i, 0] + dl[0], qk[i, 1] + dl[1], qk[i, 2] + dl[2]), [])
        cand = np.array(cand, np.int64)
        if cand.size:
            dd = m[cand] - q[i]
            dist = dd[:, 0] * dd[:, 0] + (dd[:, 1] * dd[:, 1] + dd[:, 2] * dd[:, 2])
            keep = dist.astype(np.float64) < 25.0
            cand, dist = cand[keep], dist[keep]
        if cand.size == 0:
            assert cnt[i] == -1
            continue
        o = np.argsort(dist, kind="stable")[:5]
        assert cnt[i] == min(5, cand.size)
        assert set(idx[i, :cnt[i]]) == set(cand[o].tolist())
        assert idx[i, 0] == cand[o[0]]  # the final nth_element(begin, begin, end): nearest first
        assert np.array_equal(np.sort(d[i, :cnt[i]]), dist[o])
        assert np.array_equal(xyz[i, :cnt[i]], m[idx[i, :cnt[i]]])


def test_ivox_lru_and_eviction_match_ordereddict(built):
    import oracle
    rng = np.random.default_rng(9)
    pts = rng.uniform(-1, 1, size=(4_000, 3)).astype(np.float32)
    for cap in (1, 7, 50, 10_000):
        iv = oracle.Ivox(resolution=0.3, nearby_type=6, capacity=cap)
        od = collections.OrderedDict()  # key -> [ids]; last = most recently used
        nid = 0
        for lo, hi in ((0, 1000), (1000, 1001), (1001, 4000)):
            iv.add_points(pts[lo:hi])
            for p in pts[lo:hi]:
                k = tuple(_keys(p[None], 0.3)[0])
                if k not in od:
                    od[k] = [nid]
                    if len(od) >= cap:
                        od.popitem(last=False)
                else:
                    od[k].append(nid)
                    od.move_to_end(k)
                nid += 1
        xyz, ids, gof, keys = iv.dump()
        exp_keys = list(reversed(od.keys()))
        assert [tuple(k) for k in keys] == exp_keys
        exp_ids = [i for k in exp_keys for i in od[k]]
        assert ids.tolist() == exp_ids
        assert np.array_equal(xyz, pts[np.array(exp_ids, np.int64)].reshape(-1, 3))
        assert iv.info()["num_grids"] == len(od)


def test_map_incremental_matches_numpy(built):
    import oracle
    from livo_amd import synth
    m = synth.make_map(100_000)
    iv = oracle.Ivox()
    iv.add_points(m)
    body, _, _ = synth.make_scan(4_000, 1)
    st = synth.make_state(1)
    cache = oracle.new_cache(body.shape[0])
    st1, _ = iv.iekf_update(body, st, cache, t_LI=synth.T_LI)
    n0 = iv.info()["num_points"]
    fs = 0.5
    cat, counts = iv.map_incremental(body, st1, cache, t_LI=synth.T_LI, filter_size_map=fs)
    # numpy restatement of laser_mapping.cpp:343-380
    pI = body.astype(np.float64) + synth.T_LI
    pw = ((st1["rot"] @ pI.T).T + st1["pos"]).astype(np.float32)
    f = np.float32(fs)
    c = (np.floor(pw / f) + np.float32(0.5)) * f
    near = cache["xyz"].reshape(-1, 5, 3)
    d0 = np.abs(near[:, 0] - c)
    nodown = np.all(d0.astype(np.float64) > 0.5 * fs, axis=1)

    def nrm(v):
        return np.sqrt(v[..., 0] * v[..., 0] + (v[..., 1] * v[..., 1] + v[..., 2] * v[..., 2]))
    dist = nrm(pw - c)
    dn = nrm(near - c[:, None, :])
    closer = np.any(dn.astype(np.float64) < dist[:, None].astype(np.float64) + 1e-6, axis=1)
    full = cache["cnt"] >= 5
    has = cache["cnt"] > 0
    exp = np.where(~has, 1, np.where(nodown, 2, np.where(full & closer, 0, 1)))
    assert np.array_equal(cat, exp)
    assert counts["added"] == int(np.sum(exp == 1)) and counts["no_downsample"] == int(np.sum(exp == 2))
    assert iv.info()["num_points"] == n0 + counts["added"] + counts["no_downsample"]
    # insertion order: points_to_add then point_no_need_downsample, each in point order
    xyz, ids, _, _ = iv.dump()
    new = ids >= n0
    order = np.argsort(ids[new])
    exp_pts = np.concatenate([pw[exp == 1], pw[exp == 2]])
    assert np.array_equal(xyz[new][order], exp_pts)


def test_ivox_iekf_converges(built):
    import oracle
    from livo_amd import synth
    m = synth.make_map(300_000)
    iv = oracle.Ivox()
    iv.add_points(m)
    body, _, _ = synth.make_scan(5_000, 2)
    st = synth.make_state(2)
    cache = oracle.new_cache(body.shape[0])
    st1, stats = iv.iekf_update(body, st, cache, t_LI=synth.T_LI)
    assert stats["effct_feat_num"][0] > 1000
    assert stats["iterations"] >= 2
    # a second search from the updated state re-finds about the same matches
    h = iv.h_share(body, st1["rot"], st1["pos"], np.eye(3), synth.T_LI, True, cache)
    assert h["effct"] >= 0.9 * stats["effct_feat_num"][-1]
