"""The C++ facade (fast-livo-noted_amd/host/laser_mapping_gpu.hpp) driven like LaserMapping::Run.

host/facade_demo.cpp calls h_share_model(HPH, HPL) and the IEKF loop through
LaserMappingGpu with Eigen-shaped column-major matrices; its printed results
are compared with the oracle (CPU restatement).  Without a GPU the facade must
fail loudly: livo::Error carrying LIVO_E_HIP, exit status 3, no CPU fallback.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "fast-livo-noted_amd", "lib", "facade_demo")


def _inputs(tmp_path, n_map=100_000, n_scan=10_000, scan_id=2):
    from livo_amd import synth
    m = synth.make_map(n_map)
    body, _, _ = synth.make_scan(n_scan, scan_id)
    st = synth.make_state(scan_id)
    mp, sp, tp = (str(tmp_path / f) for f in ("map.f32", "scan.f32", "state.f64"))
    np.ascontiguousarray(m, np.float32).tofile(mp)
    np.ascontiguousarray(body, np.float32).tofile(sp)
    np.concatenate([st["rot"].ravel(), st["pos"], st["vel"], st["bias_g"], st["bias_a"], st["gravity"],
                    st["cov"].ravel()]).astype(np.float64).tofile(tp)
    return m, body, st, (mp, sp, tp)


def test_facade_demo_built(built):
    assert os.access(DEMO, os.X_OK)


def test_facade_usage_error(built):
    r = subprocess.run([DEMO], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_facade_fails_loudly_without_gpu(built, tmp_path):
    import livo_amd
    try:
        livo_amd.Context(0).close()
        pytest.skip("a GPU is present")
    except livo_amd.LivoError:
        pass
    _, _, _, files = _inputs(tmp_path, n_map=2000, n_scan=500)
    r = subprocess.run([DEMO, *files, "4"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "livo::Error -2" in r.stderr


@pytest.mark.gpu
def test_facade_matches_oracle(built, tmp_path):
    import oracle
    from livo_amd import synth
    m, body, st, files = _inputs(tmp_path)
    r = subprocess.run([DEMO, *files, "4"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}
    hs = np.array(lines["hshare"], dtype=np.float64)
    tree = oracle.Tree(m)
    ref = tree.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True)
    assert int(hs[0]) == ref["effct"]
    hth, htl = hs[1:82].reshape(9, 9), hs[82:91]
    assert np.linalg.norm(hth - ref["HTH"]) <= 1e-9 * np.linalg.norm(ref["HTH"])
    assert np.linalg.norm(htl - ref["HTL"]) <= 1e-9 * np.linalg.norm(ref["HTL"])

    it = np.array(lines["iekf"], dtype=np.float64)
    sr, rs = tree.iekf_update(body, st, R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4)
    assert int(it[0]) == rs["iterations"] and int(it[1]) == rs["converged"]
    rot, pos, cov = it[2:11].reshape(3, 3), it[11:14], it[14:14 + 324].reshape(18, 18)
    upd = np.linalg.norm(sr["pos"] - st["pos"])
    assert np.linalg.norm(pos - sr["pos"]) <= 1e-5 * upd
    assert np.linalg.norm(rot - sr["rot"]) <= 1e-5 * max(np.linalg.norm(rs["solution"][:, :3]), 1e-12)
    assert np.linalg.norm(cov - sr["cov"]) <= 1e-9 * np.linalg.norm(st["cov"])


@pytest.mark.gpu
def test_facade_ivox_matches_oracle(built, tmp_path):
    """The default-build flow through the facade: use_ivox + AddPoints, h_share_model,
    the IEKF loop, map_incremental — against the oracle's IVox restatement."""
    import oracle
    from livo_amd import synth
    m, body, st, files = _inputs(tmp_path, n_map=300_000)
    r = subprocess.run([DEMO, *files, "4", "ivox"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}
    iv = oracle.Ivox()
    iv.add_points(m)
    hs = np.array(lines["hshare"], dtype=np.float64)
    ref = iv.h_share(body, st["rot"], st["pos"], np.eye(3), synth.T_LI, True, oracle.new_cache(len(body)))
    assert int(hs[0]) == ref["effct"]
    assert np.linalg.norm(hs[1:82].reshape(9, 9) - ref["HTH"]) <= 1e-9 * np.linalg.norm(ref["HTH"])
    cache = oracle.new_cache(len(body))
    sr, rs = iv.iekf_update(body, st, cache, t_LI=synth.T_LI, max_iter=4)
    it = np.array(lines["iekf"], dtype=np.float64)
    assert int(it[0]) == rs["iterations"] and int(it[1]) == rs["converged"]
    assert np.linalg.norm(it[11:14] - sr["pos"]) <= 1e-5 * np.linalg.norm(sr["pos"] - st["pos"])
    # map_incremental ran at the GPU's updated state: same categories up to that state's rounding
    _, cnt = iv.map_incremental(body, sr, cache, t_LI=synth.T_LI, filter_size_map=0.5)
    got = [int(x) for x in lines["incr"]]
    assert abs(got[0] - cnt["added"]) <= 2 and abs(got[1] - cnt["no_downsample"]) <= 2
