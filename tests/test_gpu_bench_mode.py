"""GPU parity of the exact modes the bench measures and of the committed fixture.

  * the golden fixture (tests/golden/config1_small.npz, made by
    tests/golden/make_golden.py from the oracle): the HIP path through the
    C ABI reproduces it -- k-NN, normals, flags bit-exact; HᵀH 1e-9; the IEKF
    update's counts exact and its per-evaluation state delta within 1e-5;
  * the bench's headline mode (bench.py, config 2 as the config-4 shard of one
    GPU): 8 x 100k-point scans vs the 1M-point map in ONE batched call in
    the default stream grouping, every scan against the oracle's own update;
  * the bench's N-GPU launcher: `bench.py --gpus 2` starts two ranks (here
    sharing one GPU, gloo for the counter all-reduce) and reports both;
  * the farm's counter all-reduce over RCCL (backend "nccl") on device
    tensors at world size 1.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL_HTH = 1e-9
REL_STATE = 1e-5


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def test_golden_fixture(built):
    import livo_amd
    g = np.load(os.path.join(ROOT, "tests", "golden", "config1_small.npz"))
    st0 = {k[6:]: g[k] for k in g.files if k.startswith("state_")}
    with livo_amd.Context(0, t_LI=g["t_LI"], max_iterations=int(g["max_iter"])) as ctx:
        ctx.map_build(g["map"])
        sid = ctx.scan_upload(g["scan"])
        hs = ctx.h_share(sid, st0, search_en=True)
        assert np.array_equal(hs["nn_idx"], g["nn_idx"])
        assert np.array_equal(hs["nn_d"].view(np.uint32), g["nn_d"].view(np.uint32))
        assert np.array_equal(hs["normvec"].view(np.uint32), g["normvec"].view(np.uint32))
        assert np.array_equal(hs["sel"], g["sel"])
        assert hs["effct"] == int(g["effct"]) and hs["visits"] == int(g["visits"])
        assert _rel(hs["HTH"], g["HTH"]) < REL_HTH and _rel(hs["HTL"], g["HTL"]) < REL_HTH
        out, stats = ctx.iekf_update(sid, st0)
    assert stats["iterations"] == int(g["iterations"])
    assert stats["knn_passes"] == int(g["knn_passes"])
    assert stats["effct_feat_num"] == list(g["effct_feat_num"])
    for e in range(stats["iterations"]):
        assert _rel(stats["solution"][e], g["solution"][e]) < REL_STATE, e
    assert _rel(out["pos"] - st0["pos"], g["out_pos"] - st0["pos"]) < REL_STATE
    assert np.linalg.norm(out["cov"] - g["out_cov"]) / np.linalg.norm(st0["cov"]) < 1e-9


@pytest.mark.slow
@pytest.mark.parametrize("seed0,groups", [(0, None), (8, None), (176, None), (0, 2)])
def test_bench_headline_mode_parity(built, seed0, groups, monkeypatch):
    """8 x 100k scans, 1M map, one livo_iekf_update_batch in the default stream
    grouping (four groups of two scans: the bench's step; groups=2: LIVO_STREAM_GROUPS=2,
    two groups of four): per scan, the oracle's iterations, k-NN passes,
    effective points and per-evaluation state deltas.  seed0: the bench pool's
    first batch (0), its second (8) and a late one (176)."""
    if groups is not None:
        monkeypatch.setenv("LIVO_STREAM_GROUPS", str(groups))  # (read at context creation)
    import livo_amd
    import oracle
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(100_000, seed0 + s)[0] for s in range(8)]
    states = [synth.make_state(seed0 + s) for s in range(8)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(b) for b in scans]
        outs, stats = ctx.iekf_update_batch(sids, states)
    tree = oracle.Tree(m)
    for s in range(8):
        sr, rs = tree.iekf_update(scans[s], states[s], R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=4, threads=8)
        gs = stats[s]
        assert gs["iterations"] == rs["iterations"], s
        assert gs["knn_passes"] == rs["knn_passes"], s
        assert gs["effct_feat_num"] == rs["effct_feat_num"], s
        for e in range(gs["iterations"]):
            assert _rel(gs["solution"][e], rs["solution"][e]) < REL_STATE, (s, e)
        assert _rel(outs[s]["pos"] - states[s]["pos"], sr["pos"] - states[s]["pos"]) < REL_STATE, s


def _same_update(a, b):
    import livo_amd
    for k in ("rot", "pos", "vel", "bias_g", "bias_a", "gravity", "cov"):
        assert np.array_equal(np.asarray(a[0][k]), np.asarray(b[0][k])), k
    assert a[1]["iterations"] == b[1]["iterations"] and a[1]["effct_feat_num"] == b[1]["effct_feat_num"]
    assert np.array_equal(np.asarray(a[1]["solution"]), np.asarray(b[1]["solution"]))


def test_submit_wait_pipeline(built):
    """livo_iekf_update_batch_submit / _wait (the bench's pipelined farm): two
    batches in flight on their own lanes give bit for bit the synchronous
    batch's states and stats, through several rounds of lane reuse; a third
    submit is LIVO_E_BUSY, a scan in two batches in flight LIVO_E_INVALID, a
    wrong ticket LIVO_E_INVALID, and the map / scans cannot change meanwhile."""
    import livo_amd
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(50_000, s)[0] for s in range(8)]
    states = [synth.make_state(s) for s in range(8)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(b) for b in scans]
        A, B = sids[:4], sids[4:]
        ref = ctx.iekf_update_batch(sids, states)
        ref = list(zip(*ref))
        ta = ctx.iekf_update_batch_submit(A, states[:4])
        tb = ctx.iekf_update_batch_submit(B, states[4:])
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.iekf_update_batch_submit([sids[0]], states[:1])
        assert e.value.code == -8  # LIVO_E_BUSY: both lanes in flight
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.map_build(m[:1000])
        assert e.value.code == -8
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.scan_release(sids[0])
        assert e.value.code == -8
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.iekf_update_batch(A, states[:4])
        assert e.value.code == -8
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.iekf_update_batch_wait(tb + 2, 4)
        assert e.value.code == -1
        outs = {}
        outs["a0"] = list(zip(*ctx.iekf_update_batch_wait(ta, 4)))
        with pytest.raises(livo_amd.LivoError) as e:  # scan 4 is still in batch b
            ctx.iekf_update_batch_submit([sids[0], sids[4]], states[:2])
        assert e.value.code == -1
        ta = ctx.iekf_update_batch_submit(A, states[:4])  # lane reuse while b runs
        outs["b0"] = list(zip(*ctx.iekf_update_batch_wait(tb, 4)))
        outs["a1"] = list(zip(*ctx.iekf_update_batch_wait(ta, 4)))
        with pytest.raises(livo_amd.LivoError) as e:  # collected already
            ctx.iekf_update_batch_wait(ta, 4)
        assert e.value.code == -1
        t0 = ctx.iekf_update_batch_submit([], [])  # an empty batch has a ticket too
        ctx.iekf_update_batch_wait(t0, 0)
        sync2 = list(zip(*ctx.iekf_update_batch(sids, states)))  # synchronous again afterwards
    for k in range(4):
        _same_update(outs["a0"][k], ref[k])
        _same_update(outs["a1"][k], ref[k])
        _same_update(outs["b0"][k], ref[4 + k])
    for k in range(8):
        _same_update(sync2[k], ref[k])


@pytest.mark.parametrize("serial", ["0", "1"])
def test_submit_mixed_groups_out_of_order(built, monkeypatch, serial):
    """Two batches in flight on the shared streams with different stream-group
    counts (13 x 100k = 1.3M points -> 4 groups, beside 2 x 50k -> 2 groups),
    the second ticket waited for first, with LIVO_LANE_SERIAL 0 (default) and
    1: each batch equals its synchronous update bit for bit.  While the batches
    are in flight livo_scan_neighbors of one of their scans is LIVO_E_BUSY; a
    submit on the iVox backend is refused (LIVO_E_INVALID) before anything is
    queued, and a synchronous batch runs right after it."""
    import livo_amd
    from livo_amd import synth
    monkeypatch.setenv("LIVO_LANE_SERIAL", serial)
    m = synth.cached_map(1_000_000)
    big = [synth.make_scan(100_000, 300 + s)[0] for s in range(13)]
    small = [synth.make_scan(50_000, 400 + s)[0] for s in range(2)]
    st_big = [synth.make_state(300 + s) for s in range(13)]
    st_small = [synth.make_state(400 + s) for s in range(2)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        sb = [ctx.scan_upload(b) for b in big]
        ss = [ctx.scan_upload(b) for b in small]
        ref_b = list(zip(*ctx.iekf_update_batch(sb, st_big)))
        ref_s = list(zip(*ctx.iekf_update_batch(ss, st_small)))
        for _ in range(2):
            tb = ctx.iekf_update_batch_submit(sb, st_big)
            ts = ctx.iekf_update_batch_submit(ss, st_small)
            with pytest.raises(livo_amd.LivoError) as e:
                ctx.scan_neighbors(ss[0])
            assert e.value.code == -8
            out_s = list(zip(*ctx.iekf_update_batch_wait(ts, 2)))  # the later ticket first
            out_b = list(zip(*ctx.iekf_update_batch_wait(tb, 13)))
            for k in range(2):
                _same_update(out_s[k], ref_s[k])
            for k in range(13):
                _same_update(out_b[k], ref_b[k])
        idx, _ = ctx.scan_neighbors(ss[0])  # collected: readable again
        assert idx.shape == (50_000, 5)
        ctx.set_backend(livo_amd.BACKEND_IVOX)
        ctx.ivox_init()
        ctx.ivox_add_points(m)
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.iekf_update_batch_submit(ss, st_small)
        assert e.value.code == -1
        st_iv, stats_iv = ctx.iekf_update_batch(ss, st_small)  # nothing left queued
        assert all(s["iterations"] >= 1 for s in stats_iv)
        ctx.set_backend(livo_amd.BACKEND_IKDTREE)


def test_bench_two_ranks(built):
    """bench.py --gpus 2 without a launcher starts 2 rank processes (both on this
    box's GPU; gloo all-reduce since RCCL refuses two ranks on one device)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--cpu-seconds", "0", "--legs", "headline", "--pmc", "off"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    j = json.loads(line[0])
    assert j["n_gpus"] == 2
    assert j["total_scans"] == 2 * 8 * 2
    assert j["config"]["parallelism"] == "scan farm x2"
    assert j["value"] > 0


_RCCL_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.path.join(os.environ["LIVO_ROOT"], "fast-livo-noted_amd"))
import torch
import torch.distributed as dist
from livo_amd import farm
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["LIVO_PORT"], rank=0, world_size=1,
                        device_id=dev)
c = farm.Counters(scans=8, evals=40, knn_passes=16, effct_points=123456, knn_visits=77, knn_queries=800000)
tot = farm.allreduce_counters(c, dev)
tmax = farm.allreduce_max(0.125, dev)
dist.barrier()
print("BACKEND", dist.get_backend(), tot.as_array().tolist(), tmax, flush=True)
dist.destroy_process_group()
"""


def test_rccl_counter_allreduce_world1(built):
    """The farm's collectives on device tensors over backend "nccl" (RCCL) at
    world size 1: the code path bench.py --gpus N takes on the 8-GPU node
    (one rank per GPU), here on this box's single GPU."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, LIVO_ROOT=ROOT, LIVO_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("BACKEND")]
    assert line == ["BACKEND nccl [8, 40, 16, 123456, 77, 800000] 0.125"], r.stdout[-1000:]


def test_scan_upload_async_farm(built):
    """livo_scan_upload_async (pinned staging, the upload stream) feeding the
    pipelined farm: scans uploaded while the previous batches run give bit for
    bit the synchronous uploads' updates; a scan is released (LIVO_E_BUSY while
    its batch is in flight) while another batch still runs; neighbours of an
    asynchronously uploaded scan are readable after its batch."""
    import livo_amd
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(50_000, 500 + s)[0] for s in range(12)]
    states = [synth.make_state(500 + s) for s in range(12)]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        ref_ids = [ctx.scan_upload(b) for b in scans]
        ref = list(zip(*ctx.iekf_update_batch(ref_ids, states)))
        for sid in ref_ids:
            ctx.scan_release(sid)
        a = [ctx.scan_upload_async(b) for b in scans[:4]]
        b = [ctx.scan_upload_async(b) for b in scans[4:8]]
        ta = ctx.iekf_update_batch_submit(a, states[:4])
        tb = ctx.iekf_update_batch_submit(b, states[4:8])
        c = [ctx.scan_upload_async(x) for x in scans[8:]]  # beside both batches
        with pytest.raises(livo_amd.LivoError) as e:
            ctx.scan_release(a[0])
        assert e.value.code == -8
        out_a = list(zip(*ctx.iekf_update_batch_wait(ta, 4)))
        for sid in a[1:]:
            ctx.scan_release(sid)  # batch b still in flight
        tc = ctx.iekf_update_batch_submit(c, states[8:])
        out_b = list(zip(*ctx.iekf_update_batch_wait(tb, 4)))
        out_c = list(zip(*ctx.iekf_update_batch_wait(tc, 4)))
        idx, _ = ctx.scan_neighbors(a[0])
        assert idx.shape == (50_000, 5) and (idx >= 0).all()
    for k in range(4):
        _same_update(out_a[k], ref[k])
        _same_update(out_b[k], ref[4 + k])
        _same_update(out_c[k], ref[8 + k])


@pytest.mark.parametrize("max_iter,sizes", [
    (4, [100_000] * 8),
    (4, [100_000, 3_000, 257, 1, 100_000, 65_537, 256, 20_000]),
    (2, [100_000, 50_000, 3_000, 1_000, 100_000, 7, 512, 99_999]),
    (1, [100_000] * 4),
])
def test_ragged_batches_sync_equals_pipelined(built, max_iter, sizes):
    """Ragged scans (1 .. 100k points: one partial, fewer partials than reduction
    shards, a partial short of a full block) through the sharded two-level
    reduction give bit for bit the same states and statistics synchronously and
    as two batches in flight, and every scan matches the oracle (state delta
    per evaluation within 1e-5)."""
    import livo_amd
    import oracle
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    scans = [synth.make_scan(n, 300 + s)[0] for s, n in enumerate(sizes)]
    states = [synth.make_state(300 + s) for s in range(len(sizes))]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=max_iter) as ctx:
        ctx.map_build(m)
        sids = [ctx.scan_upload(b) for b in scans]
        sync = ctx.iekf_update_batch(sids, states)
        h = len(sids) // 2
        ta = ctx.iekf_update_batch_submit(sids[:h], states[:h])
        tb = ctx.iekf_update_batch_submit(sids[h:], states[h:])
        pa = ctx.iekf_update_batch_wait(ta, h)
        pb = ctx.iekf_update_batch_wait(tb, len(sids) - h)
    pipe = (pa[0] + pb[0], pa[1] + pb[1])
    for s in range(len(sizes)):
        _same_update((pipe[0][s], pipe[1][s]), (sync[0][s], sync[1][s]))
    tree = oracle.Tree(m)
    for s in (0, 2, 3, 5):
        if s >= len(sizes):
            continue
        st_ref, stats_ref = tree.iekf_update(scans[s], states[s], R_LI=np.eye(3), t_LI=synth.T_LI,
                                             max_iter=max_iter, threads=8)
        stats = sync[1][s]
        assert stats["iterations"] == stats_ref["iterations"], s
        for e in range(stats["iterations"]):
            assert _rel(stats["solution"][e], stats_ref["solution"][e]) < REL_STATE, (s, e)
        assert np.linalg.norm(sync[0][s]["cov"] - st_ref["cov"]) / np.linalg.norm(states[s]["cov"]) < 1e-9


@pytest.mark.parametrize("pinned", [False, True])
def test_scan_upload_batch_async(built, pinned):
    """livo_scan_upload_batch_async (one copy, bounds, keys, one stable sort of the
    batch, one gather; 16 scans per pass): 18 ragged scans (an empty one, a
    single point, 1..60k points, two passes) are stored exactly as
    livo_scan_upload stores them -- bit for bit the same updates and neighbour
    records -- from ordinary arrays (pinned staging) and from page-locked ones
    (livo_host_register: the copy engine reads them directly)."""
    import livo_amd
    from livo_amd import synth
    m = synth.cached_map(1_000_000)
    sizes = [60_000, 1, 40_000, 0, 257, 30_000, 5, 12_345] + [20_000 + 1000 * s for s in range(10)]
    scans = [np.ascontiguousarray(synth.make_scan(n, 700 + s)[0][:, :3], np.float32) if n > 0
             else np.zeros((0, 3), np.float32) for s, n in enumerate(sizes)]
    states = [synth.make_state(700 + s) for s in range(len(sizes))]
    live = [s for s, n in enumerate(sizes) if n > 0]
    with livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4) as ctx:
        ctx.map_build(m)
        ref_ids = [ctx.scan_upload(scans[s]) for s in live]
        ref = list(zip(*ctx.iekf_update_batch(ref_ids, [states[s] for s in live])))
        ref_nn = [ctx.scan_neighbors(sid) for sid in ref_ids]
        for sid in ref_ids:
            ctx.scan_release(sid)
        if pinned:
            for x in scans:
                if x.nbytes:
                    ctx.host_register(x)
        ids = ctx.scan_upload_batch_async(scans)
        assert len(ids) == len(sizes) and len(set(ids)) == len(ids)
        got = list(zip(*ctx.iekf_update_batch([ids[s] for s in live], [states[s] for s in live])))
        got_nn = [ctx.scan_neighbors(ids[s]) for s in live]
        for sid in ids:
            ctx.scan_release(sid)
        if pinned:
            for x in scans:
                if x.nbytes:
                    ctx.host_unregister(x)
    for k in range(len(live)):
        _same_update(got[k], ref[k])
        assert np.array_equal(got_nn[k][0], ref_nn[k][0]) and np.array_equal(got_nn[k][1], ref_nn[k][1])
