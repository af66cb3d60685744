"""Scan-farm host logic on CPU: sharding and the counter all-reduce over gloo, world size 2.

The GPU bench runs the same code with backend "nccl" (RCCL over xGMI), one
process per GPU; here the ranks only exchange counters, no GPU is touched.
"""
import os
import socket

import numpy as np
import pytest


def test_shard_covers_everything_once():
    from livo_amd import farm
    for n in (0, 1, 7, 64, 65, 100):
        for w in (1, 2, 3, 8):
            ids = [i for r in range(w) for i in farm.shard(n, r, w)]
            assert ids == list(range(n))
            sizes = [len(farm.shard(n, r, w)) for r in range(w)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        farm.shard(10, 2, 2)


def test_counters_from_stats():
    from livo_amd import farm
    c = farm.Counters()
    c.add_stats([{"iterations": 3, "knn_passes": 2, "effct_feat_num": [10, 11, 12]},
                 {"iterations": 5, "knn_passes": 2, "effct_feat_num": [1, 1, 1, 1, 1]}])
    assert (c.scans, c.evals, c.knn_passes, c.effct_points) == (2, 8, 4, 38)
    assert farm.Counters.from_array(c.as_array()) == c


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "fast-livo-noted_amd"))
    import torch.distributed as dist
    from livo_amd import farm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = farm.shard(64, rank, world)
    c = farm.Counters(scans=len(mine), evals=3 * len(mine), knn_passes=2 * len(mine),
                      effct_points=sum(1000 + i for i in mine), knn_visits=50 * len(mine), knn_queries=len(mine))
    tot = farm.allreduce_counters(c)
    tmax = farm.allreduce_max(float(rank + 1))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, tot.as_array().tolist(), tmax))


def test_gloo_world2_counter_allreduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [64, 192, 128, sum(1000 + i for i in range(64)), 3200, 64]
    for rank, tot, tmax in res:
        assert tot == want
        assert tmax == 2.0
