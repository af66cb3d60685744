"""Scan farm across the GPUs of one node.

Independent scans are the unit of parallelism: every rank (one process per
GPU, launched by torch.distributed.run) holds a replica of the map, processes
its own contiguous shard of the scans with no data-path communication, and at
the end of a batch the ranks combine a handful of throughput counters with a
single all-reduce (RCCL over xGMI on the GPU box: backend "nccl"; gloo in the
CPU tests).  A single IEKF step does not shard (its 18x18 solve depends on
the sum over all points), so there is no per-iteration collective.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

COUNTER_FIELDS = ("scans", "evals", "knn_passes", "effct_points", "knn_visits", "knn_queries")


def shard(n_total: int, rank: int, world: int) -> range:
    """Contiguous block of scan ids owned by `rank` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


@dataclasses.dataclass
class Counters:
    scans: int = 0
    evals: int = 0
    knn_passes: int = 0
    effct_points: int = 0
    knn_visits: int = 0
    knn_queries: int = 0

    def add_stats(self, stats):
        """Accumulate livo_iter_stats dicts (or the raw ctypes array) of one batch."""
        for s in stats:
            if isinstance(s, dict):
                it, kp, eff = s["iterations"], s["knn_passes"], sum(s["effct_feat_num"])
            else:
                it, kp = s.iterations, s.knn_passes
                eff = sum(s.effct_feat_num[i] for i in range(min(it, len(s.effct_feat_num))))
            self.scans += 1
            self.evals += it
            self.knn_passes += kp
            self.effct_points += eff

    def as_array(self) -> np.ndarray:
        return np.array([getattr(self, f) for f in COUNTER_FIELDS], np.int64)

    @classmethod
    def from_array(cls, a) -> "Counters":
        return cls(**{f: int(v) for f, v in zip(COUNTER_FIELDS, list(a))})


def dist_env():
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def allreduce_counters(c: Counters, device=None) -> Counters:
    """Sum counters over all ranks (one collective of len(COUNTER_FIELDS) int64)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(c.as_array(), dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized():  # (a world of 1 still runs the collective)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return Counters.from_array(t.cpu().numpy())


def allreduce_max(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
