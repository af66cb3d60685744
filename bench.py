#!/usr/bin/env python3
"""bench.py — IEKF scan-to-map updates/s on MI355X (BASELINE.json metric, configs[1]).

Workload: synthetic Livox-Avia-shaped
100k-point scans against a 1M-point ikd-Tree map, the full IEKF scan update of
laser_mapping.cpp:171-238 with max_iteration = 4 (k-NN + plane fit + Jacobian
+ HᵀH reduction + solve per evaluation, rematch / convergence control on the
device).  A step = one batched pass over --batch independent scans per GPU
(the scan farm of config 4, §8e: 64 scans over 8 GPUs = 8 per GPU); value =
scan updates per second over the whole job, with scans and map already
resident in HBM when the timed region starts.  The farm keeps two batches in
flight per GPU (livo_iekf_update_batch_submit / _wait over two alternating
sets of scans): while the host collects one batch the device already runs the
next.  `sync_value` is the same steps one synchronous batch at a time.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1: one process per GPU.  Under torch.distributed.run (RANK set) this
process is one rank; otherwise it starts N rank processes itself (before any
GPU call), relays rank 0's JSON line and fails if any rank fails.  Every rank
processes its own scans ("weak" scaling); the ranks all-reduce only
throughput counters (RCCL; gloo when ranks share a GPU in a rehearsal).

Extra fields: `roofline` of the dominant kernel (the batch's first-evaluation
k-NN: HIP events on the library's streams, bytes the cell-grid search reads
and writes, counted by the kernel; `traffic` from rocprofv3 PMC passes run by
this bench in child processes), the drop-in regime (one scan at a time,
with and without the upload), config 5 (10M-pt map, 200k-pt scans), the
§8(f) legs, and `cpu_baseline` (oracle/, the C++ restatement, timed on this
host: 1 thread, the reference's 4, and every core available to the job).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import shutil
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "fast-livo-noted_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# Bytes the first evaluation moves by algorithm, the roofline
# unit of the fused kernel k_iekf_eval<true> (search + plane pass + solve):
# per point the body point in (16 B), the 5 neighbour indices + squared
# distances out (40 B) and the plane cache out (16 B + 1 B state); per hash
# slot read 16 B and per map point read 20 B: its 4-B position in the run and
# the 16-B point record it selects (index runs, LIVO_IDX_RUNS; both counted by
# the kernel).
B_QUERY_IO = 16 + 5 * 8 + 17
B_SLOT = 16
B_POINT = 4 + 16
# SURVEY.md §8d's reference-equivalent pricing (the reference tree's traversal):
# V_ref * 64 B per query + 12 B query + 40 B out.
B_NODE = 64
B_QUERY_REF = 12 + 5 * 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="independent scans per step per GPU")
    ap.add_argument("--scan-points", type=int, default=100_000)
    ap.add_argument("--map-points", type=int, default=1_000_000)
    ap.add_argument("--max-iter", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0: skip)")
    ap.add_argument("--legs", default="all", help="comma list: headline,latency,config5,ikfom,ivox,ikd,vio (all)")
    ap.add_argument("--pmc", default="auto", choices=("auto", "off"),
                    help="rocprofv3 PMC passes for roofline.traffic (rank 0, N = 1 only)")
    return ap.parse_args()


# ----------------------------------------------------------------- ranks ----
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """--gpus N without a launcher: start N rank processes (no GPU call here)."""
    n = a.gpus
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # rank 0's stdout is this process's (the JSON line); the others' go to stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in procs:  # a failed rank leaves the others at a barrier
                    q.kill()
        time.sleep(0.05)
    return rc


def stream_groups(batch_points: int = 800_000) -> int:
    """Stream groups of a batched update (LIVO_STREAM_GROUPS; livo_capi.cpp's default:
    4 since round 4)."""
    if os.environ.get("LIVO_STREAM_GROUPS"):
        return int(os.environ["LIVO_STREAM_GROUPS"])
    return 4


def host_threads() -> int:
    """Cores this job may use: the affinity set, capped by the cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except Exception:
        pass
    return n


def ref_calibration() -> dict:
    """The oracle's k-NN time over the reference ikd_Tree.cpp's at the 1M map, single
    thread (tests/golden/knn_calibration.json, made in the build container by
    tools/calibrate_knn.py against BASELINE.md's survey timing of the reference).
    Below 1: the oracle is the faster of the two, so a speedup over it understates
    the speedup over the reference.  A timing calibration; it pins no parity."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "knn_calibration.json")) as f:
            cal = json.load(f)
        row = next(r for r in cal["rows"] if r["map_points"] == 1_000_000)
        return {"ref_calibration_ratio": row["ratio_oracle_over_reference"],
                "ref_calibration_note": "oracle k-NN us/query over the reference ikd_Tree.cpp's at 1M map points, "
                                        "1 thread (" + cal["reference_source"] + "; " + cal["note"] + ")"}
    except (OSError, StopIteration, KeyError, ValueError):
        return {"ref_calibration_ratio": None, "ref_calibration_note": "tests/golden/knn_calibration.json missing"}


POOL_CAP = 1024  # most distinct scans a rank keeps resident (~17 MB of HBM each at 100k points)


def gen_scans(n_points: int, seeds, workers: int):
    """synth.make_scan of every seed (body points only), in a process pool before any GPU call."""
    from livo_amd import synth
    seeds = list(seeds)
    if workers <= 1 or len(seeds) < 4:
        return [synth.make_scan(n_points, s)[0] for s in seeds]
    import concurrent.futures
    import multiprocessing
    with concurrent.futures.ProcessPoolExecutor(max_workers=workers,
                                                mp_context=multiprocessing.get_context("fork")) as ex:
        return list(ex.map(_scan_body, [(n_points, s) for s in seeds], chunksize=2))


def _scan_body(arg):
    from livo_amd import synth
    return synth.make_scan(arg[0], arg[1])[0]


# ------------------------------------------------------------------- PMC ----
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"),
              ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES"))


def pmc_traffic(a, kernel_key: str):
    """rocprofv3 --pmc passes over tools/knn_probe.py (same map, scans and batch
    as the headline), one child process per pass (MI355X_MICROARCH.md §rocprofv3
    PMC slots): HBM bytes per first-evaluation k-NN of a batch = the unit
    kernel's dispatches x (2 x FETCH_SIZE + WRITE_SIZE) (FETCH_SIZE doubled on
    gfx950, §HBM), plus its L2 hit rate and wait share.  None if unavailable."""
    prof = shutil.which("rocprofv3")
    if a.pmc == "off" or not prof:
        return None
    import collections
    import csv
    import glob
    import tempfile
    out = tempfile.mkdtemp(prefix="livo_pmc_")
    per = collections.defaultdict(list)
    for k, counters in enumerate(PMC_PASSES):
        d = os.path.join(out, f"pass{k}")
        cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", *counters, "-d", d, "-o", "pmc", "--output-format",
               "csv", "--", sys.executable, os.path.join(ROOT, "tools", "knn_probe.py"), "--scan-points",
               str(a.scan_points), "--map-points", str(a.map_points), "--batch", str(a.batch)]
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            sys.stderr.write(f"pmc pass {counters} failed ({r.returncode}): {r.stderr[-400:]}\n")
            return None
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            acc = collections.defaultdict(float)
            for row in csv.DictReader(open(f)):
                if kernel_key in row["Kernel_Name"]:
                    acc[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            for (_, cname), v in acc.items():
                per[cname].append(v)
    shutil.rmtree(out, ignore_errors=True)
    mean = {k: sum(v) / len(v) for k, v in per.items() if v}
    if "FETCH_SIZE" not in mean or "WRITE_SIZE" not in mean:
        return None
    disp = len(per["FETCH_SIZE"])
    groups = min(stream_groups(a.batch * a.scan_points), a.batch)  # one first-search dispatch per stream group and batch
    res = {"hbm_bytes_per_launch": groups * (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024,
           "fetch_kib_per_dispatch": round(mean["FETCH_SIZE"], 1), "write_kib_per_dispatch": round(mean["WRITE_SIZE"], 1),
           "dispatches_sampled": disp}
    if mean.get("TCC_HIT_sum") is not None and mean.get("TCC_MISS_sum"):
        res["l2_hit_rate"] = round(mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]), 4)
    if mean.get("SQ_WAVE_CYCLES"):
        res["wait_any_share"] = round(mean.get("SQ_WAIT_ANY", 0.0) / mean["SQ_WAVE_CYCLES"], 4)
    return res


# ------------------------------------------------------------------ main ----
def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(a))
    if world > 1 and a.gpus != world:
        sys.stderr.write(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; {world} ranks run\n")
    legs = set(a.legs.split(",")) if a.legs != "all" else {"headline", "latency", "config5", "ikfom", "ivox", "ikd",
                                                           "vio"}
    if rank > 0:
        legs = {"headline"}  # the side legs are rank 0's report: other ranks only run the headline
    import livo_amd
    from livo_amd import farm, synth

    # inputs (identical generator on every rank; each rank its own scans), made
    # before any GPU call so that the PMC children find the map in the cache.
    # A pool of distinct scans (config 4's independent scans, seeds rank * pool
    # + j): every batch of the warm-up and of the timed region takes the next
    # a.batch of them, so no scan repeats within the timed region (up to
    # POOL_CAP scans; beyond that the pool rotates, and the line says so)
    m = synth.cached_map(a.map_points)
    n_batches = max(1, min(POOL_CAP // a.batch, a.steps + max(a.warmup, 2)))
    pool_n = n_batches * a.batch
    pool_seeds = [rank * pool_n + j for j in range(pool_n)]
    t = time.time()
    pool_scans = gen_scans(a.scan_points, pool_seeds, min(16, host_threads()))
    pool_st0 = [synth.make_state(s) for s in pool_seeds]
    gen_s = time.time() - t
    scan_ids = pool_seeds[:a.batch]  # the first batch: parity, latency, IKFoM / iVox legs, CPU baseline
    scans = pool_scans[:a.batch]
    st0 = pool_st0[:a.batch]
    kind = os.environ.get("LIVO_KNN_KIND", "tile")
    fused = kind == "tile" and os.environ.get("LIVO_FUSED", "1") != "0"
    unit_kernel = {"leaf": "k_knn_leaf<false", "grid": "k_knn_grid<false, false>"}.get(
        kind, "k_iekf_eval<true>" if fused else "k_knn_grid<false, true>")
    pmc = pmc_traffic(a, unit_kernel) if (rank == 0 and world == 1) else None

    import torch
    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch_dev = None
    device = local_rank
    ndev = torch.cuda.device_count()
    if torch.cuda.is_available():
        # one process per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share them
        device = local_rank % max(1, ndev)
        torch.cuda.set_device(device)
        torch_dev = torch.device("cuda", device)
    # RCCL (backend "nccl") over xGMI; gloo when ranks share a GPU (RCCL refuses that) or on request
    backend = os.environ.get("LIVO_BENCH_BACKEND") or ("nccl" if torch_dev is not None and ndev >= world else "gloo")
    coll_dev = torch_dev if backend == "nccl" else None
    if world > 1:
        dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        if torch_dev is not None:
            torch.cuda.synchronize()

    ctx = livo_amd.Context(device, t_LI=synth.T_LI, max_iterations=a.max_iter)
    t = time.time()
    ctx.map_build(m)
    map_build_s = time.time() - t
    pool_sids = [ctx.scan_upload(s) for s in pool_scans]
    # the device holds them now; the host keeps the first batch + 32 (the ikd leg maps with
    # the next 32; the upload leg streams the first four batches)
    del pool_scans[max(a.batch + 32, 4 * a.batch):]
    sids = pool_sids[:a.batch]
    # V_ref: nodes the reference traversal visits for the first search of the
    # first batch (the reference-order pass k_knn_pass, outside the timed
    # region): the reference-equivalent pricing of SURVEY.md §8d, per query
    v_ref = sum(ctx.h_share(sid, s, search_en=True)["visits"] for sid, s in zip(sids, st0))
    vq_ref = v_ref / max(sum(len(s) for s in scans), 1)
    batches = []  # (scan ids, initial states) of each batch of the pool
    for b in range(n_batches):
        ids = pool_sids[b * a.batch:(b + 1) * a.batch]
        batches.append((ids, (livo_amd.State * a.batch)(*[livo_amd.state_to_c(s) for s in
                                                          pool_st0[b * a.batch:(b + 1) * a.batch]])))
    init = batches[0][1]
    work = (livo_amd.State * a.batch)()
    nbytes = C.sizeof(init)
    # the round-3 mode beside it: the first 8 scans every step (two uploads, since
    # a scan is in one batch in flight at a time)
    fixed = [(sids, init), ([ctx.scan_upload(s) for s in scans], init)]

    def step(b=0):
        """One synchronous batch (livo_iekf_update_batch) of pool batch b: the profiled legs."""
        ids, ini = batches[b % n_batches]
        C.memmove(work, ini, nbytes)  # the scans start from their priors
        _, stats = ctx.iekf_update_batch(ids, work, raw=True)
        return stats

    # The farm's steady state: each step submits one batch of a.batch scans
    # (livo_iekf_update_batch_submit) and collects the batch submitted two steps
    # earlier, so the device always holds the next batch while the host collects
    # one.  Every submitted batch is collected before the clock stops.
    outs = [((livo_amd.State * a.batch)(), (livo_amd.IterStats * a.batch)()) for _ in range(2)]

    def pipeline(nsteps, first, counters=None, sets=None):
        """nsteps batches: pool batches first, first + 1, ... (or the two `sets` alternating)."""
        pending = []
        for k in range(nsteps):
            if len(pending) == livo_amd.MAX_INFLIGHT:
                t, j = pending.pop(0)
                _, st = ctx.iekf_update_batch_wait(t, a.batch, *outs[j])
                if counters is not None:
                    counters.add_stats(st)
            ids, ini = sets[k % 2] if sets else batches[(first + k) % n_batches]
            j = k % 2
            pending.append((ctx.iekf_update_batch_submit(ids, ini), j))
        for t, j in pending:
            _, st = ctx.iekf_update_batch_wait(t, a.batch, *outs[j])
            if counters is not None:
                counters.add_stats(st)

    # warm-up on the pool's last batches (the timed region starts at batch 0)
    n_warm = max(a.warmup, 2)
    pipeline(n_warm, n_batches - n_warm)
    for w in range(a.warmup):
        step(n_batches - 1 - w)
    first_stats = [livo_amd.stats_from_c(s) for s in step(0)]
    first_states = [livo_amd.state_from_c(s) for s in work]

    counters = farm.Counters()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    pipeline(a.steps, 0, counters)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    # the fixed-8 rate of round 3 (the same 8 scans every step), untimed for value
    fixed_counters = farm.Counters()
    pipeline(2, 0, sets=fixed)
    sync()
    t0f = time.perf_counter()
    pipeline(a.steps, 0, fixed_counters, sets=fixed)
    sync()
    elapsed_fixed = time.perf_counter() - t0f

    # The farm with each scan's upload inside the clock: every batch's scans go
    # from host arrays (four distinct batches of the pool, cycled) through ONE
    # livo_scan_upload_batch_async two batches ahead of their submit, overlapping
    # the batches in flight, and are released once collected; untimed for value.
    # value_with_upload: the host arrays page-locked once (livo_host_register, as a
    # driver filling pinned buffers would), so the copy engine reads them directly;
    # value_with_upload_pageable: ordinary arrays through the pinned staging ring.
    # (an A/B build from before livo_scan_upload_batch_async skips these legs)
    n_up = min(4, len(pool_scans) // a.batch) if hasattr(ctx._L, "livo_scan_upload_batch_async") else 0
    up_sets = [([np.ascontiguousarray(x[:, :3], np.float32) for x in pool_scans[b * a.batch:(b + 1) * a.batch]],
                batches[b][1]) for b in range(n_up)]

    def pipeline_upload(nsteps, counters=None):
        pending, ahead, nxt = [], [], 0
        for k in range(nsteps):
            while len(ahead) < 2 and nxt < nsteps:
                ahead.append((nxt, ctx.scan_upload_batch_async(up_sets[nxt % n_up][0])))
                nxt += 1
            if len(pending) == livo_amd.MAX_INFLIGHT:
                t, j, ids = pending.pop(0)
                _, st = ctx.iekf_update_batch_wait(t, a.batch, *outs[j])
                for sid in ids:
                    ctx.scan_release(sid)
                if counters is not None:
                    counters.add_stats(st)
            b, ids = ahead.pop(0)
            j = k % 2
            pending.append((ctx.iekf_update_batch_submit(ids, up_sets[b % n_up][1]), j, ids))
        for t, j, ids in pending:
            _, st = ctx.iekf_update_batch_wait(t, a.batch, *outs[j])
            for sid in ids:
                ctx.scan_release(sid)
            if counters is not None:
                counters.add_stats(st)

    def upload_leg():
        c = farm.Counters()
        pipeline_upload(4)
        sync()
        t0u = time.perf_counter()
        pipeline_upload(a.steps, c)
        sync()
        return c, time.perf_counter() - t0u

    upload_counters = upload_counters_pg = farm.Counters()
    elapsed_up = elapsed_up_pg = 0.0
    if n_up >= 1:
        for x, _ in up_sets:
            for arr in x:
                ctx.host_register(arr)
        upload_counters, elapsed_up = upload_leg()
        for x, _ in up_sets:
            for arr in x:
                ctx.host_unregister(arr)
        upload_counters_pg, elapsed_up_pg = upload_leg()

    # The same steps one synchronous batch at a time (the host waits for each
    # batch before the next is queued), untimed for the headline and reported
    # as sync_value; level-1 profiling: HIP events around the batch's
    # first-evaluation launch only (the roofline unit).  The per-stage
    # breakdown (level 2) costs ~10% and is taken from extra steps below.
    ctx.set_profiling(1)
    knn_ms = 0.0
    knn_launches = knn_visits = knn_points = knn_queries = replays = 0
    sync()
    t0s = time.perf_counter()
    for k in range(a.steps):
        step(k)
        tm = ctx.last_timings()
        knn_ms += tm["knn_ms"]
        knn_launches += tm["knn_launches"]
        knn_visits += tm["knn_visits"]
        knn_points += tm["knn_points"]
        knn_queries += tm["knn_queries"]
    sync()
    elapsed_sync = time.perf_counter() - t0s
    # per-stage device time (summed over the concurrent stream groups), untimed
    ctx.set_profiling(2)
    n_prof = 10
    t_first = t_rematch = t_plane = t_batch = t_gap = 0.0
    n_gap = n_remevals = 0
    replays = 0
    t0p = time.perf_counter()
    for k in range(n_prof):
        step(k)
        tm = ctx.last_timings()
        t_first += tm["knn_ms"]
        t_rematch += tm["rematch_knn_ms"]
        t_plane += tm["plane_ms"]
        t_batch += tm["batch_ms"]
        if tm["gap_ms"] > 0:
            t_gap += tm["gap_ms"]
            n_gap += 1
        n_remevals += sum(1 for e, sc in enumerate(tm["eval_searched"]) if e > 0 and sc > 0)
        replays += tm["knn_replays"]
    wall_prof = (time.perf_counter() - t0p) / n_prof
    ctx.set_profiling(0)
    counters.knn_visits, counters.knn_queries = knn_visits, knn_queries
    elapsed_max = farm.allreduce_max(elapsed, coll_dev)
    elapsed_sync_max = farm.allreduce_max(elapsed_sync, coll_dev)
    total = farm.allreduce_counters(counters, coll_dev)

    # roofline of the dominant kernel (rank-local): the first-evaluation k-NN of
    # one batch (4 concurrent stream-group dispatches + their replays)
    L = max(knn_launches, 1)
    launch_ms = knn_ms / L
    q_launch = knn_queries / L
    alg_bytes = (knn_visits / L) * B_SLOT + (knn_points / L) * B_POINT + q_launch * B_QUERY_IO
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    ref_equiv = (vq_ref * q_launch * B_NODE + q_launch * B_QUERY_REF) / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0

    result = None
    if rank == 0:
        value = total.scans / elapsed_max
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": round(pmc["hbm_bytes_per_launch"]) if pmc else None,
                "kernel": (f"first evaluation of the batch: {min(stream_groups(a.batch * a.scan_points), a.batch)} {unit_kernel} dispatch(es) (one "
                           "per stream group, concurrent; every scan of the group: transform + exact 5-NN of every point with in-place tie replay + plane "
                           "fit + Jacobian + HTH reduction + solve)") if fused else
                          (f"first-evaluation k-NN of the batch: {min(stream_groups(a.batch * a.scan_points), a.batch)} concurrent {unit_kernel} dispatches "
                           "(one per stream group: transform + exact 5-NN of every point) + their tie replays"),
                "avg_launch_ms": round(launch_ms, 4),
                "alg_bytes_per_launch": int(alg_bytes),
                "alg_bytes_terms": {"slots_per_query": round(knn_visits / max(knn_queries, 1), 3),
                                    "points_per_query": round(knn_points / max(knn_queries, 1), 2),
                                    "bytes_per_query": round(alg_bytes / max(q_launch, 1), 1)},
                "frac_fabric_traffic": (round(pmc["hbm_bytes_per_launch"] / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                        if pmc and launch_ms > 0 else None),
                "traffic_note": ("traffic = the L2's memory-side requests (2 x FETCH_SIZE + WRITE_SIZE per the MI355X "
                                 "guide's gfx950 correction): it counts Infinity-Cache hits as well as HBM reads, so it "
                                 "bounds HBM traffic from above; frac_fabric_traffic = traffic / launch time / HBM peak"),
                "limiter": ("dependent-load latency: the priced roofline is HBM (bound), but the measured limiter is the "
                            "chain hash probe -> run chunks per query (L2/MALL hits), not bytes (frac_fabric_traffic)"),
                "reference_equivalent_GBps": round(ref_equiv, 1),
                "reference_equivalent_note": ("not a roofline (it exceeds the HBM peak): the bytes the reference's "
                                              "ikd-Tree search would read per query (visits_per_query_ref x 64 B + "
                                              "52 B) over this launch's time, a work-equivalence figure only"),
                "visits_per_query_ref": round(vq_ref, 3)}
        if pmc:
            roof["pmc"] = {k: v for k, v in pmc.items() if k != "hbm_bytes_per_launch"}
        result = {
            "metric": "IEKF scan-to-map updates/sec (100k-pt scan, 1M-pt map)",
            "value": round(value, 3),
            "unit": "scan updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic (seeded planar room map + Livox-Avia rosette scans; reference ships no bags)",
            "config": {"workload": f"config2: {a.scan_points // 1000}k-pt scan vs {a.map_points // 1000000 or a.map_points}"
                                   f"{'M' if a.map_points >= 1000000 else ''}-pt map, max_iteration={a.max_iter}, "
                                   f"{a.batch} independent scans per GPU per step",
                       "scan_points": a.scan_points, "map_points": a.map_points, "max_iteration": a.max_iter,
                       "scans_per_step_per_gpu": a.batch, "parallelism": f"scan farm x{world}",
                       "collective": backend if world > 1 else None},
            "total_scans": total.scans,
            "mode": ("pipelined farm: livo_iekf_update_batch_submit / _wait, two batches in flight per GPU, "
                     f"every batch the next {a.batch} of a pool of {pool_n} distinct resident scans per GPU "
                     f"(seeds rank*{pool_n}+j; warm-up on the pool's last {n_warm} batches, the timed region from "
                     "batch 0"
                     + (", no scan repeated within it" if a.steps <= n_batches else
                        f", rotating: the pool holds {n_batches} batches") +
                     "), every batch collected inside the timed region"),
            "scan_pool": {"distinct_scans_per_gpu": pool_n, "batches": n_batches,
                          "repeats_in_timed_region": a.steps > n_batches,
                          "generation_s": round(gen_s, 2)},
            "value_with_upload": round(world * upload_counters.scans / elapsed_up, 3) if elapsed_up > 0 else None,
            "value_with_upload_pageable": (round(world * upload_counters_pg.scans / elapsed_up_pg, 3)
                                           if elapsed_up_pg > 0 else None),
            "upload_note": ("the same pipelined farm with every batch's scans uploaded inside the clock: host arrays "
                            "-> ONE livo_scan_upload_batch_async per batch (copy + bounds + keys + one stable sort + "
                            "gather on the upload stream) two batches ahead of its submit, released once collected; "
                            f"{n_up} distinct host batches cycled; value_with_upload from page-locked arrays "
                            "(livo_host_register once, the copy engine reads them), value_with_upload_pageable from "
                            "ordinary arrays through the pinned staging ring; untimed for value"),
            "fixed8_value": round(world * fixed_counters.scans / elapsed_fixed, 3),
            "fixed8_note": ("round 3's headline mode on this rank's GPU (scaled by the rank count): the same first 8 "
                            "scans every step (two uploads alternating), pipelined like value; untimed for value"),
            "sync_value": round(world * a.batch * a.steps / elapsed_sync_max, 3),
            "sync_ms_per_step": round(elapsed_sync_max / a.steps * 1e3, 4),
            "sync_note": ("the same pool batches with livo_iekf_update_batch (one batch at a time, the host waits for "
                          "each); untimed for value"),
            "iekf_steps_per_s": round(total.evals / elapsed_max, 3),
            "knn_queries_per_s": round((total.knn_passes * a.scan_points) / elapsed_max, 1),
            "evals_per_scan": round(total.evals / max(total.scans, 1), 3),
            "knn_passes_per_scan": round(total.knn_passes / max(total.scans, 1), 3),
            "roofline": roof,
            "device_ms_per_step": {
                "eval_first": round(t_first / n_prof, 4),
                "eval_rematch": round(t_rematch / n_prof, 4),
                "eval_nosearch": round(t_plane / n_prof, 4),
                "copies_and_launch": round((t_batch - t_first - t_rematch - t_plane) / n_prof, 4),
                "host_gap": round(t_gap / max(n_gap, 1), 4),
                "sum": round((t_batch / n_prof) + t_gap / max(n_gap, 1), 4),
                "wall_ms_per_step_profiled": round(wall_prof * 1e3, 4),
                "rematch_evals_per_step": round(n_remevals / n_prof, 2),
                "note": f"{n_prof} extra untimed steps with an event before every evaluation launch: eval_first = the "
                        "first evaluation (search for every point + plane + reduction + solve), eval_rematch = the later "
                        "evaluations in which some scan searched again, eval_nosearch = the cached-plane evaluations, "
                        "copies_and_launch = the rest of the batch span (slot copies in/out), host_gap = device idle "
                        "between two batches (the host's return, Python step, next call); sum = batch span + host_gap"},
            "knn_replays_per_step": round(replays / n_prof, 2),
            "map_build_s": round(map_build_s, 3),
        }

    # ---- the drop-in regime: one scan at a time through livo_iekf_update (the
    # facade's iterate()), resident scan; and with livo_scan_upload of the
    # host points (Morton order on the device) inside the timed region
    if "latency" in legs:
        one = (livo_amd.State * 1)()
        for _ in range(2):
            for j in range(a.batch):
                C.memmove(one, C.byref(init, j * C.sizeof(livo_amd.State)), C.sizeof(livo_amd.State))
                ctx.iekf_update_batch([sids[j]], one, raw=True)
        reps = max(2, a.steps // a.batch) * a.batch
        sync()
        t = time.perf_counter()
        for k in range(reps):
            j = k % a.batch
            C.memmove(one, C.byref(init, j * C.sizeof(livo_amd.State)), C.sizeof(livo_amd.State))
            ctx.iekf_update_batch([sids[j]], one, raw=True)
        sync()
        lat = (time.perf_counter() - t) / reps

        def upload_pass():
            for k in range(a.batch):
                C.memmove(one, C.byref(init, k * C.sizeof(livo_amd.State)), C.sizeof(livo_amd.State))
                sid = ctx.scan_upload(scans[k])
                ctx.iekf_update_batch([sid], one, raw=True)
                ctx.scan_release(sid)

        upload_pass()  # warm: a frame loop reuses the released scan buffers after its first frame
        sync()
        t = time.perf_counter()
        for _ in range(2):
            upload_pass()
        sync()
        lat_up = (time.perf_counter() - t) / (2 * a.batch)
        if rank == 0:
            result["drop_in"] = {"ms_per_scan": round(lat * 1e3, 4), "updates_per_s": round(1.0 / lat, 2),
                                 "ms_per_scan_with_upload": round(lat_up * 1e3, 4),
                                 "note": "batch 1, sequential: livo_iekf_update on a resident scan; then "
                                         "livo_scan_upload (host points -> HBM, device Morton sort) + update + "
                                         "release per scan, host-timed over two passes after one warm pass (the "
                                         "released buffers reused, as a frame loop does)"}

    # ---- config 5 (BASELINE configs[4]): 10M-point map, 200k-point scans at
    # filter_size_surf = 0.05: each scan is the device VoxelGrid (leaf 0.05,
    # livo_scan_preprocess = downSizeFilterSurf, laser_mapping.cpp:129-130,1111)
    # of a raw still frame dense enough to leave ~200k points (untimed)
    if "config5" in legs and a.map_points == 1_000_000:
        m5 = synth.cached_map(10_000_000)
        c5 = livo_amd.Context(device, t_LI=synth.T_LI, max_iterations=a.max_iter)
        t = time.time()
        c5.map_build(m5)
        b5 = time.time() - t
        del m5
        n5 = min(a.batch, 8)
        s5, n5_pts = [], []
        for s in scan_ids[:n5]:
            raw, poses, Re, pe = synth.make_config5_frame(1000 + s)
            sid5, _, down5 = c5.scan_preprocess(raw, poses, Re, pe, leaf_size=synth.CONFIG5_LEAF)
            s5.append(sid5)
            n5_pts.append(len(down5))
        i5 = (livo_amd.State * n5)(*[livo_amd.state_to_c(synth.make_state(1000 + s)) for s in scan_ids[:n5]])
        w5 = (livo_amd.State * n5)()

        def step5():
            C.memmove(w5, i5, C.sizeof(i5))
            return c5.iekf_update_batch(s5, w5, raw=True)[1]

        step5()
        c5.set_profiling(1)
        k5 = max(3, a.steps // 4)
        kms = kv = kp = kq = 0
        ev5 = 0
        sync()
        t = time.perf_counter()
        for _ in range(k5):
            st5 = step5()
            ev5 += sum(s.iterations for s in st5)
            tm = c5.last_timings()
            kms += tm["knn_ms"]; kv += tm["knn_visits"]; kp += tm["knn_points"]; kq += tm["knn_queries"]
        sync()
        e5 = time.perf_counter() - t
        c5.set_profiling(0)
        lm = kms / k5
        ab = (kv / k5) * B_SLOT + (kp / k5) * B_POINT + (kq / k5) * B_QUERY_IO
        if rank == 0:
            result["config5"] = {"updates_per_s": round(k5 * n5 / e5, 3), "ms_per_step": round(e5 / k5 * 1e3, 4),
                                 "evals_per_scan": round(ev5 / (k5 * n5), 3), "map_build_s": round(b5, 2),
                                 "knn_first_ms": round(lm, 4), "knn_alg_bytes_per_launch": int(ab),
                                 "knn_achieved_GBps": round(ab / (lm * 1e-3) / 1e9, 1) if lm > 0 else None,
                                 "points_per_query": round(kp / max(kq, 1), 2),
                                 "scan_points_mean": round(sum(n5_pts) / len(n5_pts), 1),
                                 "raw_points_per_frame": synth.CONFIG5_RAW_POINTS,
                                 "note": f"10M-pt map, {n5} scans per step, each the device VoxelGrid (leaf "
                                         f"{synth.CONFIG5_LEAF}) of a {synth.CONFIG5_RAW_POINTS // 1000}k-pt raw still "
                                         f"frame, max_iteration={a.max_iter}"}
        c5.close()

    # ---- the IKFoM formulation on the same scans
    if "ikfom" in legs:
        ik_init = (livo_amd.IkfomState * a.batch)(*[livo_amd.ikfom_to_c(synth.make_ikfom_state(s)) for s in scan_ids])
        ik_work = (livo_amd.IkfomState * a.batch)()
        ik_bytes = C.sizeof(ik_init)

        def ik_step():
            C.memmove(ik_work, ik_init, ik_bytes)
            return ctx.ikfom_update_batch(sids, ik_work, raw=True)[1]

        for _ in range(2):
            ik_step()
        ik_steps = max(5, a.steps // 2)
        sync()
        t = time.perf_counter()
        ik_evals = 0
        for _ in range(ik_steps):
            ik_evals += sum(s.iterations for s in ik_step())
        sync()
        ik_elapsed = time.perf_counter() - t  # (rank 0 only: no collective)
        ik_total = farm.Counters(scans=ik_steps * a.batch, evals=ik_evals)
        ik_first = livo_amd.ikfom_stats_from_c(ik_step()[0])
        # pipelined like the headline: two batches of distinct scans in flight
        # (livo_ikfom_update_batch_submit / _wait), the pool's first two batches
        ik_pipe = None
        if hasattr(ctx._L, "livo_ikfom_update_batch_submit") and len(batches) >= 2:
            ik_sets = []
            for b in range(2):
                ids_b = batches[b][0]
                seeds_b = pool_seeds[b * a.batch:(b + 1) * a.batch]
                st_b = (livo_amd.IkfomState * a.batch)(*[livo_amd.ikfom_to_c(synth.make_ikfom_state(x))
                                                         for x in seeds_b])
                ik_sets.append((ids_b, st_b))
            ik_outs = [((livo_amd.IkfomState * a.batch)(), (livo_amd.IkfomStats * a.batch)()) for _ in range(2)]

            def ik_pipeline(nsteps):
                pend, ev = [], 0
                for k in range(nsteps):
                    if len(pend) == 2:
                        tk, j = pend.pop(0)
                        ev += sum(x.iterations for x in ctx.ikfom_update_batch_wait(tk, a.batch, *ik_outs[j])[1])
                    pend.append((ctx.ikfom_update_batch_submit(ik_sets[k % 2][0], ik_sets[k % 2][1], raw=True),
                                 k % 2))
                for tk, j in pend:
                    ev += sum(x.iterations for x in ctx.ikfom_update_batch_wait(tk, a.batch, *ik_outs[j])[1])
                return ev

            ik_pipeline(4)
            sync()
            t = time.perf_counter()
            ik_pevals = ik_pipeline(ik_steps)
            sync()
            ik_pipe = (time.perf_counter() - t, ik_pevals)
        if rank == 0:
            ik_rate = ik_total.scans / ik_elapsed
            result["ikfom"] = {"updates_per_s": round(ik_steps * a.batch / ik_pipe[0] if ik_pipe else ik_rate, 3),
                               "ms_per_step": round((ik_pipe[0] if ik_pipe else ik_elapsed) / ik_steps * 1e3, 4),
                               "sync_updates_per_s": round(ik_rate, 3),
                               "evals_per_scan": round(ik_total.evals / max(ik_total.scans, 1), 3),
                               "note": "livo_ikfom_update_batch_submit / _wait (state_ikfom, esekfom.hpp:1619-1928), "
                                       f"two batches of {a.batch} distinct scans in flight (the pool's first two "
                                       f"batches, rank 0 only), {ik_steps} steps after the headline run; "
                                       "sync_updates_per_s: livo_ikfom_update_batch one batch at a time"}

    # ---- the iVox backend (the reference's default build)
    if "ivox" in legs:
        ctx.set_backend(livo_amd.BACKEND_IVOX)
        t = time.perf_counter()
        ctx.ivox_init()
        ctx.ivox_add_points(m)
        iv_build_s = time.perf_counter() - t
        iv_info = ctx.ivox_info()
        # fresh scan buffers: a point without iVox candidates keeps its cached
        # neighbours (ivox3d.h:165-167), so the first update starts from empty caches
        iv_sids = [ctx.scan_upload(sc) for sc in scans]

        def iv_step():
            C.memmove(work, init, nbytes)
            return ctx.iekf_update_batch(iv_sids, work, raw=True)[1]

        iv_first = [livo_amd.stats_from_c(s) for s in iv_step()]
        for _ in range(2):
            iv_step()
        iv_steps = max(5, a.steps // 2)
        sync()
        t = time.perf_counter()
        iv_evals = 0
        for _ in range(iv_steps):
            iv_evals += sum(s.iterations for s in iv_step())
        sync()
        iv_elapsed = time.perf_counter() - t
        iv_total = farm.Counters(scans=iv_steps * a.batch, evals=iv_evals)
        # odometry: one scan after the other, each updated then merged into the map;
        # two passes over the scans (fresh scan buffers each), the second timed: the
        # first warms the allocations and grows the map, as the ikd-Tree leg does
        for rep in range(2):
            odo_sids = [ctx.scan_upload(sc) for sc in scans]
            sync()
            t = time.perf_counter()
            t_incr = 0.0
            added = 0
            for sid, s in zip(odo_sids, st0):
                st, _ = ctx.iekf_update(sid, s)
                t1 = time.perf_counter()
                _, cnt = ctx.map_incremental(sid, st, filter_size_map=0.5)
                t_incr += time.perf_counter() - t1
                added += cnt["added"] + cnt["no_downsample"]
            sync()
            odo_elapsed = time.perf_counter() - t
            for sid in odo_sids:
                ctx.scan_release(sid)
        for sid in iv_sids:
            ctx.scan_release(sid)
        # the regime the reference ships (laser_mapping.cpp:145-151, 329-389): the iVox
        # map holds the first downsampled scan, grown by map_incremental at every
        # later scan (here 31 mapping scans at their true poses), not a dense
        # synthetic room; the same odometry on it, second pass timed
        m_seeds = list(pool_seeds[a.batch:a.batch + 32])
        m_scans = list(pool_scans[a.batch:a.batch + 32])
        if len(m_seeds) < 32:
            extra = [pool_seeds[-1] + 1 + j for j in range(32 - len(m_seeds))]
            m_seeds += extra
            m_scans += gen_scans(a.scan_points, extra, 1)
        R0, p0, _ = synth.true_pose(m_seeds[0])
        w0 = (m_scans[0].astype(np.float64) @ synth.R_LI.T + synth.T_LI) @ R0.T + p0
        _, first = np.unique(np.floor(w0 / 0.5).astype(np.int64), axis=0, return_index=True)
        ivr = livo_amd.Context(device, t_LI=synth.T_LI, max_iterations=a.max_iter)
        ivr.set_backend(livo_amd.BACKEND_IVOX)
        ivr.ivox_init()
        ivr.ivox_add_points(np.ascontiguousarray(w0[np.sort(first)], dtype=np.float32))
        for sd, sc in zip(m_seeds[1:], m_scans[1:]):
            # each mapping scan updated first: map_incremental's downsampling reads the
            # update's Nearest_Points (laser_mapping.cpp:343-371)
            sid = ivr.scan_upload(sc)
            stm, _ = ivr.iekf_update(sid, synth.make_state(sd, rot_deg=0.0, trans_m=0.0))
            ivr.map_incremental(sid, stm, filter_size_map=0.5)
            ivr.scan_release(sid)
        ivr_before = ivr.ivox_info()
        for rep in range(2):
            r_sids = [ivr.scan_upload(sc) for sc in scans]
            ivr.sync()
            t = time.perf_counter()
            tr_incr = 0.0
            for sid, s in zip(r_sids, st0):
                st, _ = ivr.iekf_update(sid, s)
                t1 = time.perf_counter()
                ivr.map_incremental(sid, st, filter_size_map=0.5)
                tr_incr += time.perf_counter() - t1
            ivr.sync()
            room_elapsed = time.perf_counter() - t
            for sid in r_sids:
                ivr.scan_release(sid)
        ivr.close()
        # the whole per-frame pipeline on the device: raw
        # 100k-point frame -> UndistortPcl de-skew + VoxelGrid (filter_size_surf
        # 0.5, livo_scan_preprocess) -> IEKF update (iVox) -> map_incremental
        raws = [synth.make_raw_scan(a.scan_points, s) for s in scan_ids]
        n_down = 0
        prev = None
        for rep in range(2):  # first pass warms the allocations
            t_pre = t_upd = t_inc = 0.0
            sync()
            t = time.perf_counter()
            for (raw, poses, Re, pe), s in zip(raws, st0):
                t1 = time.perf_counter()
                sid, _, down = ctx.scan_preprocess(raw, poses, Re, pe, leaf_size=0.5)
                t2 = time.perf_counter()
                if prev is not None:
                    ctx.scan_inherit_neighbors(sid, prev)
                    ctx.scan_release(prev)
                st, _ = ctx.iekf_update(sid, s)
                t3 = time.perf_counter()
                ctx.map_incremental(sid, st, filter_size_map=0.5)
                t4 = time.perf_counter()
                t_pre += t2 - t1
                t_upd += t3 - t2
                t_inc += t4 - t3
                n_down += len(down)
                prev = sid
            sync()
            pipe_elapsed = time.perf_counter() - t
        ctx.scan_release(prev)
        ctx.set_backend(livo_amd.BACKEND_IKDTREE)
        if rank == 0:
            result["ivox"] = {
                "updates_per_s": round(iv_total.scans / iv_elapsed, 3),
                "ms_per_step": round(iv_elapsed / iv_steps * 1e3, 4),
                "evals_per_scan": round(iv_total.evals / max(iv_total.scans, 1), 3),
                "effct_first_eval_scan0": iv_first[0]["effct_feat_num"][0],
                "map": {"points": iv_info["num_points"], "grids": iv_info["num_grids"],
                        "max_grid_points": iv_info["max_grid_points"], "add_points_s": round(iv_build_s, 3)},
                "odometry": {"scans_per_s": round(len(odo_sids) / odo_elapsed, 3),
                             "ms_per_scan": round(odo_elapsed / len(odo_sids) * 1e3, 3),
                             "map_incremental_ms_per_scan": round(t_incr / len(odo_sids) * 1e3, 3),
                             "points_added_per_scan": round(added / len(odo_sids), 1),
                             "note": "sequential: livo_iekf_update + livo_map_incremental per scan (map grows); "
                                     "second pass over the scans timed (the first warms and grows the map)",
                             "mapped_room": {"ms_per_scan": round(room_elapsed / len(scans) * 1e3, 3),
                                             "scans_per_s": round(len(scans) / room_elapsed, 3),
                                             "map_incremental_ms_per_scan": round(tr_incr / len(scans) * 1e3, 3),
                                             "map_points_before": ivr_before["num_points"],
                                             "max_grid_points_before": ivr_before["max_grid_points"],
                                             "note": "the same odometry on the map the reference's iVox holds: the "
                                                     "first scan (0.5 m voxel-downsampled) grown by 31 mapping scans, "
                                                     "each updated from its true pose then merged by "
                                                     "livo_map_incremental"}},
                "pipeline": {"frames_per_s": round(len(raws) / pipe_elapsed, 3),
                             "ms_per_frame": round(pipe_elapsed / len(raws) * 1e3, 3),
                             "preprocess_ms": round(t_pre / len(raws) * 1e3, 3),
                             "iekf_ms": round(t_upd / len(raws) * 1e3, 3),
                             "map_incremental_ms": round(t_inc / len(raws) * 1e3, 3),
                             "points_after_voxel_grid": round(n_down / (2 * len(raws)), 1),
                             "note": f"raw {a.scan_points // 1000}k-pt frame with 21 IMU poses -> livo_scan_preprocess "
                                     "(de-skew + VoxelGrid 0.5 m) -> livo_iekf_update (iVox) -> livo_map_incremental, "
                                     "host-timed per call (includes the host<->device copies of the raw frame)"},
                "note": "LIVO_BACKEND_IVOX: IVox GetClosestPoint (NEARBY18, 0.2 m grids, 5 m range) on the same "
                        f"{a.batch} scans (rank 0 only), {iv_steps} steps; not part of `value`"}

    # ---- the ikd-Tree incremental map (the USE_ikdtree
    # branch of map_incremental): sequential odometry on a second context
    if "ikd" in legs:
        def odometry(ik_ctx):
            """Two passes of sequential odometry over the first batch's scans (the
            first warms the allocations and activates the incremental map)."""
            rows = []
            for rep in range(2):
                ik_sids = [ik_ctx.scan_upload(sc) for sc in scans]
                t_upd = t_add = 0.0
                events = added = deleted = 0
                sync()
                t = time.perf_counter()
                for sid, s in zip(ik_sids, st0):
                    t1 = time.perf_counter()
                    stn, _ = ik_ctx.iekf_update(sid, s)
                    t2 = time.perf_counter()
                    _, ast = ik_ctx.map_incremental(sid, stn, filter_size_map=0.5)
                    t3 = time.perf_counter()
                    t_upd += t2 - t1
                    t_add += t3 - t2
                    events += ast["events"]
                    added += ast["added"]
                    deleted += ast["deleted"]
                sync()
                elapsed = time.perf_counter() - t
                for sid in ik_sids:
                    ik_ctx.scan_release(sid)
                rows.append((elapsed, t_upd, t_add, events, added, deleted))
            elapsed, t_upd, t_add, events, added, deleted = rows[-1]
            nsc = len(scans)
            return {"scans_per_s": round(nsc / elapsed, 3),
                    "iekf_ms_per_scan": round(t_upd / nsc * 1e3, 3),
                    "add_points_ms_per_scan": round(t_add / nsc * 1e3, 3),
                    "add_points_events_per_scan": round(events / nsc, 1),
                    "points_added_per_scan": round(added / nsc, 1),
                    "points_deleted_per_scan": round(deleted / nsc, 1),
                    "map_points_after": ik_ctx.map_info()["num_points"]}

        ik_ctx = livo_amd.Context(device, t_LI=synth.T_LI, max_iterations=a.max_iter)
        ik_ctx.map_build(m)
        ikd_row = odometry(ik_ctx)
        ik_ctx.close()
        # The reference's own regime: its ikd-Tree is built from the first
        # downsampled scan (laser_mapping.cpp's first-scan Build) and grows by
        # Add_Points with the 0.5 m box downsampling, so the map is the room at
        # one point per box.  Mapping scans (pool scans after the first batch,
        # at their true poses) build it up before the timed odometry passes.
        map_seeds = list(pool_seeds[a.batch:a.batch + 32])
        map_scans = list(pool_scans[a.batch:a.batch + 32])
        if len(map_seeds) < 32:  # a pool of fewer than batch + 32 scans: the rest made here (in-process: the GPU is up)
            extra = [pool_seeds[-1] + 1 + j for j in range(32 - len(map_seeds))]
            map_seeds += extra
            map_scans += gen_scans(a.scan_points, extra, 1)
        R0, p0, _ = synth.true_pose(map_seeds[0])
        w0 = (map_scans[0].astype(np.float64) @ synth.R_LI.T + synth.T_LI) @ R0.T + p0
        _, first = np.unique(np.floor(w0 / 0.5).astype(np.int64), axis=0, return_index=True)
        room_rows = {}
        for runs in ("0", "1"):  # the cell walk (default) / the runs kept on the incremental map (LIVO_DYN_RUNS=1)
            os.environ["LIVO_DYN_RUNS"] = runs  # (read when the map first changes)
            room = livo_amd.Context(device, t_LI=synth.T_LI, max_iterations=a.max_iter)
            room.map_build(np.ascontiguousarray(w0[np.sort(first)], dtype=np.float32))
            for sd, sc in zip(map_seeds[1:], map_scans[1:]):
                sid = room.scan_upload(sc)
                room.map_incremental(sid, synth.make_state(sd, rot_deg=0.0, trans_m=0.0), filter_size_map=0.5)
                room.scan_release(sid)
            room_points = room.map_info()["num_points"]
            room_rows[runs] = odometry(room)
            room.close()
        os.environ.pop("LIVO_DYN_RUNS", None)
        room_row = room_rows["0"]
        room_row["with_runs"] = {k: room_rows["1"][k] for k in ("scans_per_s", "iekf_ms_per_scan", "add_points_ms_per_scan")}
        if rank == 0:
            result["ikd_incremental"] = dict(ikd_row, note=(
                f"sequential odometry on the {a.map_points}-pt map: livo_iekf_update + livo_map_incremental "
                "(ikd-Tree backend: KD_TREE::Add_Points of all scan points, downsample 0.5 m) per scan, "
                "second pass over the scans (the map has grown), host-timed; not part of `value`"))
            result["ikd_incremental"]["mapped_room"] = dict(room_row, map_points_before=room_points, note=(
                f"the same odometry on the map the reference's ikd-Tree holds: built from the first scan "
                f"(0.5 m voxel-downsampled) and grown by {len(map_scans) - 1} mapping scans through "
                "livo_map_incremental at their true poses (one point per 0.5 m box); with_runs: the same with "
                "LIVO_DYN_RUNS=1 (the runs kept on the incremental map)"))

    # ---- the VIO photometric update
    vio_frames = {}
    if "vio" in legs:
        vio = {}
        for nv in (192, 20000):
            fr, vst, _ = synth.make_vio_frame(nv, 100 + rank)
            vio_frames[nv] = (fr, vst)
            ctx.vio_update(fr, vst)  # warm-up
            reps = 20 if nv < 1000 else 10
            sync()
            t = time.perf_counter()
            for _ in range(reps):
                _, vstats, _ = ctx.vio_update(fr, vst)
            sync()
            dt = (time.perf_counter() - t) / reps
            # the same frames from page-locked arrays (livo_host_register: a camera /
            # projection stage writing into pinned buffers); the copy engine reads them
            pf = dict(fr)
            pf["image"] = np.ascontiguousarray(fr["image"], np.uint8)
            pf["pos"] = np.ascontiguousarray(np.asarray(fr["pos"], np.float64).reshape(-1, 3))
            pf["levels"] = np.ascontiguousarray(fr["levels"], np.int32)
            pf["patches"] = np.ascontiguousarray(fr["patches"], np.float32)
            keys = [k for k in ("image", "pos", "levels", "patches") if pf[k].nbytes > 0]
            for k in keys:
                ctx.host_register(pf[k])
            ctx.vio_update(pf, vst)
            sync()
            t = time.perf_counter()
            for _ in range(reps):
                ctx.vio_update(pf, vst)
            sync()
            dtp = (time.perf_counter() - t) / reps
            for k in keys:
                ctx.host_unregister(pf[k])
            vio[str(len(fr["pos"]))] = {"frames_per_s": round(1.0 / dt, 2), "ms_per_frame": round(dt * 1e3, 4),
                                        "ms_per_frame_pinned": round(dtp * 1e3, 4),
                                        "iterations_per_level": vstats["iterations"]}
        if rank == 0:
            result["vio"] = {"by_points": vio,
                             "note": "livo_vio_update (LidarSelector::ComputeJ/UpdateState, patch 4x4, 3 levels, "
                                     "max_iteration 4) on synthetic 640x512 frames, host-timed incl. the frame upload "
                                     "(image, pixel positions, levels, 3-level patches host -> HBM, state back): "
                                     "ms_per_frame from ordinary arrays, ms_per_frame_pinned from page-locked ones "
                                     "(livo_host_register once; the copy engine reads them directly)"}

    # ---- CPU baseline: the oracle (CPU restatement) on this host, BASELINE.md's
    # protocol: 3 warm-ups, then the median of >= 10 timed scan updates (one
    # scan update per timing, steady clock), at 1 thread, the reference's 4
    # (MP_PROC_NUM, CMakeLists.txt:30-33) and every core available to the job;
    # + parity of scan 0 against it
    if rank == 0 and a.cpu_seconds > 0:
        import oracle
        tree = oracle.Tree(m)

        def cpu_median(nt, runs):
            times = []
            for k in range(3 + runs):
                j = k % a.batch
                t = time.perf_counter()
                out_rs = tree.iekf_update(scans[j], st0[j], R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=a.max_iter,
                                          threads=nt)
                if k >= 3:
                    times.append(time.perf_counter() - t)
            return float(np.median(times)), len(times), out_rs

        # runs sized to the --cpu-seconds budget (about a third per thread count), at least 10
        t = time.perf_counter()
        ref0 = tree.iekf_update(scans[0], st0[0], R_LI=np.eye(3), t_LI=synth.T_LI, max_iter=a.max_iter, threads=1)
        one = time.perf_counter() - t
        runs = max(10, min(40, int(a.cpu_seconds / 3 / max(one, 1e-3))))
        med1, n1, _ = cpu_median(1, runs)
        result["cpu_baseline"] = {"value": round(1.0 / med1, 4), "unit": "scan updates/s", "cores": 1,
                                  "kind": "port",
                                  "sample": f"median of {n1} single scan updates after 3 warm-ups "
                                            f"({a.scan_points // 1000}k-pt scans vs {a.map_points}-pt map, "
                                            f"max_iteration={a.max_iter}) by oracle/ (C++ restatement), 1 thread",
                                  **ref_calibration()}
        result["speedup_vs_cpu_1thread"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
        out, rs = ref0
        gs = first_stats[0]
        rel = max(np.linalg.norm(gs["solution"][e] - rs["solution"][e]) / np.linalg.norm(rs["solution"][e])
                  for e in range(min(gs["iterations"], rs["iterations"])))
        result["parity_scan0"] = {"iterations_equal": gs["iterations"] == rs["iterations"],
                                  "effct_equal": gs["effct_feat_num"] == rs["effct_feat_num"],
                                  "max_rel_state_delta": float(f"{rel:.3e}")}
        all_t = host_threads()
        by_threads = {}
        for nt in sorted({4, all_t}):
            med, _, _ = cpu_median(nt, runs)
            by_threads[str(nt)] = round(1.0 / med, 4)
        result["cpu_baseline"]["by_threads"] = by_threads
        result["cpu_baseline"]["host_threads_available"] = all_t
        result["speedup_vs_cpu_all_threads"] = round(result["value"] / by_threads[str(all_t)], 1)
        if "ikfom" in legs:
            ir, irs = tree.ikfom_update(scans[0], synth.make_ikfom_state(scan_ids[0]), max_iter=a.max_iter, threads=8)
            # per evaluation, relative to that evaluation's own step
            irel = max(np.linalg.norm(ik_first["dx"][e] - irs["dx"][e]) / max(np.linalg.norm(irs["dx"][e]), 1e-300)
                       for e in range(min(ik_first["iterations"], irs["iterations"])))
            result["ikfom"]["parity_scan0"] = {"iterations_equal": ik_first["iterations"] == irs["iterations"],
                                               "effct_equal": ik_first["effct_feat_num"] == irs["effct_feat_num"],
                                               "max_rel_dx_per_eval": float(f"{irel:.3e}")}
        if "ivox" in legs:
            ivo = oracle.Ivox()
            ivo.add_points(m)
            t = time.perf_counter()
            ivs, ivst = ivo.iekf_update(scans[0], st0[0], oracle.new_cache(len(scans[0])), t_LI=synth.T_LI,
                                        max_iter=a.max_iter, threads=1)
            iv_cpu_s = time.perf_counter() - t
            ig = iv_first[0]
            ivrel = max(np.linalg.norm(ig["solution"][e] - ivst["solution"][e]) / np.linalg.norm(ivst["solution"][e])
                        for e in range(min(ig["iterations"], ivst["iterations"])))
            result["ivox"]["cpu_baseline"] = {"value": round(1.0 / iv_cpu_s, 4), "unit": "scan updates/s",
                                              "cores": 1, "kind": "port",
                                              "sample": "1 full scan update of scan 0 by oracle/ (IVox "
                                                        f"restatement), 1 thread, {iv_cpu_s:.2f} s"}
            raw, poses, Re, pe = raws[0]
            t = time.perf_counter()
            und = oracle.undistort(raw, poses, Re, pe, t_LI=synth.T_LI)
            oracle.voxel_grid(und, 0.5)
            result["ivox"]["pipeline"]["cpu_preprocess_ms"] = round((time.perf_counter() - t) * 1e3, 3)
            result["ivox"]["parity_scan0"] = {"iterations_equal": ig["iterations"] == ivst["iterations"],
                                              "effct_equal": ig["effct_feat_num"] == ivst["effct_feat_num"],
                                              "max_rel_state_delta": float(f"{ivrel:.3e}")}
        if "ikd" in legs:
            dyn = oracle.DynMap(m)
            t = time.perf_counter()
            dyn.map_incremental(scans[0], first_states[0], t_LI=synth.T_LI, filter_size_map=0.5)
            result["ikd_incremental"]["cpu_add_points_ms"] = round((time.perf_counter() - t) * 1e3, 3)
            del dyn
        for nv, (fr, vst) in vio_frames.items():
            t = time.perf_counter()
            vr, vrs, _ = oracle.vio_update(fr, vst)
            key = str(len(fr["pos"]))
            result["vio"]["by_points"][key]["cpu_ms_per_frame"] = round((time.perf_counter() - t) * 1e3, 3)
        if vio_frames:
            vg, vgs, _ = ctx.vio_update(*vio_frames[20000])
            result["vio"]["parity_20k"] = {"iterations_equal": vgs["iterations"] == vrs["iterations"],
                                           "max_abs_pos_delta": float(f"{np.abs(vg['pos'] - vr['pos']).max():.3e}")}
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
