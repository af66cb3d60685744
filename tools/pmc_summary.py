"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel -> JSON.

HBM traffic of the bench's roofline unit (the first evaluation of one batch):
the batch runs as `groups` stream groups, each with one k_iekf_eval<true>
dispatch (k_knn_grid<false> / k_knn_leaf<false> in the unfused builds), so

    traffic = groups * (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024

MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads 1/2 of the bytes of a
wide coalesced streaming read (doubled here); other access widths are
uncalibrated, so the raw figure is recorded alongside.  Dispatches are grouped
by (kernel, grid size) and the most frequent grid of each kernel is taken: the
timed steps' dispatches, not the bench's one-off V_ref passes.
usage: python tools/pmc_summary.py <pmc_dir> <workload tag> <out.json> [groups=1]
"""
import collections
import csv
import glob
import json
import os
import sys

UNIT_KERNELS = ("k_iekf_eval<true>", "k_knn_leaf<false>", "k_knn_grid<false>")


def main(d, workload, out, groups="1"):
    groups = int(groups)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(collections.Counter)
    for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            acc[(r["Dispatch_Id"], r["Kernel_Name"], r["Grid_Size"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, kname, grid, cname), v in acc.items():
            per[(kname, grid)][cname].append(v)
            if cname in ("FETCH_SIZE", "SQ_WAVES"):
                grids[kname][grid] += 1
    res = {"workload": workload, "groups": groups, "kernels": {}}
    for kname, cnt in grids.items():
        grid = cnt.most_common(1)[0][0]
        cs = per[(kname, grid)]
        res["kernels"][kname] = {"grid": int(grid), **{c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()}}
    raw = corr = 0.0
    found = []
    for k, kc in res["kernels"].items():
        if not any(u in k for u in UNIT_KERNELS):
            continue
        fetch = kc.get("FETCH_SIZE", {}).get("mean")
        write = kc.get("WRITE_SIZE", {}).get("mean")
        if fetch is None or write is None:
            continue
        found.append(k)
        raw += (fetch + write) * 1024
        corr += (2 * fetch + write) * 1024
        hit, miss = kc.get("TCC_HIT_sum", {}).get("mean"), kc.get("TCC_MISS_sum", {}).get("mean")
        if hit is not None and miss:
            kc["l2_hit_rate"] = hit / (hit + miss)
    if found:
        res["hbm_bytes_per_launch_raw"] = groups * raw
        res["hbm_bytes_per_launch"] = groups * corr
        res["unit_kernels"] = found
        res["note"] = ("per first-evaluation k-NN of one batch: groups x k-NN first-search dispatch (leaf or grid); FETCH_SIZE "
                       "doubled per MI355X_MICROARCH.md §HBM (gfx950 reports 1/2 of wide reads); gather widths are "
                       "uncalibrated, raw value kept alongside")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
