"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel -> JSON.

HBM traffic per launch = (FETCH_SIZE + WRITE_SIZE) KiB * 1024 for the
dominant kernel.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads 1/2 of
the bytes of a wide coalesced streaming read; other access widths are
uncalibrated.  Both the raw and the x2-corrected fetch figures are recorded.
usage: python tools/pmc_summary.py <pmc_dir> <workload tag> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, workload, out):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        # one row per (dispatch, counter)
        acc = collections.defaultdict(float)
        for r in rows:
            acc[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, kname, cname), v in acc.items():
            per[kname][cname].append(v)
    res = {"workload": workload, "kernels": {}}
    for k, cs in per.items():
        res["kernels"][k] = {c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()}
    dom = [k for k in res["kernels"] if "k_knn_pass<false>" in k]
    if dom:
        kc = res["kernels"][dom[0]]
        fetch = kc.get("FETCH_SIZE", {}).get("mean")
        write = kc.get("WRITE_SIZE", {}).get("mean")
        if fetch is not None and write is not None:
            res["hbm_bytes_per_launch_raw"] = (fetch + write) * 1024
            res["hbm_bytes_per_launch"] = (2 * fetch + write) * 1024
            res["note"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports 1/2 of wide reads); "
                           "gather widths are uncalibrated, raw value kept alongside")
        hit, miss = kc.get("TCC_HIT_sum", {}).get("mean"), kc.get("TCC_MISS_sum", {}).get("mean")
        if hit is not None and miss:
            res["l2_hit_rate"] = hit / (hit + miss)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
