"""Per-batch span of the first-evaluation k-NN from a rocprofv3 kernel trace.

bench.py's roofline unit is the first evaluation of one batch: one
k_iekf_eval<true> (fused default; k_knn_grid<false>/k_knn_leaf<false> in the
unfused builds) dispatch per stream group (2 groups run concurrently) plus
their tie replays, timed with HIP events as the wall time from the batch's
start to the last group's end.  This groups the k_knn_leaf<false> dispatches
of a rocprofv3 --kernel-trace run into batches of `groups` and reports the
mean span (first start -> last end, extended to the replay dispatch that
follows each one on its queue) so it can be compared with bench's
roofline.avg_launch_ms.
usage: python tools/kt_span.py <kernel_trace.csv> [groups=2] [skip_batches=4] [max_batches=all]
(max_batches: only the headline run's batches, before the later legs of bench.py)
"""
import csv
import sys


def main(path, groups="2", skip="4", max_batches="0"):
    groups, skip, mb = int(groups), int(skip), int(max_batches)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    by_q = {}
    for r in rows:
        by_q.setdefault(r["Queue_Id"], []).append(r)
    items = []  # (start, end incl. following replay) per k_knn_leaf<false> dispatch
    for q, rs in by_q.items():
        for i, r in enumerate(rs):
            if any(k in r["Kernel_Name"] for k in ("k_knn_leaf<false>", "k_knn_grid<false", "k_iekf_eval<true>")):
                end = int(r["End_Timestamp"])
                if i + 1 < len(rs) and "k_knn_replay" in rs[i + 1]["Kernel_Name"]:
                    end = int(rs[i + 1]["End_Timestamp"])
                items.append((int(r["Start_Timestamp"]), end, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    items.sort()
    if mb > 0:
        items = items[:mb * groups]
    spans, durs = [], [d for _, _, d in items]
    for b in range(skip, len(items) // groups):
        chunk = items[b * groups:(b + 1) * groups]
        spans.append(max(e for _, e, _ in chunk) - min(s for s, _, _ in chunk))
    print(f"first-evaluation dispatches (fused, grid or leaf): {len(items)}, mean dispatch {sum(durs) / len(durs) / 1e3:.1f} us")
    print(f"batches of {groups}: {len(spans)} (first {skip} skipped), mean first-eval k-NN span "
          f"{sum(spans) / len(spans) / 1e3:.1f} us (min {min(spans) / 1e3:.1f}, max {max(spans) / 1e3:.1f})")


if __name__ == "__main__":
    main(*sys.argv[1:5])
