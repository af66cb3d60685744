"""Per-evaluation dispatch durations of k_iekf_eval by stream group, from a rocprofv3 kernel trace.

Each stream group's batch is k_iekf_eval<true> followed by max_iteration (4) k_iekf_eval<false>
on the group's stream; this lines up the dispatches of every group of a batch by position and
prints, per position, the mean duration over the batches and the mean ratio of the slowest
group's dispatch to the fastest's (the groups of one batch run concurrently).
usage: python tools/kt_evals.py <kernel_trace.csv> [evals=5] [skip_batches=4]
"""
import collections
import csv
import sys


def main(path, evals="5", skip="4"):
    evals, skip = int(evals), int(skip)
    rows = [r for r in csv.DictReader(open(path)) if "k_iekf_eval" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per_stream = collections.defaultdict(list)
    for r in rows:
        per_stream[r["Stream_Id"]].append(r)
    # per stream: split into batches at each k_iekf_eval<true>
    batches = collections.defaultdict(list)  # stream -> list of [durations...]
    for sid, rs in per_stream.items():
        cur = None
        for r in rs:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if "<true>" in r["Kernel_Name"]:
                cur = [d]
                batches[sid].append(cur)
            elif cur is not None and len(cur) < evals:
                cur.append(d)
    streams = sorted(batches)
    nb = min(len(batches[s]) for s in streams)
    print(f"streams {len(streams)}, batches per stream {nb} (first {skip} skipped)")
    for e in range(evals):
        means, ratios = [], []
        for b in range(skip, nb):
            ds = [batches[s][b][e] for s in streams if len(batches[s][b]) > e]
            if len(ds) < 2:
                continue
            means.append(sum(ds) / len(ds))
            ratios.append(max(ds) / min(ds))
        if means:
            print(f"eval {e}: mean dispatch {sum(means) / len(means):.1f} us, slowest/fastest group "
                  f"{sum(ratios) / len(ratios):.2f} (max {max(ratios):.2f})")


if __name__ == "__main__":
    main(*sys.argv[1:])
