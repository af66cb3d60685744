"""One batch step's kernel timeline from a rocprofv3 --kernel-trace CSV.

A step starts at a first-evaluation dispatch (k_iekf_eval<true>, or
k_knn_leaf<false> / k_knn_grid<false> in the unfused builds); the window runs
to the next such dispatch group.  Copies (__amd_rocclr_copyBuffer) are listed
with the kernels.  Prints
every dispatch in the window (queue, start offset, duration, name) and a
per-kernel-name summary of busy time, so launch gaps and the critical path
of the stream groups are visible.
usage: python tools/kt_timeline.py <kernel_trace.csv> [step_index=-3] [groups=1]
"""
import csv
import sys


def main(path, step="-3", groups="1"):
    step, groups = int(step), int(groups)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    firsts = [r for r in rows if "k_iekf_eval<true>" in r["Kernel_Name"]] or \
        [r for r in rows if "<false>" in r["Kernel_Name"] and "k_knn_" in r["Kernel_Name"] and "replay" not in r["Kernel_Name"]]
    starts = [int(r["Start_Timestamp"]) for r in firsts[::groups]]
    t0 = starts[step]
    t1 = starts[step + 1] if step + 1 < len(starts) and step != -1 else None
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and (t1 is None or int(r["Start_Timestamp"]) < t1)]
    qs = {q: i for i, q in enumerate(sorted({r["Queue_Id"] for r in win}))}
    busy = {}
    for r in win:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].replace("livo::", "").split("(")[0].replace("void ", "")
        busy[name] = busy.get(name, 0) + (e - s)
        print(f"q{qs[r['Queue_Id']]} {s / 1e3:8.1f} us  +{(e - s) / 1e3:7.1f}  {name}")
    end = max(int(r["End_Timestamp"]) for r in win) - t0
    print(f"window {end / 1e3:.1f} us (next step at {(t1 - t0) / 1e3 if t1 else float('nan'):.1f} us)")
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"  {k:32s} {v / 1e3:8.1f} us busy")


if __name__ == "__main__":
    main(*sys.argv[1:4])
