"""One Add_Points call's device timeline from a rocprofv3 kernel trace of the
bench's ikd leg (development tool; runs on the trace CSV, no GPU).

    python tools/ikd_trace_summary.py KERNEL_TRACE.csv [CALL_INDEX]

Prints the kernels from k_add_prep to the rebuild's k_dyn_slots of the chosen
call (start offset, duration, grid size, name) and, over every call, the
average device time per kernel of those spans.
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    starts = [i for i, x in enumerate(rows) if "k_add_prep" in x["Kernel_Name"]]
    spans = []
    for j in starts:
        k, span = j, []
        while k < len(rows):
            span.append(rows[k])
            if "k_dyn_slots" in rows[k]["Kernel_Name"]:
                break
            k += 1
        spans.append(span)
    span = spans[min(pick, len(spans) - 1)]
    t0 = int(span[0]["Start_Timestamp"])
    print(f"Add_Points call {min(pick, len(spans) - 1)} of {len(spans)}: start offset / duration (us), grid, kernel")
    for x in span:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        name = x["Kernel_Name"].split("(")[0].replace("void ", "")
        if "rocprim" in name:
            name = "rocprim " + ("scan" if "scan" in x["Kernel_Name"] else "sort/other")
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {x['Grid_Size_X']:>8} {name[:70]}")
    last = span[-1]
    print(f"span {(int(last['End_Timestamp']) - t0) / 1e3:.1f} us, device busy "
          f"{sum(int(x['End_Timestamp']) - int(x['Start_Timestamp']) for x in span) / 1e3:.1f} us, {len(span)} kernels")
    tot = collections.defaultdict(float)
    for sp in spans:
        for x in sp:
            name = x["Kernel_Name"].split("(")[0].replace("void ", "")
            if "rocprim" in name:
                name = "rocprim (sort / scan kernels)"
            tot[name] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    print(f"\naverage device time per call over {len(spans)} calls (us):")
    for name, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{t / len(spans):9.1f}  {name[:80]}")


if __name__ == "__main__":
    main()
