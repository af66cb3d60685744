"""Split a rocprofv3 kernel trace into phases at idle gaps and print per-phase kernel stats.

bench.py runs its legs one after the other with host work between them (the
config-5 leg builds a 10M-point map for several seconds first), so an idle gap
of more than `gap_s` seconds separates the headline's dispatches from
config 5's.  Prints, per phase, the same columns as rocprofv3's
kernel_stats.csv (name, calls, total ns, average ns, min, max).
usage: python tools/kt_phases.py <kernel_trace.csv> [gap_s=1.0]
"""
import csv
import sys
from collections import defaultdict


def main(path, gap_s="1.0"):
    gap = float(gap_s) * 1e9
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > gap and cur:
            phases.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], e - s))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        phases.append(cur)
    for i, ph in enumerate(phases):
        st = defaultdict(list)
        for name, d in ph:
            st[name].append(d)
        tot = sum(sum(v) for v in st.values())
        print(f"# phase {i}: {len(ph)} dispatches, {tot / 1e6:.3f} ms kernel time")
        print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
        for name, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
            print(f'"{name[:160]}",{len(v)},{sum(v)},{sum(v) / len(v):.1f},{100 * sum(v) / tot:.2f},{min(v)},{max(v)}')


if __name__ == "__main__":
    main(*sys.argv[1:3])
