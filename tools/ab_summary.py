"""Summarise tools/ab_run.sh output: per variant, mean/min/max of the bench value
and of the per-stage device times.  usage: python tools/ab_summary.py [dir=gpurun_out]"""
import glob
import json
import os
import sys


def main(d="gpurun_out"):
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "ab_*_*.log"))):
        name = os.path.basename(f)[3:-4].rsplit("_", 1)[0]
        lines = [x for x in open(f) if x.startswith("{")]
        if not lines:
            print("no JSON in", f)
            continue
        j = json.loads(lines[-1])
        dm = j.get("device_ms_per_step", {})
        res.setdefault(name, []).append((j["value"], dm.get("eval_first", dm.get("knn_first", 0)),
                                         dm.get("eval_rematch", dm.get("knn_rematch", 0)),
                                         dm.get("eval_nosearch", dm.get("plane_H_solve", 0)),
                                         dm.get("host_gap", 0), j.get("knn_replays_per_step", 0)))
    print(f"{'variant':12s} {'n':>2s} {'value mean':>10s} {'min':>8s} {'max':>8s} {'first':>6s} {'rematch':>7s} "
          f"{'nosrch':>6s} {'gap':>6s} {'replays':>7s}")
    for k, v in res.items():
        n = len(v)
        m = [sum(x[i] for x in v) / n for i in range(6)]
        print(f"{k:12s} {n:2d} {m[0]:10.1f} {min(x[0] for x in v):8.1f} {max(x[0] for x in v):8.1f} "
              f"{m[1]:6.3f} {m[2]:7.3f} {m[3]:6.3f} {m[4]:6.3f} {m[5]:7.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
