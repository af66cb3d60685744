"""Per-evaluation PMC summary of the fused IEKF kernel (tools/pmc_quick.sh output).

tools/knn_probe.py runs batches of max_iteration + 1 = 5 k_iekf_eval
dispatches each (one k_iekf_eval<true>, then four k_iekf_eval<false>); this
splits the <false> dispatches by their position in the batch, so the
rematch evaluation (position 3 in the bench's batch: every scan searches
again at iterCount == NUM_MAX_ITERATIONS - 2) and the cached-plane ones are
reported apart.  Prints, per position, the mean of every counter and a few
ratios (VALU instructions per wave, L2 hit rate, wait share).
usage: python tools/pmc_evals.py <pmc_dir> [evals=5]
"""
import collections
import csv
import glob
import os
import sys


def main(d, evals="5"):
    evals = int(evals)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if "k_iekf_eval" not in r["Kernel_Name"]:
                continue
            acc[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        order = sorted(names)
        pos, k = {}, -1
        for disp in order:  # position within the batch: 0 at each <true> dispatch
            k = 0 if "<true>" in names[disp] else k + 1
            pos[disp] = k
        for (disp, cname), v in acc.items():
            per[pos[disp]][cname].append(v)
    for p in sorted(per):
        cs = {c: sum(v) / len(v) for c, v in per[p].items()}
        n = max(len(v) for v in per[p].values())
        line = [f"eval {p} ({n} dispatches)"]
        w = cs.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"):
                if c in cs:
                    line.append(f"{c[9:]}/wave {cs[c] / w:.0f}")
        if cs.get("SQ_WAVE_CYCLES"):
            line.append(f"wait_any {cs.get('SQ_WAIT_ANY', 0) / cs['SQ_WAVE_CYCLES']:.3f}")
            line.append(f"wave_cycles {cs['SQ_WAVE_CYCLES']:.3e}")
        if cs.get("TCC_HIT_sum") is not None and cs.get("TCC_MISS_sum"):
            line.append(f"l2_hit {cs['TCC_HIT_sum'] / (cs['TCC_HIT_sum'] + cs['TCC_MISS_sum']):.3f}")
        if "FETCH_SIZE" in cs:
            line.append(f"fetch {cs['FETCH_SIZE'] / 1024:.1f} MiB")
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in cs:
            line.append(f"tcp_acc {cs['TCP_TOTAL_CACHE_ACCESSES_sum']:.3e}")
        print("  ".join(line))


if __name__ == "__main__":
    main(*sys.argv[1:3])
