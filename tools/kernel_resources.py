"""Per-kernel register / scratch / LDS / occupancy table of the device sources
(development tool): compiles each .hip of build.SOURCES with the build's own
flags plus -Rpass-analysis=kernel-resource-usage and prints a markdown table.

    python tools/kernel_resources.py [--md OUT.md] [-DMACRO=VALUE ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-livo-noted_amd"))
import build as B  # noqa: E402

KEYS = [("VGPRs", "VGPRs"), ("AGPRs", "AGPRs"), ("TotalSGPRs", "SGPRs"), ("ScratchSize [bytes/lane]", "scratch B/lane"),
        ("Occupancy [waves/SIMD]", "waves/SIMD"), ("LDS Size [bytes/block]", "LDS B/block"),
        ("VGPRs Spill", "VGPR spill"), ("SGPRs Spill", "SGPR spill")]


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.split("\n")
    return out[:len(names)]


def resources(src, flags):
    cmd = [B.HIPCC] + B.COMMON + B.DEVICE + ["-x", "hip"] + flags + ["--cuda-device-only", "-c", "-o", os.devnull,
                                                                      os.path.join(B.CSRC, src),
                                                                      "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1), "src": src}
            rows.append(cur)
            continue
        for key, _ in KEYS:
            m = re.search(r"\s" + re.escape(key) + r": (\d+)", line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return [r for r in rows if "Occupancy [waves/SIMD]" in r]  # kernels only (device functions have none)


def main():
    args = sys.argv[1:]
    md = None
    if "--md" in args:
        i = args.index("--md")
        md = args[i + 1]
        del args[i:i + 2]
    rows = []
    for src, dev in B.SOURCES:
        if dev:
            rows += resources(src, args)
    names = demangle([r["name"] for r in rows])
    lines = ["| kernel | source | " + " | ".join(h for _, h in KEYS) + " |",
             "|---|---|" + "---|" * len(KEYS)]
    for r, n in zip(rows, names):
        if "rocprim" in n:  # (the library's sort / scan instantiations in prims.hip)
            continue
        n = re.sub(r"^void ", "", n)
        n = re.sub(r"^livo::", "", n)
        n = re.sub(r"\(.*\)$", "", n)
        lines.append(f"| `{n}` | {r['src']} | " + " | ".join(str(r.get(k, "")) for k, _ in KEYS) + " |")
    text = "\n".join(lines) + "\n"
    if md:
        with open(md, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
