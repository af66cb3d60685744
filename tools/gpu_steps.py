"""Run GPU steps in order on the box; stop at the first hard failure.

usage: python tools/gpu_steps.py "<timeout_s>::<log name>::<command>" ...

Each step runs under its own time limit with output in gpurun_out/<log>.
A step that exits 0 or 1 (pass / ordinary test or assertion failure) lets the
next step run; anything else (abort 134, segfault 139, time limit 124/137,
negative signal codes) ends the call: nothing more touches the GPU.
"""
import os
import subprocess
import sys

os.makedirs("gpurun_out", exist_ok=True)
worst = 0
for spec in sys.argv[1:]:
    tmo, log, cmd = spec.split("::", 2)
    with open(os.path.join("gpurun_out", log), "w") as f:
        f.write(f"$ {cmd}\n")
        f.flush()
        rc = subprocess.call(["timeout", "-k", "10", tmo, "bash", "-c", cmd], stdout=f, stderr=subprocess.STDOUT)
    print(f"[step] rc={rc} {log}: {cmd}", flush=True)
    worst = max(worst, 0 if rc == 0 else 1)
    if rc not in (0, 1):
        print("[step] hard failure: stopping", flush=True)
        sys.exit(rc if rc > 0 else 2)
sys.exit(worst)
