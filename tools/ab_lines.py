"""Bench lines of a tools/ab_lib.sh session: per library and rep, value, ms/step and per-launch times.
    python tools/ab_lines.py TAG"""
import glob
import json
import os
import sys

d = os.path.join("gpurun_out", sys.argv[1])
idx = {}
if os.path.exists(os.path.join(d, "index.txt")):
    for line in open(os.path.join(d, "index.txt")):
        k, v = line.strip().split(": ", 1)
        idx[k] = v
for f in sorted(glob.glob(os.path.join(d, "l*_*.log"))):
    name = os.path.basename(f)[:-4]
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(name, "no bench line")
        continue
    j = json.loads(lines[-1])
    la = j["roofline"]["launches"]
    t = " ".join(f"{k}={1e3 * v['ms']:.1f}" for k, v in la.items() if isinstance(v, dict) and "ms" in v)
    lib = idx.get(name.split("_")[0], "")
    print(f"{name:6s} {j['value'] / 1e9:.3f} G  {j['ms_per_step']:.4f} ms  {t}  {os.path.basename(os.path.dirname(lib)) or lib}")
