"""Summary of an A/B session (tools/gpu_abm.sh, tools/gpu_abt.sh): per configuration, every rep's
value, ms/step and per-launch-type times from the bench lines.   python tools/ab_summary.py TAG"""
import glob
import json
import os
import re
import sys

d = os.path.join("gpurun_out", sys.argv[1])
cfgs = {}
names = {}
if os.path.exists(os.path.join(d, "configs.txt")):
    for k, line in enumerate(open(os.path.join(d, "configs.txt")).read().split("\n")[:-1]):
        names[str(k)] = line or "defaults"
for f in sorted(glob.glob(os.path.join(d, "b_*_*.log"))):
    m = re.match(r"b_(.+)_(\d+)\.log", os.path.basename(f))
    line = [x for x in open(f).read().splitlines() if x.startswith("{")]
    if not m or not line:
        continue
    j = json.loads(line[-1])
    launches = j.get("roofline", {}).get("launches", {})
    t = " ".join(f"{k}={1e3 * v['ms']:.1f}" for k, v in launches.items() if isinstance(v, dict) and 'ms' in v)
    cfgs.setdefault(m.group(1), []).append(f"{j['value'] / 1e9:.3f} G  {j['ms_per_step']:.3f} ms  {t}")
for k, v in cfgs.items():
    print(f"[{names.get(k, k)}]")
    for x in v:
        print("   ", x)
