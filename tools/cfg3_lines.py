"""bench lines of a tools/gpu_r06_cfg3.sh session, and the top kernels of its trace:
    python tools/cfg3_lines.py TAG"""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
d = f"gpurun_out/{tag}"
for f in sorted(glob.glob(f"{d}/*_[12].log")):
    lines = [x for x in open(f) if x.startswith("{")]
    if lines:
        j = json.loads(lines[-1])
        print(f"{os.path.basename(f)[:-4]:12s} {j['value'] / 1e6:8.1f} M  {j['ms_per_step']:.4f} ms")
p = f"{d}/prof/run_kernel_stats.csv"
if os.path.exists(p):
    for r in list(csv.DictReader(open(p)))[:14]:
        print(f"{r['Name'][:70]:72s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1000:9.1f} us")
