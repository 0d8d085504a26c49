"""Bench values and local-launch times of an A/B session (tools/gpu_r05*.sh layout: configs.txt,
b_<k>_<rep>.log, p<k>/ kernel stats):  python tools/ab_summary2.py TAG [kernel filter]"""
import csv
import glob
import json
import sys

tag = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "k_local"
d = f"gpurun_out/{tag}"
cfgs = open(f"{d}/configs.txt").read().split("\n")
for k, c in enumerate(cfgs):
    if not c and k:
        continue
    vals, loc = [], []
    for f in sorted(glob.glob(f"{d}/b_{k}_*.log")):
        try:
            j = json.loads(open(f).read().strip().splitlines()[-1])
            vals.append(round(j["value"] / 1e9, 3))
            loc.append(round(j["roofline"]["launch_ms"] * 1e3, 1))
        except Exception as e:  # noqa: BLE001
            vals.append(f"ERR {str(e)[:30]}")
    ks = []
    for f in glob.glob(f"{d}/p{k}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Name"].split("(")[0].replace("void ", "").replace("hkv::", "")
            if flt in n:
                ks.append(f"{n[:34]} {float(r['AverageNs']) / 1e3:.1f}")
    print(f"{k} {c!r}: G ops/s {vals}  local us {loc}")
    for x in ks:
        print("      ", x)
