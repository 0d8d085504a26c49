"""A/B summary of tools/gpu_abt.sh output: python tools/absum.py TAG"""
import csv
import glob
import json
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}/b_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]["launches"]
            print(f.split("/")[-1], f"{d['value'] / 1e9:.3f} G/s", f"{d['ms_per_step']:.4f} ms/step",
                  {k: round(v["ms"] * 1e3, 1) for k, v in r.items()}, "flags", d["detail"].get("error_flags"))
for f in glob.glob(f"gpurun_out/{tag}/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hkv" in r["Name"]:
            print(" ", r["Name"].split("(")[0].replace("void ", "")[:40].ljust(40), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
