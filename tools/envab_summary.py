"""Summary of a tools/gpu_envab.sh run: per configuration, the bench lines (G ops/s, ms/step, local
launch ms) and the rocprofv3 average duration of the main kernels.   python tools/envab_summary.py TAG"""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
d = f"gpurun_out/{tag}"
cfgs = open(f"{d}/configs.txt").read().split("\n")
keys = ("k_local_pre", "k_local_fused", "k_local_deferred", "k_commit_w", "k_marshal_invs", "k_ack_offsets",
        "k_unique_lds", "k_peer_acks", "k_unique_rows", "k_lookup", "k_refill_plan", "k_peer_ts")
for k, c in enumerate(x for x in cfgs if x):
    vals = []
    for f in sorted(glob.glob(f"{d}/b_{k}_*.log")):
        lines = [l for l in open(f) if l.startswith("{")]
        if lines:
            j = json.loads(lines[-1])
            vals.append(f"{j['value'] / 1e9:.3f}/{j['ms_per_step']:.4f}/{j['roofline']['launch_ms']:.4f}")
    st = glob.glob(f"{d}/p{k}/**/*kernel_stats.csv", recursive=True)
    kern = {}
    if st:
        for r in csv.DictReader(open(st[0])):
            n = r["Name"].replace("void ", "").replace("hkv::", "")
            for key in keys:
                if n.startswith(key):
                    kern[key] = kern.get(key, []) + [round(float(r["AverageNs"]) / 1e3, 1)]
    print(f"[{k}] {c or 'defaults'}: {' '.join(vals)}")
    print("     " + " ".join(f"{a}={'/'.join(map(str, b))}" for a, b in kern.items()))
