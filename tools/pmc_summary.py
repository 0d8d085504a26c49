"""Per-kernel PMC summary from tools/pmc.sh output: python tools/pmc_summary.py TAG
Prints the mean per dispatch of every counter collected (FETCH_SIZE/WRITE_SIZE in MB; FETCH_SIZE
also doubled: on gfx950 it reports half the bytes of wide reads, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}/pmc/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("hkv::", "")
        if "rocprim" in name:
            short = "rocprim:" + ("onesweep" if "onesweep" in name else "scan" if "scan" in name else "other")
        res[(short, r.get("Grid_Size", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for v in res.values() for c in v})
short = lambda c: c.replace("TCC_EA0_", "").replace("_sum", "")[:14]  # noqa: E731
hdr = f"{'kernel':40s} {'grid':>9s} " + " ".join(f"{short(c):>14s}" for c in cols)
print(hdr)
def key(kv):
    v = kv[1].get(cols[0], [0])
    return -sum(v) / max(1, len(v))
for (k, g), v in sorted(res.items(), key=key):
    vals = []
    for c in cols:
        x = v.get(c, [])
        m = sum(x) / len(x) if x else float("nan")
        if c in ("FETCH_SIZE", "WRITE_SIZE"):
            m /= 1024.0  # KB -> MB
        if c == "FETCH_SIZE":
            m *= 2.0     # gfx950: half the bytes of wide reads (128-B requests tallied at 64 B)
        vals.append(f"{m:14.1f}")
    print(f"{k[:40]:40s} {g:>9s} " + " ".join(vals))
