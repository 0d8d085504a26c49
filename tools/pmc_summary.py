"""Per-kernel HBM traffic from tools/pmc.sh output: python tools/pmc_summary.py TAG
FETCH_SIZE is doubled (gfx950: it reports half the bytes of wide reads, MI355X_MICROARCH.md)."""
import csv, sys, collections
tag = sys.argv[1]
res = collections.defaultdict(lambda: {"FETCH_SIZE": [], "WRITE_SIZE": []})
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(f"gpurun_out/{tag}/pmc/{c}/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("hkv::", "")
        if "rocprim" in name:
            short = "rocprim:" + ("onesweep" if "onesweep" in name else "scan" if "scan" in name else "other")
        grid = r.get("Grid_Size", "")
        res[(short, grid)][c].append(float(r["Counter_Value"]))
print(f"{'kernel':44s} {'grid':>9s} {'n':>4s} {'fetch MB':>9s} {'x2 MB':>8s} {'write MB':>9s}")
for (k, g), v in sorted(res.items(), key=lambda kv: -sum(kv[1]["FETCH_SIZE"] or [0]) / max(1, len(kv[1]["FETCH_SIZE"]))):
    f = v["FETCH_SIZE"]; w = v["WRITE_SIZE"]
    fa = sum(f) / len(f) / 1024 if f else float("nan")   # KB -> MB
    wa = sum(w) / len(w) / 1024 if w else float("nan")
    print(f"{k[:44]:44s} {g:>9s} {len(f):4d} {fa:9.1f} {2*fa:8.1f} {wa:9.1f}")
