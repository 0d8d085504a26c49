"""Average kernel durations (us) from rocprofv3 --stats runs: python tools/kstats.py DIR... [filter]"""
import csv
import glob
import sys

args = sys.argv[1:]
flt = args.pop() if args and not args[-1].startswith("gpurun_out") else ""
for d in args:
    for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
        print(d)
        for r in csv.DictReader(open(f)):
            n = r["Name"].split("(")[0].replace("void ", "").replace("hkv::", "")
            if flt in n:
                print(f"   {n[:40]:40s} {float(r['AverageNs']) / 1e3:8.1f} us  x{r['Calls']}")
