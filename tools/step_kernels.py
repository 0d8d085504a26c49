"""Print every kernel of one bench step (the last step delimited by the refill (k_refill* or k_plan_peer_ts) of the timed region)
from a rocprofv3 kernel trace: name, grid, duration, gap to the previous kernel.
    python tools/step_kernels.py TAG [step_from_end]"""
import csv
import glob
import sys

tag = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
f = glob.glob(f"gpurun_out/{tag}/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_refill" in r["Kernel_Name"] or "k_plan_peer_ts" in r["Kernel_Name"]]
a, b = starts[-back - 1], starts[-back]
prev = None
tot = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hkv::", "")[:38]
    gap = (s - prev) / 1e3 if prev else 0.0
    tot += (e - s) / 1e3
    print(f"{name:40s} grid {int(r['Grid_Size_X']):>9d}  {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}")
    prev = e
print(f"kernel sum {tot:.1f} us, wall {(int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
