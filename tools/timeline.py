"""Per-step kernel timeline from a rocprofv3 kernel trace (csv): python tools/timeline.py TAG [--full]"""
import csv, sys, collections
tag = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/{tag}/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_refill" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
phase = "refill"
agg = collections.OrderedDict()
prev = t0
for r in rows[a:b]:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    short = n.split("(")[0].replace("void ", "").replace("hkv::", "")
    if "rocprim" in n:
        short = "rocprim"
    if "k_lookup" in n:
        phase = {0: "local", 1: "inv", 2: "ack", 3: "val"}[sum(1 for x in agg if x.endswith("lookup"))]
    key = f"{phase}:{short.split('<')[0]}"
    d = agg.setdefault(key, [0.0, 0, 0.0])
    d[0] += (e - s) / 1e3
    d[1] += 1
    d[2] += max(0, s - prev) / 1e3
    prev = e
    if "--full" in sys.argv:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {short[:60]}")
tot = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
BATCH = ("k_lookup", "__amd_rocclr_fillBufferAligned", "rocprim", "k_segment_exec", "k_round_cand",
         "k_round_apply", "k_round_resolve", "k_long_exec")
sums = collections.OrderedDict()
for k, (d, c, g) in agg.items():
    ph, name = k.split(":", 1)
    if name in BATCH:
        sums[ph] = sums.get(ph, 0.0) + d
print("batch launch = sum of its kernels (compare bench.py roofline.batch_ms):",
      {k: round(v / 1e3, 4) for k, v in sums.items()}, "ms")
for k, (d, c, g) in agg.items():
    print(f"{k:32s} {d:8.1f} us  x{c:<3d} gaps {g:6.1f}")
print(f"step total {tot:.1f} us")
