"""Counter calibration table from a tools/gpu_calib.sh run (tools/calib_bench.hip): for every kernel of
known access shape, what each rocprofv3 counter reports against the bytes and 128-B lines the kernel
actually touches.

    python tools/calib_summary.py gpurun_out/TAG > profiles/r06_counter_calibration.txt
    python tools/calib_summary.py gpurun_out/TAG --json profiles/r06_counter_calibration.json

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3's derived counters); the other counters are counts.
"fetch/useful" is FETCH_SIZE x 1024 over the useful bytes read; "fetch/lines" over 128 B per distinct
line touched. The multiplier a traffic figure needs for a shape is lines x 128 / FETCH_SIZE bytes.
"""
import csv
import glob
import json
import os
import sys


def counters(run_dir):
    """{kernel short name: {counter: mean value over its dispatches}}"""
    out = {}
    for path in glob.glob(os.path.join(run_dir, "pmc", "*", "run_counter_collection.csv")):
        acc = {}
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith("__amd"):
                continue
            acc.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            out.setdefault(k, {})[c] = sum(v) / len(v)
    return out


def main():
    run = sys.argv[1]
    shapes = {}
    for line in open(os.path.join(run, "calib.jsonl")):
        d = json.loads(line)
        if "error" not in d:
            shapes[d["kernel"]] = d
    ctr = counters(run)
    rows = []
    for k, d in shapes.items():
        c = ctr.get(k, {})
        wr = k.startswith("wr_") or k.startswith("at_")
        useful, lines = d["useful_bytes"], d["lines128"]
        f = c.get("FETCH_SIZE", float("nan")) * 1024
        w = c.get("WRITE_SIZE", float("nan")) * 1024
        row = {"kernel": k, "ms": d["ms"], "useful_bytes": useful, "lines128": lines,
               "FETCH_SIZE_bytes": f, "WRITE_SIZE_bytes": w,
               "RDREQ": c.get("TCC_EA0_RDREQ_sum"), "RDREQ_32B": c.get("TCC_EA0_RDREQ_32B_sum"),
               "WRREQ": c.get("TCC_EA0_WRREQ_sum"), "WRREQ_64B": c.get("TCC_EA0_WRREQ_64B_sum"),
               "TCC_HIT": c.get("TCC_HIT_sum"), "TCC_MISS": c.get("TCC_MISS_sum"),
               "UTCL1_MISS": c.get("TCP_UTCL1_TRANSLATION_MISS_sum"),
               "UTCL1_HIT": c.get("TCP_UTCL1_TRANSLATION_HIT_sum")}
        if wr:
            row["write_over_useful"] = w / useful
            row["write_over_lines128"] = w / (lines * 128)
        else:
            row["fetch_over_useful"] = f / useful
            row["fetch_over_lines128"] = f / (lines * 128)
            row["multiplier_to_lines128"] = lines * 128 / f if f else None
        rows.append(row)
    if "--json" in sys.argv:
        dst = sys.argv[sys.argv.index("--json") + 1]
        json.dump({"source": run, "kernels": rows}, open(dst, "w"), indent=1)
    hdr = ("kernel", "ms", "lines128", "FETCH/useful", "FETCH/lines", "WRITE/useful", "RDREQ/line", "WRREQ/line",
           "TCC hit%", "UTCL1 miss%")
    print("# counter calibration: known access shapes (tools/calib_bench.hip) under rocprofv3 --pmc, one pass per")
    print("# counter group; FETCH/lines = FETCH_SIZE bytes over 128 B per distinct line touched")
    print("%-24s %8s %10s %12s %11s %12s %10s %10s %8s %11s" % hdr)
    for r in rows:
        rd = r["RDREQ"] / r["lines128"] if r["RDREQ"] is not None else float("nan")
        wq = r["WRREQ"] / r["lines128"] if r["WRREQ"] is not None else float("nan")
        hit = (100 * r["TCC_HIT"] / (r["TCC_HIT"] + r["TCC_MISS"])
               if r["TCC_HIT"] is not None and (r["TCC_HIT"] + r["TCC_MISS"]) else float("nan"))
        um = (100 * r["UTCL1_MISS"] / (r["UTCL1_MISS"] + r["UTCL1_HIT"])
              if r["UTCL1_MISS"] is not None and (r["UTCL1_MISS"] + r["UTCL1_HIT"]) else float("nan"))
        print("%-24s %8.4f %10d %12.3f %11.3f %12.3f %10.3f %10.3f %8.1f %11.1f" % (
            r["kernel"], r["ms"], r["lines128"], r["FETCH_SIZE_bytes"] / r["useful_bytes"],
            r["FETCH_SIZE_bytes"] / (r["lines128"] * 128), r["WRITE_SIZE_bytes"] / r["useful_bytes"], rd, wq, hit, um))


if __name__ == "__main__":
    main()
