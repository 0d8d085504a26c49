"""HBM bytes per local batch launch from a tools/pmc.sh run (FETCH_SIZE and WRITE_SIZE passes):
    python tools/pmc_local.py TAG OUT.json [WORKERS KEYS REFILL SKEW]

A local launch is k_local_pre, k_local_fused, k_local_deferred and the k_commit after them (the
direct path), or, on the rounds engine, the two k_lookup dispatches before a k_resolve0<0, ...>
dispatch, that dispatch and the k_commit after it. Counters are KB per dispatch; FETCH_SIZE is doubled (on gfx950 it
reports half the bytes of wide reads, MI355X_MICROARCH.md, HBM section). The median over the
launches of the run is written to OUT.json, which bench.py reports as roofline.traffic."""
import csv
import json
import statistics
import sys


def dispatches(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        rows[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
    return rows


def local_launches(rows):
    ids = sorted(rows)
    out = []
    for k, d in enumerate(ids):
        if "k_local_pre" in rows[d][0] and k + 3 < len(ids):
            grp = ids[k:k + 4]
            names = [rows[g][0] for g in grp]
            if "k_local_fused" in names[1] and "k_local_deferred" in names[2] and "k_commit" in names[3]:
                out.append(grp)
            continue
        if "k_resolve0<0," not in rows[d][0]:
            continue
        grp = [ids[k - 2], ids[k - 1], d, ids[k + 1]]
        names = [rows[g][0] for g in grp]
        if "k_lookup" in names[0] and "k_lookup" in names[1] and "k_commit" in names[3]:
            out.append(grp)
    return out


def main():
    tag, dst = sys.argv[1], sys.argv[2]
    f = dispatches(f"gpurun_out/{tag}/pmc/FETCH_SIZE/run_counter_collection.csv")
    w = dispatches(f"gpurun_out/{tag}/pmc/WRITE_SIZE/run_counter_collection.csv")
    fl = [sum(2.0 * f[g][1] for g in grp) for grp in local_launches(f)]
    wl = [sum(w[g][1] for g in grp) for grp in local_launches(w)]
    res = {
        "what": "HBM bytes per local batch launch (k_local_pre, k_local_fused, k_local_deferred, k_commit; "
                "or k_lookup x2, k_resolve0, k_commit), rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE "
                "in separate passes of bench.py",
        "launches": len(fl),
        "fetch_bytes": statistics.median(fl),
        "write_bytes": statistics.median(wl),
    }
    res["traffic_bytes"] = res["fetch_bytes"] + res["write_bytes"]
    if len(sys.argv) > 6:   # the bench configuration the counters belong to (bench.py checks it)
        res["config"] = {"workers": int(sys.argv[3]), "keys": int(sys.argv[4]), "refill": sys.argv[5],
                         "skew": int(sys.argv[6])}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
