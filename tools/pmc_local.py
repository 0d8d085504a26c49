"""HBM bytes per batch launch from a tools/pmc.sh run (FETCH_SIZE and WRITE_SIZE passes):
    python tools/pmc_local.py TAG OUT.json WORKERS KEYS REFILL SKEW

Per protocol round of bench.py (the dispatches from one k_local_pre to the next) the launches are
grouped the way bench.py times them:
* local: k_local_pre, k_local_fused, k_local_deferred and k_commit_w (the direct path);
* invs:  every INV launch of the round (one unique-key launch per virtual peer: k_unique_lds<2, ...>);
* acks:  the ACK launch (k_unique_rows<3, ...>, all peers' rows in one pass);
* vals:  the VAL launch (the one-pass k_lookup after the ACKs).
Counters are KB per dispatch; FETCH_SIZE is doubled. Calibrated on this access mix (tools/calib_bench.hip,
profiles/r06_counter_calibration.txt): every read shape the batch kernels use -- random 8-, 16-, 64- and
128-byte records and 16-byte streaming lanes -- costs one 128-byte memory request, which FETCH_SIZE counts
as 64 bytes (TCC_EA0_RDREQ = lines touched, RDREQ_32B = 0), and takes the same time per record whatever
its width; WRITE_SIZE is exact for 64- and 128-byte writes and counts smaller ones as 32-byte granules. The median over the run's rounds is written to OUT.json,
stamped with the bench configuration (bench.py reports it only for that configuration) as
roofline.traffic and roofline.launches.*.traffic."""
import csv
import json
import statistics
import sys

KIND_PATTERNS = {
    "local": ("k_local_pre", "k_local_fused", "k_local_deferred", "k_commit_w"),
    "invs": ("k_unique_lds<2,", "k_unique_rows<2,", "k_unique<2,"),
    "acks": ("k_unique_lds<3,", "k_unique_rows<3,", "k_unique<3,"),
    "vals": ("k_lookup<",),
}


def dispatches(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        rows[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
    return rows


def per_round(rows, scale):
    """{kind: [bytes per round]} over complete rounds"""
    ids = sorted(rows)
    starts = [k for k, d in enumerate(ids) if "k_local_pre" in rows[d][0]]
    out = {k: [] for k in KIND_PATTERNS}
    for s, e in zip(starts, starts[1:]):
        acc = {k: 0.0 for k in KIND_PATTERNS}
        seen = {k: 0 for k in KIND_PATTERNS}
        acks_done = False
        for d in ids[s:e]:
            name = rows[d][0]
            for kind, pats in KIND_PATTERNS.items():
                if kind == "vals" and not acks_done:
                    continue
                if any(p in name for p in pats):
                    acc[kind] += scale * rows[d][1]
                    seen[kind] += 1
                    if kind == "acks":
                        acks_done = True
                    break
        if seen["local"] == 4 and all(seen[k] for k in KIND_PATTERNS):
            for k in KIND_PATTERNS:
                out[k].append(acc[k])
    return out


def main():
    tag, dst = sys.argv[1], sys.argv[2]
    f = per_round(dispatches(f"gpurun_out/{tag}/pmc/FETCH_SIZE/run_counter_collection.csv"), 2.0)
    w = per_round(dispatches(f"gpurun_out/{tag}/pmc/WRITE_SIZE/run_counter_collection.csv"), 1.0)
    launches = {}
    for k in KIND_PATTERNS:
        fb, wb = statistics.median(f[k]), statistics.median(w[k])
        launches[k] = {"kernels": list(KIND_PATTERNS[k]), "fetch_bytes": fb, "write_bytes": wb,
                       "traffic_bytes": fb + wb}
    res = {
        "what": "HBM bytes per batch launch of one bench round (median over rounds): local = k_local_pre + "
                "k_local_fused + k_local_deferred + k_commit_w; invs = the round's INV launches; acks = the ACK "
                "rows launch; vals = the VAL lookup. rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE in "
                "separate passes of bench.py",
        "source": f"gpurun_out/{tag}/pmc",
        "launches_counted": min(len(f["local"]), len(w["local"])),
        "fetch_bytes": launches["local"]["fetch_bytes"],
        "write_bytes": launches["local"]["write_bytes"],
        "traffic_bytes": launches["local"]["traffic_bytes"],
        "launches": launches,
        # the bench configuration the counters belong to (bench.py checks it)
        "config": {"workers": int(sys.argv[3]), "keys": int(sys.argv[4]), "refill": sys.argv[5],
                   "skew": int(sys.argv[6])},
    }
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
