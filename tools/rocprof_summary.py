"""Summarise a rocprofv3 kernel trace (.db from --kernel-trace, or kernel_stats.csv) per kernel.

    python tools/rocprof_summary.py gpurun_out/prof1/run_results.db [--top 25]
"""
import argparse
import csv
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    view = [r[0] for r in cur.execute("select name from sqlite_master where name='kernels'")]
    if view:
        q = "select name, end - start from kernels"
    else:
        q = ("select s.string, d.end - d.start from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol k on d.kernel_id = k.id join rocpd_string s on k.display_name = s.id")
    stats = {}
    for name, dur in cur.execute(q):
        s = stats.setdefault(name, [0, 0.0, float("inf"), 0.0])
        s[0] += 1
        s[1] += dur
        s[2] = min(s[2], dur)
        s[3] = max(s[3], dur)
    return stats


def from_csv(path):
    stats = {}
    for r in csv.DictReader(open(path)):
        stats[r["Name"]] = [int(r["Calls"]), float(r["TotalDurationNs"]), float(r["MinNs"]), float(r["MaxNs"])]
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    stats = from_db(a.path) if a.path.endswith(".db") else from_csv(a.path)
    tot = sum(v[1] for v in stats.values())
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}")
    for name, (n, t, mn, mx) in sorted(stats.items(), key=lambda kv: -kv[1][1])[: a.top]:
        short = name if len(name) <= 70 else name[:67] + "..."
        print(f"{short:70s} {n:6d} {t/1e6:10.3f} {t/n/1e3:10.2f} {mn/1e3:9.2f} {mx/1e3:9.2f} {100*t/tot:6.1f}")
    print(f"total kernel time {tot/1e6:.3f} ms", file=sys.stderr)


if __name__ == "__main__":
    main()
