"""Summarise a bench.py JSON line (tools/benchsum.py FILE)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "error" in d:
        print(d["error"])
        d = d["partial"]
    print(f"value {d['value'] / 1e9:.3f} G {d['unit']}  ms/step {d['ms_per_step']:.3f}  refill {d['config'].get('refill')}")
    r = d["roofline"]
    for k, v in r.get("launches", {}).items():
        print(f"  {k:6s} {v['elements']:>10.0f} el  {v['ms'] * 1e3:7.1f} us  {v['achieved']:7.0f} GB/s  frac {v['frac']:.3f}")
    if "step" in r:
        print(f"  step frac {r['step']['frac']:.3f}")
    det = d["detail"]
    print("  detail:", {k: v for k, v in det.items() if k not in ("round_stats_rank0", "host_api", "retry")})
    print("  stats:", det.get("round_stats_rank0"))
    if "retry" in det:
        print(f"  retry {det['retry']['value'] / 1e6:.1f} M/s")
    if "host_api" in det:
        h = det["host_api"]
        print("  host_api", {k: round(v / 1e6, 2) for k, v in h.items() if k.startswith("threads_")}, "M local ops/s")
    if "cpu_baseline" in d:
        c = d["cpu_baseline"]
        print(f"  cpu {c['value'] / 1e6:.2f} M/s cores {c['cores']} kind {c['kind']}")
