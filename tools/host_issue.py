"""How close the one-GPU bench round is to host-bound (diagnostics, not the bench): per step of the
default configs[1] round, the host's wall time in Round.step, the part of it spent waiting in the
step's one host synchronisation (the ACK layout read-back), and the GPU time of the step (events).
Host busy = step wall - wait; when host busy approaches the GPU step time, GPU savings stop
showing in the step.

  python tools/host_issue.py --steps 40 > gpurun_out/host_issue.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workers", type=int, default=16384)
    p.add_argument("--keys", type=int, default=100_000_000)
    a = p.parse_args()
    import torch
    from hermes_amd import layout as L
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params

    bkts, cap = sized_geometry(a.keys, L.DEFAULT)
    kvs = HermesKV(a.keys, bkts, cap, machine_id=0, skew=3)
    z = zipf_params(a.keys, 0.99)
    r = Round(kvs, a.workers, L.membership(3, 0), [1, 2], z, 200, 0, seed=0x5EED,
              max_steps=a.steps + a.warmup + 4, retry_stalled=True)
    for _ in range(a.warmup):
        r.step()
    torch.cuda.synchronize()
    waits = []
    ev = r.maxc_ev
    orig = ev.synchronize

    class Timed:
        def record(self, *x):
            ev.record(*x)

        def synchronize(self):
            t0 = time.perf_counter()
            orig()
            waits.append(time.perf_counter() - t0)

        def __getattr__(self, k):
            return getattr(ev, k)

    r.maxc_ev = Timed()
    walls, gpu = [], []
    for _ in range(a.steps):
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b0.record()
        t0 = time.perf_counter()
        r.step()
        walls.append(time.perf_counter() - t0)
        b1.record()
        gpu.append((b0, b1))
    torch.cuda.synchronize()
    g = [x.elapsed_time(y) * 1e3 for x, y in gpu]
    w = [x * 1e6 for x in walls]
    wt = [x * 1e6 for x in waits[-a.steps:]] if waits else [0.0] * a.steps
    busy = [x - y for x, y in zip(w, wt)]
    med = lambda v: sorted(v)[len(v) // 2]
    print(json.dumps({"steps": a.steps, "host_wall_us_median": med(w), "host_wait_us_median": med(wt),
                      "host_busy_us_median": med(busy), "host_busy_us_max": max(busy),
                      "gpu_step_us_median": med(g), "syncs_per_step": len(waits) / (a.steps + 0.0)}))
    assert kvs.take_error_flags() == 0


if __name__ == "__main__":
    main()
