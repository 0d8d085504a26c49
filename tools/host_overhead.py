"""Host time to enqueue one N=1 round (no GPU wait inside): the GPU is held busy by a sleep kernel
while the host enqueues steps, so the time measured is the host's alone.
    python tools/host_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from hermes_amd import layout as L
from hermes_amd.kvs import HermesKV, sized_geometry
from hermes_amd.workload import Round, zipf_params

n_keys = 1_000_000
bkts, cap = sized_geometry(n_keys)
g = HermesKV(n_keys, bkts, cap, machine_id=0)
r = Round(g, 8192, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 200, seed=1, max_steps=16,
          fit_ack_stride=False)
r.count_elems = False
for _ in range(3):
    r.step()
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda._sleep(2_000_000_000)      # hold the GPU (about a second) while the host enqueues
    t0 = time.perf_counter()
    for _ in range(8):
        r.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host enqueue: {(t1 - t0) / 8 * 1e6:.1f} us per round")
t0 = time.perf_counter()
for _ in range(20):
    r.step()
torch.cuda.synchronize()
print(f"wall: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us per round")
