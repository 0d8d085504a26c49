"""CPU baseline scaling probe (oracle/hkv_oracle_bench.c) on this host: refill policy x thread
count on a populated oracle table (no GPU).   python tools/cpu_threads.py [keys] [seconds]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hermes_amd import layout as L  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.cpu_baseline import HkoZipf, host_threads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
theta = 0.99
zetan = float(np.sum(np.arange(1, n + 1, dtype=np.float64) ** -theta))
zeta2 = 1.0 + 2.0 ** -theta
z = HkoZipf(theta, zetan, 1.0 / (1.0 - theta), (1.0 - (2.0 / n) ** (1.0 - theta)) / (1.0 - zeta2 / zetan),
            1.0 + 0.5 ** theta, n)
lib = O.lib()
lib.hko_bench_rounds.restype = ctypes.c_int64
lib.hko_bench_rounds.argtypes = [ctypes.c_void_p, ctypes.POINTER(O.Config), ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                 ctypes.POINTER(HkoZipf), ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]
bk = 1 << max(4, (2 * n - 1).bit_length())
cap = 1 << (n * 64 + 4096).bit_length()
print(f"host_threads() = {host_threads()}, affinity {len(os.sched_getaffinity(0))}, keys {n}", flush=True)
for flags, skew in ((1, 0), (2, 3)):
    kv = O.OracleKVS(bk, cap, machine_id=0, skew=skew)
    kv.populate(n, L.DEFAULT.kvs_value)
    for t in (1, 4, 8, 16):
        r, s = ctypes.c_int64(0), ctypes.c_double(0)
        c = lib.hko_bench_rounds(kv.h, ctypes.byref(kv.cfg), t, t, secs, ctypes.byref(z), 200, 2, 50, 0x5EED, flags,
                                 ctypes.byref(r), ctypes.byref(s))
        print(f"refill flags {flags} skew {skew} threads {t:2d}: {c / s.value / 1e6:8.2f} M ops/s, "
              f"slowest thread {r.value} rounds", flush=True)
    del kv
