"""bench.py's cpu_baseline leg -- TEST INFRASTRUCTURE ONLY.

Times the oracle (the CPU restatement of the reference batch path, hkv_oracle.c) on the GPU
host's own cores -- one worker thread per core over one shared table, as the reference runs --
on a bounded sample of the same workload (see hkv_oracle_bench.c). The table image is copied out of HBM so the CPU starts from the same
state the device produced (the two populates are bit-identical, tests/test_gpu_parity.py).
"""
from __future__ import annotations

import ctypes
import os

from .oracle import Config, build, lib


class HkoZipf(ctypes.Structure):
    _fields_ = [("theta", ctypes.c_double), ("zetan", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eta", ctypes.c_double), ("half_pow", ctypes.c_double), ("n", ctypes.c_uint64)]


def host_threads(cap: int = 16) -> int:
    """Cores this process may use: its affinity set, capped by OMP_NUM_THREADS (16 on the GPU
    box, which shows the whole machine's CPUs) and `cap`."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        n = min(n, omp)
    return max(1, min(n, cap))


def host_cores() -> dict:
    """The host's cores beside the ones the baseline may use: the machine's CPUs, this process's
    affinity set, and the usable count (host_threads: capped by OMP_NUM_THREADS, 16 on the GPU box)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"host_cpus": os.cpu_count(), "host_affinity_cpus": aff, "host_usable_threads": host_threads()}


class TableSnapshot:
    """The device table's image (index and log) copied into an oracle table, taken before the GPU
    rounds change it, so the CPU baseline can run after the GPU's timed region (nothing of it then
    competes with the GPU run's host thread)."""

    def __init__(self, kvs, skew: int | None = None):
        """skew: the oracle table's skew flags (default: the device table's)"""
        build()
        self.L = L = lib()
        L.hko_set_log_head.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        c = kvs.cfg
        self.c = c
        self.cfg = Config(c.big_objects, c.extra_cache_lines, c.rmw_enabled, c.machine_id, c.num_bkts, c.log_cap,
                          c.skew_flags if skew is None else int(skew), 0)
        self.h = L.hko_create(ctypes.byref(self.cfg))
        from hermes_amd.lib import check, raw
        R = raw()
        idx = ctypes.cast(L.hko_index(self.h), ctypes.c_void_p)
        log = ctypes.cast(L.hko_log(self.h), ctypes.c_void_p)
        check(R.hkv_copy_index(kvs.h, idx, 0, c.num_bkts * 64), "copy index")
        check(R.hkv_copy_log(kvs.h, log, 0, min(kvs.log_head, c.log_cap)), "copy log")
        L.hko_set_log_head(self.h, kvs.log_head)

    def close(self):
        if self.h:
            self.L.hko_destroy(self.h)
            self.h = None


def run_cpu_baseline(kvs, zipf, write_permille: int, workers: int, seconds: float, seed: int,
                     n_peers: int = 2, per_peer: int = 50, refill_flags: int = 1, threads: int = 0,
                     snapshot: TableSnapshot | None = None) -> dict:
    """threads = 0: the thread count among 1, 4, 8, ... host_threads() that runs this workload fastest,
    by a short probe of each (the reference's seqlocks make hot keys contended, and under refill_ops'
    retry more threads can be slower); workers = 0: one 250-op buffer per thread, as the reference's
    workers (main.c:193-210). refill_flags: hkv_wl_refill's (1 fresh batches, 2 GET timestamps
    reset, 4 hot-request coalescing; 0 = refill_ops' retry). The table's skew flags come with it.
    snapshot: a TableSnapshot taken earlier (consumed); default: the table as it is now."""
    snap = snapshot if snapshot is not None else TableSnapshot(kvs)
    L, h, cfg = snap.L, snap.h, snap.cfg
    L.hko_bench_rounds.restype = ctypes.c_int64
    L.hko_bench_rounds.argtypes = [ctypes.c_void_p, ctypes.POINTER(Config), ctypes.c_int, ctypes.c_int,
                                   ctypes.c_double, ctypes.POINTER(HkoZipf), ctypes.c_uint32, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(ctypes.c_double)]
    probe = {}
    try:
        hz = HkoZipf(zipf.theta, zipf.zetan, zipf.alpha, zipf.eta, zipf.half_pow, zipf.n)
        rounds, secs = ctypes.c_int64(0), ctypes.c_double(0.0)

        def run(t, w, s):
            return L.hko_bench_rounds(h, ctypes.byref(cfg), w, t, s, ctypes.byref(hz), write_permille, n_peers,
                                      per_peer, seed, int(refill_flags), ctypes.byref(rounds), ctypes.byref(secs))
        if not threads:
            top = host_threads()
            for t in sorted({1, 4, 8, top} & set(range(1, top + 1))):
                probe[t] = run(t, workers or t, min(1.5, seconds / 8)) / secs.value
            threads = max(probe, key=probe.get)
        workers = workers or threads
        committed = run(threads, workers, seconds)
    finally:
        snap.close()
    return {"value": committed / secs.value, "unit": "ops/s", "cores": threads, "kind": "port",
            "probe_ops_per_s_by_threads": probe,
            "sample": (f"{threads} worker threads sharing one table (per-key seqlocks, concur_ctrl.h:144-224), "
                       f"{workers} x 250-op {'fresh' if refill_flags & 1 else 'retried (refill_ops)'} local batches "
                       f"per round, refill flags {refill_flags}, skew flags {cfg.skew_flags}, "
                       f">= {rounds.value} rounds each in {secs.value:.1f} s; +{n_peers} virtual peers (one write per "
                       f"key and round each, live timestamps, up to {per_peer} per worker-round), 2 ACKs per write; "
                       f"same table ({cfg.num_bkts} buckets, copied from HBM) and Zipf/write mix as the GPU run")}
