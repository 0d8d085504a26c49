"""The multi-core CPU baseline (oracle/hkv_oracle_bench.c): worker threads share one table under
the reference's seqlock (concur_ctrl.h:144-224) and lock-free reads (hermesKV.c:81-96), as the
reference's workers do (main.c:193-210). Runs here on the container's cores."""
import ctypes

import numpy as np
import pytest

from hermes_amd import layout as L
from oracle import oracle as O
from oracle.cpu_baseline import HkoZipf, host_threads


def _bench(kv, threads, workers, seconds, theta=0.99, write_pm=200, refill_flags=1):
    lib = O.lib()
    lib.hko_bench_rounds.restype = ctypes.c_int64
    lib.hko_bench_rounds.argtypes = [ctypes.c_void_p, ctypes.POINTER(O.Config), ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, ctypes.POINTER(HkoZipf), ctypes.c_uint32, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                     ctypes.POINTER(ctypes.c_double)]
    n = 20000
    zetan = float(np.sum(np.arange(1, n + 1, dtype=np.float64) ** -theta))
    zeta2 = 1.0 + 2.0 ** -theta
    z = HkoZipf(theta, zetan, 1.0 / (1.0 - theta), (1.0 - (2.0 / n) ** (1.0 - theta)) / (1.0 - zeta2 / zetan),
                1.0 + 0.5 ** theta, n)
    rounds, secs = ctypes.c_int64(0), ctypes.c_double(0.0)
    c = lib.hko_bench_rounds(kv.h, ctypes.byref(kv.cfg), workers, threads, seconds, ctypes.byref(z), write_pm, 2, 50,
                             0x5EED, refill_flags, ctypes.byref(rounds), ctypes.byref(secs))
    return c, rounds.value, secs.value


@pytest.mark.parametrize("threads", [1, 4])
def test_shared_table_threads_leave_consistent_state(threads):
    kv = O.OracleKVS(1 << 15, 1 << 21, machine_id=0)
    kv.populate(20000, L.DEFAULT.kvs_value)
    committed, rounds, secs = _bench(kv, threads, 2 * threads, 0.5)
    assert committed > 0 and rounds > 0 and secs > 0
    ents = kv.log_bytes()[: kv.log_head()].view(L.entry_dtype())
    assert (ents["lock"] == 0).all(), "a seqlock was left held"
    assert (ents["ts_ver"] % 2 == 0).all(), "odd (locked) version left behind"
    # every round ACKs and VALidates all writes it INV'd: no key is left mid-write
    assert np.isin(ents["state"], [int(L.State.VALID)]).mean() > 0.999


@pytest.mark.parametrize("refill_flags,skew", [(0, 0), (2, 3), (6, 3)])
def test_reference_refill_policies_leave_consistent_state(refill_flags, skew):
    """refill_ops' retry policy (stalled ops keep their slots), alone, with the skew optimisations
    (GET timestamps reset, read completion, write coalescing) and with hot-request coalescing: the
    shared table ends consistent and ops commit."""
    kv = O.OracleKVS(1 << 15, 1 << 21, machine_id=0, skew=skew)
    kv.populate(20000, L.DEFAULT.kvs_value)
    committed, rounds, secs = _bench(kv, 4, 8, 0.5, refill_flags=refill_flags)
    assert committed > 0 and rounds > 0 and secs > 0
    ents = kv.log_bytes()[: kv.log_head()].view(L.entry_dtype())
    assert (ents["lock"] == 0).all() and (ents["ts_ver"] % 2 == 0).all()
    assert np.isin(ents["state"], [int(L.State.VALID)]).mean() > 0.999


def test_host_threads_capped():
    assert 1 <= host_threads() <= 16
