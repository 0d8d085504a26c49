"""The drop-in boundary as the reference's worker uses it, from gcc-built C callers
(tools/capi_*.c, built by __graft_entry__.build):

* tools/capi_known_answers: the SURVEY section 4 known-answer scenario through spacetime_init +
  hermes_batch_ops_to_KVS (the by-value membership ABI of a gcc caller).
* tools/capi_threads shared: batches of several types on shared keys, combined into one launch
  in a known order and replayed on the oracle in that order.
* tools/capi_threads: 8 worker threads calling hermes_batch_ops_to_KVS concurrently on one table
  (main.c:193-210), their batches combined into shared launches by the library. Threads use
  disjoint keys, so any interleaving gives every key the same history: each thread's recorded
  calls (inputs, outputs, read_write_ops) are replayed one after another on the oracle and must
  match byte for byte.
"""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402
from oracle.oracle import OracleKVS, gen_keys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu_and_tools():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for t in ("capi_known_answers", "capi_threads"):
        if not os.path.exists(os.path.join(TOOLS, t)):
            pytest.fail(f"tools/{t} was not built (run __graft_entry__.build())")


def test_gcc_caller_known_answers():
    keys = gen_keys(7)
    p = subprocess.run([os.path.join(TOOLS, "capi_known_answers"), str(int(keys[5])), str(int(keys[6]))],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "C-ABI known answers: OK" in p.stdout


def _read_calls(path):
    raw = open(path, "rb").read()
    off, calls = 0, []
    while off < len(raw):
        t, n, esz = np.frombuffer(raw, np.int32, 3, off)
        off += 12
        ein = np.frombuffer(raw, np.uint8, n * esz, off).copy()
        off += n * esz
        eout = np.frombuffer(raw, np.uint8, n * esz, off).copy()
        off += n * esz
        has_rw = int(np.frombuffer(raw, np.int32, 1, off)[0])
        off += 4
        rin = rout = None
        if has_rw:
            rin = np.frombuffer(raw, np.uint8, 250 * 56, off).copy()
            off += 250 * 56
            rout = np.frombuffer(raw, np.uint8, 250 * 56, off).copy()
            off += 250 * 56
        calls.append((int(t), int(n), int(esz), ein, eout, rin, rout))
    return calls


# the host boundary's switches (hkv_runtime.hip), each a different serving path or limit for the same results:
# the default (serving kernel over BAR-staged batches, partitioned launches), one launch per serving pass
# (HKV_HOST_SERVE=0), batches staged in pinned host memory (HKV_STAGE_VRAM=0), launches not partitioned by
# key (HKV_HOST_PART=0), and one launch in flight taking one published launch per pass
SWITCHES = [{}, {"HKV_HOST_SERVE": "0"}, {"HKV_STAGE_VRAM": "0"}, {"HKV_HOST_PART": "0"},
            {"HKV_SERVE_MERGE": "1", "HKV_PART_INFLIGHT": "1", "HKV_SERVE_IDLE_MS": "0.5"}]


@pytest.mark.parametrize("env", SWITCHES, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_concurrent_callers_match_oracle(tmp_path, env):
    threads, rounds = 8, 30
    p = subprocess.run([os.path.join(TOOLS, "capi_threads"), "trace", str(threads), str(rounds), str(tmp_path)],
                       capture_output=True, text=True, timeout=240, env=dict(os.environ, **env))
    assert p.returncode == 0, p.stdout + p.stderr
    o = OracleKVS(1 << 21, 1 << 30, machine_id=0)
    o.populate(1_000_000, L.DEFAULT.kvs_value)
    mb = L.membership(3, 0)
    n_put = 0
    for k in range(threads):
        calls = _read_calls(os.path.join(tmp_path, f"thread{k}.bin"))
        assert len(calls) >= rounds
        for c, (t, n, esz, ein, eout, rin, rout) in enumerate(calls):
            e = ein.view(np.dtype((np.void, esz))).copy()
            rw = rin.view(np.dtype((np.void, 56))).copy() if rin is not None else None
            o.batch(t, e, mb, rw=rw)
            assert np.array_equal(e.view(np.uint8), eout), f"thread {k} call {c} (type {t}): elements differ"
            if rw is not None:
                assert np.array_equal(rw.view(np.uint8), rout), f"thread {k} call {c}: read_write_ops differ"
            if t == int(L.BatchType.local_ops):
                n_put += int((eout.reshape(n, esz)[:, 9] == int(L.Resp.PUT_SUCCESS)).sum())
    assert n_put > 0


def test_mixed_batches_on_shared_keys_match_oracle(tmp_path):
    """Five gcc-built threads on 32 shared keys, their batches of four types combined into one
    launch per round in thread order (hkv_debug_host_hold): local ops, INVs, the ACKs of the
    previous round's writes (with read_write_ops), VALs, local ops. So one single-workgroup launch
    applies an INV, a local PUT and an ACK completing an earlier write to the same key, each
    batch under its own header (membership, read_write_ops). Replayed on the oracle round by
    round in thread order, every call's elements and read_write_ops must match byte for byte."""
    rounds = 20
    p = subprocess.run([os.path.join(TOOLS, "capi_threads"), "shared", str(rounds), str(tmp_path)],
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    o = OracleKVS(1 << 21, 1 << 30, machine_id=0)
    o.populate(1_000_000, L.DEFAULT.kvs_value)
    mb = L.membership(3, 0)
    calls = [_read_calls(os.path.join(tmp_path, f"thread{k}.bin")) for k in range(5)]
    assert all(len(c) == rounds for c in calls)
    seen = set()
    for r in range(rounds):
        for k in range(5):
            t, n, esz, ein, eout, rin, rout = calls[k][r]
            e = ein.view(np.dtype((np.void, esz))).copy()
            rw = rin.view(np.dtype((np.void, 56))).copy() if rin is not None else None
            o.batch(t, e, mb, rw=rw)
            assert np.array_equal(e.view(np.uint8), eout), f"round {r} thread {k} (type {t}): elements differ"
            if rw is not None:
                assert np.array_equal(rw.view(np.uint8), rout), f"round {r} thread {k}: read_write_ops differ"
            out = eout.reshape(n, esz)
            seen.update((t, int(c)) for c in out[:, 9 if t == int(L.BatchType.local_ops) else 8])
    # the mix did what it is for: writes completed by ACKs in the same launch as new local ops, INVs
    # that raised keys written locally, VALs that validated them
    assert (int(L.BatchType.acks), int(L.Resp.LAST_ACK_SUCCESS)) in seen, sorted(seen)
    assert (int(L.BatchType.local_ops), int(L.Resp.PUT_SUCCESS)) in seen
    assert (int(L.BatchType.local_ops), int(L.Resp.GET_STALL)) in seen
    assert (int(L.BatchType.invs), int(L.Resp.INV_SUCCESS)) in seen


def test_concurrent_callers_throughput():
    p = subprocess.run([os.path.join(TOOLS, "capi_threads"), "throughput", "8", "1.0", "50"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    print(d)
    assert d["threads"] == 8 and d["local_ops_per_s"] > 0
