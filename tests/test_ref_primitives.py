"""Pins the oracle's seqlock, Lamport-timestamp and ack-quorum restatements (hkv_oracle.c) and the
device's folded arithmetic (hkv_exec.h, layout.py) against the reference's OWN primitives:
include/utils/concur_ctrl.h and include/utils/bit_vector.h, compiled unmodified from where they lie
into oracle/_ref/libhkv_refprims.so (oracle/Makefile, oracle/ref_prims.c). Skipped where the
reference is absent (the GPU box); the committed oracle it pins is what travels there.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from hermes_amd import layout as L
from oracle import oracle as O

REF = os.path.join(os.path.dirname(O.__file__), "_ref", "libhkv_refprims.so")
U8P = ctypes.POINTER(ctypes.c_uint8)


@pytest.fixture(scope="module")
def libs():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libhkv_refprims.so not built (no /root/reference here)")
    r = ctypes.CDLL(REF)
    o = O.lib()
    for f in (r.hkr_cctrl_lock_unlock, o.hko_test_cctrl_lock_unlock):
        f.restype = ctypes.c_uint32
        f.argtypes = [U8P, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint32]
    for f in (r.hkr_ts_equal, r.hkr_ts_smaller, o.hko_test_ts_less, o.hko_test_ts_equal):
        f.argtypes = [ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint8]
    r.hkr_is_last_ack.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
    o.hko_test_is_last_ack.argtypes = [ctypes.c_uint8, U8P]
    o.hko_test_has_node.argtypes = [U8P, ctypes.c_uint8]
    r.hkr_membership_init.argtypes = [ctypes.c_int, ctypes.c_uint8, U8P]
    r.hkr_membership_update.argtypes = [ctypes.c_uint8, ctypes.c_uint8, U8P]
    r.hkr_bv_bit_get.argtypes = [ctypes.c_uint8, ctypes.c_int]
    r.hkr_cctrl_same_and_valid.argtypes = [U8P, U8P]
    return r, o


def _cc(lock, cid, ver):
    b = (ctypes.c_uint8 * 6)()
    b[0], b[1] = lock, cid
    for k in range(4):
        b[2 + k] = (ver >> (8 * k)) & 0xFF
    return b


def test_layout_sizes(libs):
    r, _ = libs
    assert r.hkr_conc_ctrl_size() == 6 and r.hkr_timestamp_size() == 5   # spacetime_object_meta offsets 4..9


def test_bv_unit_test_runs_clean():
    """bit_vector.h:508-552 (with dbv_unit_test :341-384): defined, never called by the reference.
    Runs in a child process because a failing reference assert aborts."""
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref not built")
    code = f"import ctypes; ctypes.CDLL({REF!r}).hkr_bv_unit_test()"
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert "Static  Bit Vector Unit Test was Successful" in p.stdout


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_cctrl_lock_unlock_matches_reference(libs, variant):
    """cctrl_lock + each unlock variant (concur_ctrl.h:144-213) vs the oracle's cc_* restatement,
    from random unlocked states (even versions: the batch-boundary invariant the reference's lock
    asserts check), including versions next to 2^32."""
    r, o = libs
    rng = np.random.default_rng(7 + variant)
    vers = np.concatenate([rng.integers(0, 2**31, size=3000) * 2, [0, 2, 0xFFFFFFFE, 0xFFFFFFFC, 0xFFFFFFFA]])
    for v in vers:
        v = int(v)
        cid0, cid, cv = (int(x) for x in rng.integers(0, 256, size=3))
        newv = int(rng.integers(0, 2**32))
        a, b = _cc(0, cid0, v), _cc(0, cid0, v)
        ra = r.hkr_cctrl_lock_unlock(a, variant, cid, newv)
        rb = o.hko_test_cctrl_lock_unlock(b, variant, cid, newv)
        assert bytes(a) == bytes(b) and ra == rb, (variant, v, cid0, cid, newv, bytes(a), bytes(b))
        # the device folds lock+unlock into one step (hkv_exec.h): +0, +2, +4, or the custom ts
        got = int.from_bytes(bytes(a)[2:6], "little")
        want = {0: v, 1: (v + 2) & 0xFFFFFFFF, 2: (v + 4) & 0xFFFFFFFF, 3: newv}[variant]
        assert got == want and a[0] == 0
        assert a[1] == (cid0 if variant == 0 else cid)
        del cv


def test_timestamp_order_matches_reference(libs):
    """timestamp_is_smaller / timestamp_is_equal (concur_ctrl.h:63-75) vs the oracle, and vs the
    device's packed ts64 = version << 8 | cid compared as one u64 (hkv_exec.h pack_ts)."""
    r, o = libs
    rng = np.random.default_rng(3)
    n = 20000
    v1 = rng.integers(0, 6, size=n).astype(np.uint64)
    v1[::3] = rng.integers(0, 2**32, size=len(v1[::3]), dtype=np.uint64)
    v2 = np.where(rng.random(n) < 0.5, v1, rng.integers(0, 6, size=n).astype(np.uint64))
    c1 = rng.integers(0, 256, size=n).astype(np.uint64)
    c2 = np.where(rng.random(n) < 0.3, c1, rng.integers(0, 256, size=n).astype(np.uint64))
    p1, p2 = L.ts64(v1, c1), L.ts64(v2, c2)
    for i in range(n):
        a = (int(v1[i]), int(c1[i]), int(v2[i]), int(c2[i]))
        s, e = r.hkr_ts_smaller(*a), r.hkr_ts_equal(*a)
        assert s == o.hko_test_ts_less(*a) and e == o.hko_test_ts_equal(*a), a
        assert bool(s) == bool(p1[i] < p2[i]) and bool(e) == bool(p1[i] == p2[i]), a


def test_is_last_ack_matches_reference(libs):
    """is_last_ack (spacetime.h:253-259: bv_and + bv_are_equal) over every 8-bit ack vector and
    membership, vs the oracle and the device's (bv & g) == g."""
    r, o = libs
    mb = (ctypes.c_uint8 * 8)()
    for g in range(256):
        mb[1] = g
        for bv in range(256):
            ref = r.hkr_is_last_ack(bv, g)
            assert ref == o.hko_test_is_last_ack(bv, mb) == int((bv & g) == g), (bv, g)
        for node in range(8):
            assert o.hko_test_has_node(mb, node) == r.hkr_bv_bit_get(g, node)


def test_membership_vectors_match_reference(libs):
    """layout.membership() -- the spacetime_group_membership every batch gets by value -- vs the
    reference's bit-vector steps of group_membership_init (main.c:37-49) and
    group_membership_update (inline-util.h:26-43)."""
    r, _ = libs
    out = (ctypes.c_uint8 * 3)()
    for n in range(1, 9):
        for mid in range(n):
            r.hkr_membership_init(n, mid, out)
            m = L.membership(n, mid)
            assert (m[1], m[2], m[0]) == (out[0], out[1], n - 1), (n, mid)
    for g in range(256):
        for mid in range(8):
            r.hkr_membership_update(g, mid, out)
            m = L.membership(0, mid, alive=g)
            assert (m[1], m[2], m[0]) == (out[0], out[1], out[2]), (g, mid)


def test_lock_free_read_validation(libs):
    """cctrl_timestamp_is_same_and_valid (concur_ctrl.h:217-224), the check of the reference's
    lock-free meta snapshot (hermesKV.c:81-96): valid only for equal, even-version timestamps.
    The device and the oracle read a meta only at batch boundaries, where versions are even."""
    r, _ = libs
    rng = np.random.default_rng(11)
    for _ in range(3000):
        v, c = int(rng.integers(0, 2**32)), int(rng.integers(0, 256))
        v2 = v if rng.random() < 0.6 else int(rng.integers(0, 2**32))
        c2 = c if rng.random() < 0.6 else int(rng.integers(0, 256))
        got = r.hkr_cctrl_same_and_valid(_cc(0, c, v), _cc(0, c2, v2))
        assert got == int(v % 2 == 0 and v == v2 and c == c2)
