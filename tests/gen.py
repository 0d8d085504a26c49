"""Seeded random batch generators for parity tests (device path vs oracle).

They deliberately pile many elements onto few keys, mix protocol-plausible timestamps
(versions the table actually holds, +2, equal with another cid) with random ones, and
include the elements the reference skips, so every branch of hermesKV.c:251-703 is hit.
"""
from __future__ import annotations

import numpy as np

from hermes_amd import layout as L


def bytecopy(a: np.ndarray) -> np.ndarray:
    """Copy including padding bytes (numpy's structured copy leaves holes uninitialised)."""
    b = np.empty_like(a)
    b.view(np.uint8)[...] = a.view(np.uint8)
    return b


class TsPool:
    """Timestamps seen recently (writes, INVs) so ACKs/VALs/INVs can match on purpose."""

    def __init__(self, rng):
        self.rng = rng
        self.items = [(0, 255), (2, 0), (2, 1), (2, 2)]

    def add(self, ver, cid):
        self.items.append((int(ver), int(cid)))
        if len(self.items) > 4000:
            self.items = self.items[-2000:]

    def pick(self, n):
        idx = self.rng.integers(0, len(self.items), size=n)
        return np.array([self.items[i][0] for i in idx], dtype=np.uint32), \
            np.array([self.items[i][1] for i in idx], dtype=np.uint8)


def key_pool(rng, all_keys: np.ndarray, hot: int, n_missing: int = 4) -> np.ndarray:
    ids = rng.choice(len(all_keys), size=min(hot, len(all_keys)), replace=False)
    missing = rng.integers(1, 2**63, size=n_missing, dtype=np.int64).astype(np.uint64)
    return np.concatenate([all_keys[ids], missing])


def draw_keys(rng, pool: np.ndarray, n: int) -> np.ndarray:
    # skewed: a few keys take most elements
    w = 1.0 / (np.arange(1, len(pool) + 1) ** 0.9)
    w /= w.sum()
    return pool[rng.choice(len(pool), size=n, p=w)]


def local_ops(rng, pool, n, sizes: L.Sizes, rmw: bool, tsp: TsPool) -> np.ndarray:
    a = np.zeros(n, dtype=L.op_dtype(sizes))
    a["key"] = draw_keys(rng, pool, n)
    codes = [int(L.Op.GET), int(L.Op.PUT)] + ([int(L.Op.RMW)] if rmw else [])
    probs = [0.5, 0.5] if not rmw else [0.45, 0.35, 0.2]
    a["opcode"] = rng.choice(codes, size=n, p=probs)
    st = rng.choice([int(L.Bucket.NEW), int(L.Resp.GET_STALL), int(L.Resp.PUT_STALL), int(L.Resp.PUT_SUCCESS),
                     int(L.Bucket.IN_PROGRESS_PUT), int(L.Bucket.IN_PROGRESS_REPLAY), int(L.Resp.RMW_STALL),
                     int(L.Bucket.IN_PROGRESS_RMW)],
                    size=n, p=[0.62, 0.08, 0.08, 0.04, 0.04, 0.04, 0.04, 0.06])
    a["state"] = st
    ver, cid = tsp.pick(n)
    a["ts_ver"] = ver
    a["ts_cid"] = cid
    a["val_len"] = sizes.st_value >> sizes.shift
    a["flags"] = rng.integers(0, 1 << 16, size=n)
    a["value"] = rng.integers(0, 256, size=(n, sizes.st_value))
    return a


def memb_ops(rng, pool, n, sizes, rmw, tsp) -> np.ndarray:
    a = local_ops(rng, pool, n, sizes, rmw, tsp)
    a["state"] = rng.choice([int(L.Bucket.IN_PROGRESS_PUT), int(L.Bucket.IN_PROGRESS_RMW),
                             int(L.Bucket.IN_PROGRESS_REPLAY), int(L.Bucket.NEW), int(L.Resp.GET_COMPLETE)],
                            size=n, p=[0.35, 0.2, 0.25, 0.1, 0.1])
    return a


def invs(rng, pool, n, sizes, rmw, tsp, machine_num=5) -> np.ndarray:
    a = np.zeros(n, dtype=L.op_dtype(sizes))
    a["key"] = draw_keys(rng, pool, n)
    a["opcode"] = rng.choice([int(L.Op.INV), int(L.Op.MEMBERSHIP_CHANGE)], size=n, p=[0.97, 0.03])
    a["state"] = rng.integers(0, machine_num, size=n)          # sender
    ver, cid = tsp.pick(n)
    bump = rng.choice([0, 2, 4], size=n, p=[0.4, 0.45, 0.15]).astype(np.uint32)
    newcid = rng.integers(0, machine_num, size=n).astype(np.uint8)
    keep = rng.random(n) < 0.5
    a["ts_ver"] = ver + bump
    a["ts_cid"] = np.where(keep, cid, newcid)
    a["val_len"] = sizes.st_value >> sizes.shift
    a["flags"] = rng.integers(0, 1 << 16, size=n) if rmw else rng.integers(0, 2, size=n)
    a["value"] = rng.integers(0, 256, size=(n, sizes.st_value))
    for v, c in zip(a["ts_ver"][:64], a["ts_cid"][:64]):
        tsp.add(v, c)
    return a


def acks(rng, pool, n, sizes, rmw, tsp, machine_num=5):
    """16-byte ACKs, or (RMW build) 56-byte elements mixing ACKs and INV-aborts."""
    if rmw:
        a = np.zeros(n, dtype=L.op_dtype(sizes))
        a["value"] = rng.integers(0, 256, size=(n, sizes.st_value))
        a["flags"] = rng.integers(0, 1 << 16, size=n)
        a["opcode"] = rng.choice([int(L.Op.ACK), int(L.Resp.OP_INV_ABORT)], size=n, p=[0.85, 0.15])
        sender_field = "state"
    else:
        a = np.zeros(n, dtype=L.msg_dtype())
        a["opcode"] = int(L.Op.ACK)
        sender_field = "sender"
    a["key"] = draw_keys(rng, pool, n)
    snd = rng.integers(0, machine_num, size=n)
    memb = rng.random(n) < 0.03
    a[sender_field] = np.where(memb, int(L.Op.MEMBERSHIP_CHANGE), snd)
    ver, cid = tsp.pick(n)
    a["ts_ver"] = ver
    a["ts_cid"] = cid
    return a


def vals(rng, pool, n, sizes, rmw, tsp, machine_num=5):
    a = np.zeros(n, dtype=L.msg_dtype())
    a["key"] = draw_keys(rng, pool, n)
    a["opcode"] = int(L.Op.VAL)
    a["sender"] = rng.integers(0, machine_num, size=n)
    ver, cid = tsp.pick(n)
    a["ts_ver"] = ver
    a["ts_cid"] = cid
    return a


def harvest_ts(tsp: TsPool, elems: np.ndarray):
    """Remember timestamps that local writes produced (ACKs / VALs can then match them)."""
    ok = np.isin(elems["state"], [int(L.Resp.PUT_SUCCESS), int(L.Resp.RMW_SUCCESS), int(L.Resp.REPLAY_SUCCESS)])
    for v, c in zip(elems["ts_ver"][ok][:256], elems["ts_cid"][ok][:256]):
        tsp.add(v, c)
