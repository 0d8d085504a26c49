"""ctypes binding of the CPU restatement (hkv_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker or the timed CPU baseline. The product path (hermes_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libhkv_oracle.so")
CITY_REF_PATH = os.path.join(HERE, "_ref", "libcity_ref.so")


class Config(ctypes.Structure):
    _fields_ = [("big_objects", ctypes.c_uint32), ("extra_cache_lines", ctypes.c_uint32),
                ("rmw_enabled", ctypes.c_uint32), ("machine_id", ctypes.c_uint32),
                ("num_bkts", ctypes.c_uint64), ("log_cap", ctypes.c_uint64),
                ("skew_flags", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


def build(force: bool = False) -> None:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "build/libhkv_oracle.so"], check=True,
                       stdout=subprocess.DEVNULL)


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P, U8P = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)
        L.hko_create.restype = P
        L.hko_create.argtypes = [ctypes.POINTER(Config)]
        L.hko_destroy.argtypes = [P]
        L.hko_populate.argtypes = [P, ctypes.c_int64, ctypes.c_int]
        L.hko_set_machine_id.argtypes = [P, ctypes.c_uint32]
        L.hko_batch.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_uint16, P,
                                ctypes.POINTER(ctypes.c_int), P]
        L.hko_batch_multi.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P,
                                      ctypes.c_uint16, P, P, P, ctypes.c_int64]
        L.hko_index.restype = U8P
        L.hko_index.argtypes = [P]
        L.hko_log.restype = U8P
        L.hko_log.argtypes = [P]
        L.hko_log_head.restype = ctypes.c_uint64
        L.hko_log_head.argtypes = [P]
        L.hko_num_index_evictions.restype = ctypes.c_int64
        L.hko_num_index_evictions.argtypes = [P]
        L.hko_lookup.restype = U8P
        L.hko_lookup.argtypes = [P, ctypes.c_uint64]
        L.hko_cityhash128.argtypes = [P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
        L.hko_gen_keys.argtypes = [P, ctypes.c_int64]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def cityhash128(data: bytes):
    f, s = ctypes.c_uint64(), ctypes.c_uint64()
    buf = ctypes.create_string_buffer(data, len(data))
    lib().hko_cityhash128(ctypes.cast(buf, ctypes.c_void_p), len(data), ctypes.byref(f), ctypes.byref(s))
    return f.value, s.value


def gen_keys(n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint64)
    lib().hko_gen_keys(_ptr(out), n)
    return out


class OracleKVS:
    """One MICA-herd/HermesKV table on the host, driven exactly like the reference."""

    def __init__(self, num_bkts: int, log_cap: int, machine_id: int = 0, rmw: bool = False,
                 big_objects: bool = False, extra_cache_lines: int = 0, skew: int = 0):
        """skew: hko_config.skew_flags (bit 0 read completion, bit 1 write coalescing, config.h:79-80)"""
        self.cfg = Config(int(big_objects), int(extra_cache_lines), int(rmw), machine_id, num_bkts, log_cap,
                          int(skew), 0)
        self.h = lib().hko_create(ctypes.byref(self.cfg))
        self.num_bkts, self.log_cap = num_bkts, log_cap

    def __del__(self):
        if getattr(self, "h", None):
            lib().hko_destroy(self.h)
            self.h = None

    def populate(self, n: int, val_len: int) -> None:
        lib().hko_populate(self.h, n, val_len)

    def batch(self, btype: int, ops: np.ndarray, membership: bytes, rw: np.ndarray | None = None,
              op_num: int | None = None) -> int:
        """hermes_batch_ops_to_KVS on a numpy structured array (mutated in place).
        Returns node_suspected (-1 when unchanged)."""
        mb = np.frombuffer(membership, dtype=np.uint8).copy()
        ns = ctypes.c_int(-1)
        n = len(ops) if op_num is None else op_num
        lib().hko_batch(self.h, int(btype), _ptr(ops), n, ops.dtype.itemsize, _ptr(mb),
                        ctypes.byref(ns), _ptr(rw) if rw is not None else None)
        return ns.value

    def batch_multi(self, btype: int, ops: np.ndarray, n_batches: int, stride: int,
                    counts: np.ndarray | None, membership: bytes, rw: np.ndarray | None = None,
                    rw_stride_elems: int = 0, node_suspected: np.ndarray | None = None) -> None:
        mb = np.frombuffer(membership, dtype=np.uint8).copy()
        c = None if counts is None else np.ascontiguousarray(counts, dtype=np.int32)
        lib().hko_batch_multi(self.h, int(btype), _ptr(ops), n_batches, stride,
                              _ptr(c) if c is not None else None, ops.dtype.itemsize, _ptr(mb),
                              _ptr(node_suspected) if node_suspected is not None else None,
                              _ptr(rw) if rw is not None else None,
                              rw_stride_elems * (rw.dtype.itemsize if rw is not None else 0))

    def index_bytes(self) -> np.ndarray:
        return np.ctypeslib.as_array(lib().hko_index(self.h), shape=(self.num_bkts * 64,))

    def log_bytes(self) -> np.ndarray:
        return np.ctypeslib.as_array(lib().hko_log(self.h), shape=(self.log_cap,))

    def log_head(self) -> int:
        return lib().hko_log_head(self.h)

    def evictions(self) -> int:
        return lib().hko_num_index_evictions(self.h)

    def lookup(self, key: int):
        """Return the byte offset of the key's log entry, or None on a miss."""
        p = lib().hko_lookup(self.h, ctypes.c_uint64(int(key)))
        if not p:
            return None
        return ctypes.cast(p, ctypes.c_void_p).value - ctypes.cast(lib().hko_log(self.h), ctypes.c_void_p).value


class _U128(ctypes.Structure):
    _fields_ = [("first", ctypes.c_uint64), ("second", ctypes.c_uint64)]


def reference_cityhash128(data: bytes):
    """The reference's own CityHash128 (src/mica-herd/city.c), built into _ref/ by the Makefile.
    Returns None when /root/reference is absent and the library was never built."""
    if not os.path.exists(CITY_REF_PATH):
        if os.path.isdir("/root/reference"):
            subprocess.run(["make", "-C", HERE, "ref"], check=True, stdout=subprocess.DEVNULL)
        else:
            return None
    L = ctypes.CDLL(CITY_REF_PATH)
    L.CityHash128.restype = _U128
    L.CityHash128.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    r = L.CityHash128(data, len(data))
    return r.first, r.second
