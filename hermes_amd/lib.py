"""ctypes binding of libhermeskv.so (the C ABI in include/hermeskv.h).

The shared library is built in-tree by `__graft_entry__.build()` (hipcc, gfx950). There is no
fallback: if the library is missing or cannot be loaded, importing this module raises.
torch is imported first so that libhermeskv.so binds to the same HIP runtime torch uses
(both carry SONAME libamdhip64.so.7), which lets torch tensors be passed as device buffers.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# HKV_LIB: another build of the same library (A/B timing of two revisions in one GPU session)
LIB_PATH = os.environ.get("HKV_LIB") or os.path.join(HERE, "libhermeskv.so")
ABI_VERSION = 8

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")

_L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)


class HkvConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("machine_id", ctypes.c_uint32),
                ("rmw_enabled", ctypes.c_uint32), ("big_objects", ctypes.c_uint32),
                ("extra_cache_lines", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("rw_len", ctypes.c_uint32), ("skew_flags", ctypes.c_uint32),
                ("num_keys", ctypes.c_uint64), ("num_bkts", ctypes.c_uint64),
                ("log_cap", ctypes.c_uint64)]


class HkvBatchDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("n_batches", ctypes.c_int32), ("stride", ctypes.c_int32),
                ("elem_size", ctypes.c_uint16), ("flags", ctypes.c_uint16),
                ("d_elems", ctypes.c_void_p), ("d_counts", ctypes.c_void_p), ("d_rw", ctypes.c_void_p),
                ("rw_stride_bytes", ctypes.c_int64), ("d_node_suspected", ctypes.c_void_p),
                ("membership", ctypes.c_uint8 * 8), ("d_state_out", ctypes.c_void_p),
                ("d_opcode_in", ctypes.c_void_p), ("d_patch", ctypes.c_void_p), ("d_rw_state", ctypes.c_void_p),
                ("d_put_keys", ctypes.c_void_p), ("n_rows", ctypes.c_int32), ("skip_row", ctypes.c_int32),
                ("row_stride", ctypes.c_int64), ("d_ack_out", ctypes.c_void_p), ("ack_out_size", ctypes.c_uint32),
                ("d_phys", ctypes.c_void_p)]


class Membership(ctypes.Structure):
    """spacetime_group_membership (8 bytes) by value. Declared as one 64-bit field: the SysV
    x86-64 ABI classifies both as a single INTEGER eightbyte, and libffi handles a scalar
    field more reliably than an 8-byte array member."""
    _fields_ = [("bits", ctypes.c_uint64)]


_P = ctypes.c_void_p
_L.hkv_abi_version.restype = ctypes.c_int
_L.hkv_debug_modes.restype = ctypes.c_int
_L.hkv_last_error.restype = ctypes.c_char_p
_L.hkv_table_create.argtypes = [ctypes.POINTER(HkvConfig), ctypes.POINTER(_P)]
_L.hkv_table_destroy.argtypes = [_P]
_L.hkv_table_populate.argtypes = [_P, ctypes.c_int64, ctypes.c_int]
_L.hkv_table_config.argtypes = [_P, ctypes.POINTER(HkvConfig)]
_L.hkv_table_set_skew.argtypes = [_P, ctypes.c_uint32]
_L.hkv_batch_async.argtypes = [_P, ctypes.POINTER(HkvBatchDesc), _P]
_L.hkv_sync.argtypes = [_P, _P]
_L.hkv_copy_index.argtypes = [_P, _P, ctypes.c_uint64, ctypes.c_uint64]
_L.hkv_copy_log.argtypes = [_P, _P, ctypes.c_uint64, ctypes.c_uint64]
_L.hkv_log_head.restype = ctypes.c_uint64
_L.hkv_log_head.argtypes = [_P]
_L.hkv_num_index_evictions.restype = ctypes.c_int64
_L.hkv_num_index_evictions.argtypes = [_P]
_L.hkv_device_index.restype = _P
_L.hkv_device_index.argtypes = [_P]
_L.hkv_take_error_flags.argtypes = [_P, ctypes.POINTER(ctypes.c_uint32)]
_L.hkv_device_log.restype = _P
_L.hkv_device_log.argtypes = [_P]
_L.hkv_set_default_config.argtypes = [ctypes.POINTER(HkvConfig)]
_L.hkv_default_table.restype = _P
_L.hkv_hash_ids.argtypes = [_P, _P, ctypes.c_int64, _P]
_L.spacetime_init.argtypes = [ctypes.c_int]
_L.spacetime_populate_fixed_len.argtypes = [_P, ctypes.c_int, ctypes.c_int]
_L.hermes_batch_ops_to_KVS.argtypes = [ctypes.c_int, _P, ctypes.c_int, ctypes.c_uint16, Membership,
                                       ctypes.POINTER(ctypes.c_int), _P, ctypes.c_uint8]

if _L.hkv_abi_version() != ABI_VERSION:
    raise ImportError(f"libhermeskv ABI {_L.hkv_abi_version()} != {ABI_VERSION}")


class HkvError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise HkvError(f"{what}: rc={rc}: {_L.hkv_last_error().decode(errors='replace')}")


def raw() -> ctypes.CDLL:
    return _L


def loaded_path() -> str:
    return LIB_PATH
