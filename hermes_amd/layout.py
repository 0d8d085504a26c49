"""Byte layouts and protocol codes of the HermesKV batch path.

Everything here restates the reference's C definitions so that host code can build and
read the exact byte images the reference's `hermes_batch_ops_to_KVS` consumes:

* codes: include/hermes/spacetime.h:32-121
* spacetime_op_meta_t / ack / val (16 B): spacetime.h:151-166
* spacetime_op_t / spacetime_inv_t (56 B, 312 B with big objects): spacetime.h:170-185
* spacetime_object_meta (15 B): spacetime.h:138-148, inside a mica_op log entry
  (include/mica-herd/mica.h:55-60) at byte 18
* spacetime_group_membership (8 B): spacetime.h:188-195
* value sizes: include/mica-herd/hrd.h:36-47 (BASE_VALUE_SIZE 46, big objects add
  EXTRA_CACHE_LINES * 64 and use SHIFT_BITS 3)
"""
from __future__ import annotations

import dataclasses
import enum

import numpy as np


class State(enum.IntEnum):  # spacetime.h:42-48
    VALID = 1
    INVALID = 2
    INVALID_WRITE = 3
    WRITE = 4
    REPLAY = 5


class Op(enum.IntEnum):  # input opcodes, spacetime.h:51-62
    GET = 111
    PUT = 112
    RMW = 113
    INV = 114
    ACK = 115
    VAL = 116
    CRD = 117
    MEMBERSHIP_CHANGE = 118
    MEMBERSHIP_COMPLETE = 119


class Resp(enum.IntEnum):  # response opcodes, spacetime.h:65-89
    GET_COMPLETE = 121
    PUT_SUCCESS = 122
    REPLAY_SUCCESS = 123
    INV_SUCCESS = 124
    ACK_SUCCESS = 125
    LAST_ACK_SUCCESS = 126
    LAST_ACK_NO_BCAST_SUCCESS = 127
    PUT_COMPLETE = 128
    VAL_SUCCESS = 129
    MISS = 130
    GET_STALL = 131
    PUT_STALL = 132
    PUT_COMPLETE_SEND_VALS = 133
    SEND_CRD = 134
    RMW_SUCCESS = 135
    RMW_STALL = 136
    RMW_COMPLETE = 137
    RMW_ABORT = 138
    OP_INV_ABORT = 139


class Bucket(enum.IntEnum):  # op-bucket states, spacetime.h:95-106
    EMPTY = 140
    NEW = 141
    COMPLETE = 142
    IN_PROGRESS_PUT = 143
    IN_PROGRESS_REPLAY = 144
    REPLAY_COMPLETE = 145
    IN_PROGRESS_GET = 146
    REPLAY_COMPLETE_SEND_VALS = 147
    IN_PROGRESS_RMW = 148
    RMW_COMPLETE_SEND_VALS = 149


INV_OUT_OF_GROUP = 153  # spacetime.h:109-113
NOP = 150
OBI_EMPTY = 255
LWID_EMPTY = 127
CID_EMPTY = 255


class BatchType(enum.IntEnum):  # enum hermes_batch_type_t, spacetime.h:219-226
    local_ops = 0
    local_ops_after_membership_change = 1
    invs = 2
    acks = 3
    vals = 4


OP_META_SIZE = 16
OP_VALUE_OFF = 18         # spacetime_op_t.value (after the 16-B meta and the 2-B flags)
OBJ_META_SIZE = 15
ENTRY_META_OFF = 18
BUCKET_SIZE = 64
MAX_LOCAL_BATCH = 250      # MAX_BATCH_KVS_OPS_SIZE, config.h:42
MAX_MSG_BATCH = 900        # HERMES_MAX_BATCH_SIZE, config.h:158-159


@dataclasses.dataclass(frozen=True)
class Sizes:
    """Derived sizes for one build variant (default, or USE_BIG_OBJECTS)."""

    big_objects: bool = False
    extra_cache_lines: int = 0

    @property
    def kvs_value(self) -> int:  # KVS_VALUE_SIZE, hrd.h:47
        return self.extra_cache_lines * 64 + 46 if self.big_objects else 46

    @property
    def st_value(self) -> int:  # ST_VALUE_SIZE, spacetime.h:29
        return self.kvs_value - OBJ_META_SIZE

    @property
    def shift(self) -> int:  # SHIFT_BITS, hrd.h:39
        return 3 if self.big_objects else 0

    @property
    def entry(self) -> int:  # sizeof(struct mica_op)
        return (ENTRY_META_OFF + self.kvs_value + 7) & ~7

    @property
    def op(self) -> int:  # sizeof(spacetime_op_t)
        return (OP_META_SIZE + 2 + self.st_value + 7) & ~7


DEFAULT = Sizes()
BIG = Sizes(True, 4)


def op_dtype(sz: Sizes = DEFAULT) -> np.dtype:
    """numpy view of spacetime_op_t / spacetime_inv_t (spacetime.h:170-185)."""
    return np.dtype({
        "names": ["key", "opcode", "state", "val_len", "ts_cid", "ts_ver", "flags", "value"],
        "formats": ["<u8", "u1", "u1", "u1", "u1", "<u4", "<u2", ("u1", sz.st_value)],
        "offsets": [0, 8, 9, 10, 11, 12, 16, 18],
        "itemsize": sz.op,
    })


def msg_dtype() -> np.dtype:
    """numpy view of spacetime_ack_t / spacetime_val_t (spacetime.h:151-166)."""
    return np.dtype({
        "names": ["key", "opcode", "sender", "val_len", "ts_cid", "ts_ver"],
        "formats": ["<u8", "u1", "u1", "u1", "u1", "<u4"],
        "offsets": [0, 8, 9, 10, 11, 12],
        "itemsize": OP_META_SIZE,
    })


def entry_dtype(sz: Sizes = DEFAULT) -> np.dtype:
    """numpy view of a mica_op log entry carrying a spacetime_object_meta (spacetime.h:138-148)."""
    return np.dtype({
        "names": ["key_first", "key", "opcode", "val_len", "state", "ack_bv", "rmw_lwid", "obi",
                  "lock", "ts_cid", "ts_ver", "llw_cid", "llw_ver", "value"],
        "formats": ["<u8", "<u8", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "<u4", "u1",
                    "<u4", ("u1", sz.st_value)],
        "offsets": [0, 8, 16, 17, 18, 19, 20, 21, 22, 23, 24, 28, 29, 33],
        "itemsize": sz.entry,
    })


def membership(machine_num: int, machine_id: int, alive: int | None = None) -> bytes:
    """spacetime_group_membership by value (group_membership_init, main.c:37-49).

    `alive` overrides g_membership (a bit mask) to model a membership change
    (group_membership_update, inline-util.h:26-43)."""
    g = ((1 << machine_num) - 1) if alive is None else alive
    g &= 0xFF
    w_ack_init = ((~g) & 0xFF) | (1 << machine_id)
    n_alive = bin(g).count("1") if alive is not None else machine_num - 1
    return bytes([n_alive & 0xFF, g, w_ack_init & 0xFF, 0, 0, 0, 0, 0])


def ts64(version, cid):
    """Packed Lamport timestamp: (version, cid) order == integer order (concur_ctrl.h:70-75)."""
    return (np.asarray(version, dtype=np.uint64) << np.uint64(8)) | np.asarray(cid, dtype=np.uint64)
