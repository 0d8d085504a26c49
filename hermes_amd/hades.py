"""Hades membership agreement for a replica group (include/hermeskv_hades.h).

`Hades` wraps one replica's hkv_hades context. `exchange_views` is one heartbeat exchange: every
replica's view for every destination, as a [N][N] table of 4-byte hades_view_t images (row =
sender), with HKV_HADES_NO_VIEW where a message was lost (a failed node, a cut link); each
replica then receives its column.
"""
from __future__ import annotations

import ctypes

from .lib import check, raw

_L = raw()
NO_VIEW = 0xFF


class HkvHadesView(ctypes.Structure):
    _fields_ = [("node_id", ctypes.c_uint8), ("epoch_id", ctypes.c_uint8), ("flags", ctypes.c_uint8),
                ("view", ctypes.c_uint8)]


_P = ctypes.c_void_p
_L.hkv_hades_create.argtypes = [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_int, ctypes.POINTER(_P)]
_L.hkv_hades_destroy.argtypes = [_P]
_L.hkv_hades_destroy.restype = None
_L.hkv_hades_view_for.argtypes = [_P, ctypes.c_uint8, ctypes.POINTER(HkvHadesView)]
_L.hkv_hades_receive.argtypes = [_P, ctypes.POINTER(HkvHadesView)]
_L.hkv_hades_update.argtypes = [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
_L.hkv_hades_state.argtypes = [_P, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint8)]


class MajorityLost(RuntimeError):
    """group_membership_update (inline-util.h:39-42) exits when fewer than half the machines remain"""


class Hades:
    def __init__(self, max_nodes: int, machine_id: int, arbitration: bool = True):
        self.n, self.me = max_nodes, machine_id
        h = _P()
        check(_L.hkv_hades_create(max_nodes, machine_id, int(arbitration), ctypes.byref(h)), "hkv_hades_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            _L.hkv_hades_destroy(self.h)
            self.h = None

    def view_for(self, dst: int) -> bytes:
        v = HkvHadesView()
        check(_L.hkv_hades_view_for(self.h, dst, ctypes.byref(v)), "hkv_hades_view_for")
        return bytes(v)

    def receive(self, view: bytes) -> None:
        v = HkvHadesView.from_buffer_copy(view)
        check(_L.hkv_hades_receive(self.h, ctypes.byref(v)), "hkv_hades_receive")

    def update(self) -> tuple[bool, bytes, bool]:
        """One view-update period -> (membership changed, spacetime_group_membership, majority)"""
        out = ctypes.create_string_buffer(8)
        maj = ctypes.c_int(0)
        rc = _L.hkv_hades_update(self.h, out, ctypes.byref(maj))
        if rc < 0:
            check(rc, "hkv_hades_update")
        return rc == 1, out.raw, bool(maj.value)

    def state(self) -> tuple[int, int]:
        g, e = ctypes.c_uint8(), ctypes.c_uint8()
        check(_L.hkv_hades_state(self.h, ctypes.byref(g), ctypes.byref(e)), "hkv_hades_state")
        return g.value, e.value

    def views_row(self) -> bytes:
        """this replica's heartbeats, one 4-byte view per destination (its own slot empty)"""
        return b"".join(self.view_for(d) if d != self.me else bytes([NO_VIEW, 0, 0, 0]) for d in range(self.n))

    def receive_column(self, table: bytes) -> None:
        """poll: the views addressed to this replica in an [N][N] table of 4-byte views"""
        for s in range(self.n):
            if s != self.me:
                self.receive(table[(s * self.n + self.me) * 4:(s * self.n + self.me + 1) * 4])


def exchange_views(hs: list[Hades | None], lost=lambda src, dst: False) -> bytes:
    """One heartbeat exchange among replicas in one process (None = a failed replica, which sends
    nothing); lost(src, dst) cuts a link one way. Returns the [N][N] table after the losses."""
    n = len(hs)
    rows = []
    for s, h in enumerate(hs):
        row = bytearray(h.views_row() if h is not None else bytes([NO_VIEW, 0, 0, 0]) * n)
        for d in range(n):
            if lost(s, d):
                row[d * 4:(d + 1) * 4] = bytes([NO_VIEW, 0, 0, 0])
        rows.append(bytes(row))
    table = b"".join(rows)
    for h in hs:
        if h is not None:
            h.receive_column(table)
    return table
