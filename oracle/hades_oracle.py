"""CPU restatement of Hades' membership agreement (src/hades/hades.c, include/hades/hades.h,
include/hermes/inline-util.h:26-43), one view-update period per `update()` call.

TEST INFRASTRUCTURE ONLY: tests/ compare libhermeskv's hkv_hades_* (hermes_amd/hades.py) with this
model. Parity pinning: the bit-vector primitives it relies on (bit get/set/reset, equality) are
pinned against the reference's bit_vector.h in tests/test_ref_primitives.py; the agreement itself
cannot be run from the reference here (hades.c needs the wings/ibverbs transport), so it is
"parity unpinned" beyond those primitives and the scenarios in tests/test_hades.py.

Views are (node_id, epoch_id, same_w_local_membership, have_ostracised_for_dst_node, view)
tuples with the hades_view_t fields (hades.h:47-55); bit vectors are ints (bit i = node i).
"""
from __future__ import annotations

import dataclasses

NO_VIEW = 0xFF


@dataclasses.dataclass
class View:
    node_id: int = 0
    epoch_id: int = 0
    same_w: int = 0
    ostracised_for_dst: int = 0
    view: int = 0

    def pack(self) -> bytes:
        """the 4-byte hades_view_t image (gcc bit-field order)"""
        return bytes([self.node_id, self.epoch_id, (self.same_w & 1) | ((self.ostracised_for_dst & 0x7F) << 1),
                      self.view])

    @staticmethod
    def unpack(b: bytes) -> "View":
        return View(b[0], b[1], b[2] & 1, b[2] >> 1, b[3])


def _bit(bv: int, i: int) -> int:
    return (bv >> i) & 1


class HadesModel:
    def __init__(self, max_nodes: int, machine_id: int, arbitration: bool = True):
        """hades_ctx_init, hades.h:99-141"""
        assert 2 <= max_nodes <= 8 and machine_id < max_nodes
        self.n, self.me, self.arbitration = max_nodes, machine_id, arbitration
        self.intermediate = View(machine_id, 0, 0, 0, 1 << machine_id)
        self.curr_g = 1 << machine_id
        self.last_local = dataclasses.replace(self.intermediate)
        self.recved = [0] * max_nodes
        self.remote = [View() for _ in range(max_nodes)]
        self.ostracized_for = [0] * max_nodes

    def majority(self) -> int:  # majority_of_nodes, hades.c:62-67
        return 2 if self.n == 2 else self.n // 2 + 1

    def skip(self, i: int) -> bool:  # skip_arbitration, hades.c:127-139
        return (i == self.me or not self.recved[i] or self.remote[i].ostracised_for_dst == 1
                or not _bit(self.remote[i].view, self.me))

    def ostracism(self):  # view_arbitration_via_ostracism, hades.c:150-184
        self.ostracized_for = [0] * self.n
        for i in range(self.n):
            if self.skip(i):
                continue
            for j in range(self.n):
                if i >= j or self.skip(j):
                    continue
                ivj, jvi = _bit(self.remote[i].view, j), _bit(self.remote[j].view, i)
                if ivj == 0 or jvi == 0:
                    out, fr = (i, j) if ivj == 1 else (j, i)
                    self.recved[out] = 0
                    self.ostracized_for[fr] = 1
                    self.intermediate.view &= ~(1 << out) & 0xFF

    def max_received_epoch(self) -> int:  # get_max_received_epoch_id, hades.c:186-195
        m = 0
        for i in range(self.n):
            if self.recved[i] and self.remote[i].epoch_id > m:
                m = self.remote[i].epoch_id
        return m

    def view_for(self, dst: int) -> View:  # issue_heartbeats, hades.c:256-283
        v = dataclasses.replace(self.last_local)
        v.ostracised_for_dst = self.ostracized_for[dst]
        return v

    def receive(self, v: View):  # poll_for_remote_views, hades.c:296-331
        s = v.node_id
        if s == NO_VIEW or s >= self.n:
            return
        self.recved[s] = 1
        self.remote[s] = dataclasses.replace(v)
        self.intermediate.view |= 1 << s

    def update(self) -> tuple[bool, bool]:
        """update_view_n_membership, hades.c:197-253 -> (membership changed, majority in view)"""
        before = self.curr_g
        agreeing, same_w, max_epoch = 1, 0, self.intermediate.epoch_id
        if self.arbitration:
            self.ostracism()
        if self.intermediate.view != self.curr_g or self.max_received_epoch() > self.intermediate.epoch_id:
            for i in range(self.n):
                if i == self.me or not self.recved[i]:
                    continue
                if self.intermediate.view == self.remote[i].view:
                    agreeing += 1
                    if max_epoch < self.remote[i].epoch_id:
                        max_epoch = self.remote[i].epoch_id
                        same_w = self.remote[i].same_w
                self.recved[i] = 0
            if agreeing >= self.majority():
                self.intermediate.epoch_id = (max_epoch + (0 if same_w == 1 else 1)) & 0xFF
                self.curr_g = self.intermediate.view
        maj = bin(self.intermediate.view).count("1") >= self.majority()
        self.last_local = dataclasses.replace(self.intermediate)
        self.last_local.same_w = int(self.last_local.view == self.curr_g)
        self.intermediate.view = 1 << self.me
        return self.curr_g != before, maj

    def membership(self) -> bytes:
        """group_membership_update, inline-util.h:26-43: the 8-byte spacetime_group_membership"""
        g = self.curr_g
        return bytes([bin(g).count("1"), g, (~g | (1 << self.me)) & 0xFF, 0, 0, 0, 0, 0])
