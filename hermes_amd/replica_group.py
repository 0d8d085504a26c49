"""A Hermes replica group with one replica per GPU.

Hermes replicates every key on every node, so N GPUs form an N-replica group (N <= 8: the
membership bit vectors are 8 bits wide, spacetime.h:188-195). The wings RDMA layer
(wings.h:770-916) becomes three data collectives per protocol round, on torch's current stream:

  1. every replica packs the round's INVs (at most C per worker: the send credits) into one
     contiguous slab, worker after worker; the totals are all-gathered and the host reads the
     largest, the round's width (the one host synchronisation of a round). The INV slabs are
     all-gathered as [N][width] x op_size
  2. every replica applies its peers' INVs as one INV batch launch of N batches (one per peer,
     its own masked out by a zero count); the ACKs (INV-aborts with RMWs) are written in the
     positions of the INVs they answer and go back to the coordinators with an all-to-all:
     row p of the ACK slab holds rank p's ACKs, lined up with the slab rank p sent
  3. coordinators regroup the ACKs per worker through their own packing offsets (one receive
     poll over all peers), apply them as an ACK batch against the worker's op buffer
     (read_write_ops), pack the VALs of the writes that completed and all-gather them at the
     same width (a round completes at most the writes it INV'd); every replica applies its
     peers' VALs as one VAL batch.

Packed slabs carry what a round sends, not the credits' worst case: at 20 % writes about 24 INVs
per worker go out, against C = 104 slots, so the collectives and the INV/VAL launches are about
4x smaller than with [N][W][C] rows. `ReplicaRound` holds one replica's buffers and phases;
`ReplicaGroupRound` drives one replica per process over torch.distributed (RCCL);
`LoopbackGroup` drives N replicas in one process (tests: the same phases and kernels, with the
collectives done by tensor copies).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import layout as L
from .kvs import HermesKV
from .lib import check, raw
from .hades import NO_VIEW, Hades, MajorityLost, exchange_views
from .workload import HkvZipf, _ptr, _s, init_mirrors, refill_flags, slots_per_worker  # noqa: F401 (re-exported)

_L = raw()
_P = ctypes.c_void_p
_L.hkv_wl_marshal_acks_rows.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P,
                                        ctypes.c_uint32, _P, ctypes.c_uint32, _P]
_L.hkv_wl_regroup.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P,
                              ctypes.c_int32, _P, _P]
_L.hkv_wl_collect_vals.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32,
                                   _P, ctypes.c_uint32, _P, _P, _P]
_L.hkv_wl_fold_counters.argtypes = [_P, _P]
_L.hkv_wl_pack_rows.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, _P, _P]
_L.hkv_wl_marshal_acks_aligned.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P,
                                           ctypes.c_uint32, ctypes.c_uint32, _P]
_L.hkv_wl_marshal_memb_vals.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32, _P,
                                        ctypes.c_uint32, _P, _P]
_L.hkv_wl_regroup_aligned.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_uint32,
                                      _P, ctypes.c_int32, _P, _P]
_L.hkv_wl_marshal_invs_packed.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32,
                                          ctypes.c_int32, _P, _P, _P, _P, ctypes.c_uint32, _P, _P]
_L.hkv_wl_collect_vals_rows.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, _P,
                                        ctypes.c_int32, _P, ctypes.c_uint32, _P, _P, _P]

MAX_REPLICAS = 8
LOCAL = 250  # MAX_BATCH_KVS_OPS_SIZE, config.h:42


class ReplicaRound:
    """Buffers and phases of one replica (machine id = rank) of an N-replica group."""

    def __init__(self, kvs: HermesKV, n_workers: int, world: int, rank: int, zipf: HkvZipf,
                 write_permille: int = 200, rmw_permille: int = 0, seed: int = 0x5EED,
                 trace_len: int = 8192, retry_stalled: bool = False, slots: int | None = None,
                 fused_refill: bool = True):
        if not 2 <= world <= MAX_REPLICAS:
            raise ValueError(f"a replica group has 2..{MAX_REPLICAS} replicas, got {world}")
        if kvs.machine_id != rank:
            raise ValueError("the replica's table must use machine_id == rank")
        self.kvs, self.W, self.N, self.rank = kvs, n_workers, world, rank
        self.sizes = kvs.sizes
        self.op = kvs.sizes.op
        self.ack_size = self.op if kvs.rmw else L.OP_META_SIZE
        self.mb = L.membership(world, rank)
        self.retry = retry_stalled
        self.rflags = refill_flags(kvs, retry_stalled)
        self.C = slots or slots_per_worker(write_permille, rmw_permille)
        W, N, C = n_workers, world, self.C
        dev = torch.device("cuda", kvs.device)
        u8 = dict(dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.ops = torch.zeros(W * LOCAL * self.op, **u8)
        self.states = torch.zeros(W * LOCAL, dtype=torch.uint8, device=dev)  # local batch state mirror
        self.opcodes = torch.zeros(W * LOCAL, dtype=torch.uint8, device=dev)  # the refill's opcode mirror
        # refills planned from the state mirror and applied by the next local launch (workload.Round)
        self.fused = fused_refill and self.op <= 64
        self.patch = torch.zeros(W * LOCAL * 16, **u8) if self.fused else None
        # outgoing INVs: [W][C] rows, then packed (worker w at inv_off[w]; inv_off[W] = total)
        self.inv_count = torch.zeros(W, **i32)           # INVs each worker sends this round
        self.inv_sendable = torch.zeros(W, **i32)        # ... and could send (the rest are held)
        self.inv_off = torch.zeros(W + 1, **i32)
        # the INVs go straight into the packed slab, at most `cap` per rank and round (local(cap)), so the
        # group can size its collectives without a host read
        self.packed_marshal = True
        self.inv_pack = torch.zeros(W * C * self.op, **u8)
        self.inv_totals = torch.zeros(N, **i32)          # all ranks' INV totals (this round's width: max)
        self.inv_maxc = torch.zeros(1, **i32)            # this rank's largest per-worker INV count
        # receive buffers at the largest width (W * C); a round uses [N][width] of them
        self.inv_recv = torch.zeros(N * W * C * self.op, **u8)
        self.ack_slab = torch.zeros(N * W * C * self.ack_size, **u8)
        self.ack_recv = torch.zeros(N * W * C * self.ack_size, **u8)
        self.ack_batch = torch.zeros(W * N * C * self.ack_size, **u8)
        self.ack_batch_count = torch.zeros(W, **i32)
        self.val_slab = torch.zeros(W * C * L.OP_META_SIZE, **u8)
        self.val_count = torch.zeros(W, **i32)
        self.val_off = torch.zeros(W + 1, **i32)
        self.val_pack = torch.zeros(W * C * L.OP_META_SIZE, **u8)
        self.val_totals = torch.zeros(N, **i32)
        self.val_recv = torch.zeros(N * W * C * L.OP_META_SIZE, **u8)
        self.held = torch.zeros(2, dtype=torch.int64, device=dev)    # INVs held back, VALs dropped
        self.cursor = torch.zeros(W, **i32)
        self.counters = torch.zeros(4096, dtype=torch.int64, device=dev)  # HKV_WL_COUNTER_WORDS
        self.inv_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.elem_totals = torch.zeros(3, dtype=torch.int64, device=dev)  # INV, ACK, VAL elements applied
        self.count_elems = True        # keep inv_total / elem_totals (small torch ops per phase)
        self.trace_len = trace_len
        self.trace_key = torch.empty(W * trace_len, dtype=torch.int64, device=dev)
        self.trace_op = torch.empty(W * trace_len, **u8)
        check(_L.hkv_wl_gen_trace(_ptr(self.trace_key), _ptr(self.trace_op), None, W, trace_len,
                                  ctypes.byref(zipf), write_permille, rmw_permille,
                                  ctypes.c_uint64(seed ^ (rank << 48)), _s()), "gen_trace")
        self.failed = False            # this replica has failed (fail()): it sends nothing more
        # ACK rows applied as they arrive, one unique-key launch per peer (a peer answers each of this
        # replica's INVs once, and a key has one local write in flight), with no regroup pass; once any
        # replica has failed, its rows hold empty slots and the regrouped batch takes over for good
        self.unique_acks = True
        # ... all peers' rows in one launch (HKV_BATCH_ROWS, this rank's own row skipped; 64-B entries and
        # 16-B ACKs, otherwise one launch per peer)
        self.ack_rows = self.sizes.entry == 64 and self.ack_size <= 64
        self.own_total = None          # this round's packed INV total, when read back (round_shape)
        # this replica's ACKs to a peer's INVs written by that peer's INV launch itself (hkv_batch_desc.d_ack_out,
        # as at N = 1) instead of a marshal pass over the applied row
        self.fused_acks = (self.sizes.entry == 64 and self.op <= 64) or (self.sizes.entry == 320 and self.op <= 320)
        self.refill(first=True)

    # -- Hades: one view-update period per round when enabled
    def hades_start(self):
        self.hades = Hades(self.N, self.rank)

    def hades_row(self, changed: bool) -> bytes:
        """this replica's heartbeats (one 4-byte view per destination) and a 4-byte trailer:
        [membership changed this period, membership is the whole group]; a failed replica sends
        nothing"""
        if self.failed:
            return bytes([NO_VIEW, 0, 0, 0]) * self.N + bytes(4)
        g, _ = self.hades.state()
        return self.hades.views_row() + bytes([int(changed), int(g == (1 << self.N) - 1), 0, 0])

    # -- phases (all asynchronous on torch's current stream)
    def fail(self):
        """This replica fails after its INVs of the current round went out: from now on it sends
        no ACKs, VALs or INVs (it still joins the collectives, with empty slabs)."""
        self.failed = True
        self.unique_acks = False

    def peer_failing(self):
        """Some replica fails this round: its ACK rows hold empty slots from now on"""
        self.unique_acks = False

    def refill(self, first: bool = False):
        if self.failed:
            return
        if self.fused and not first:
            check(_L.hkv_wl_refill_plan(_ptr(self.states), self.W, LOCAL, self.sizes.st_value, self.sizes.shift,
                                        _ptr(self.trace_key), _ptr(self.trace_op), self.trace_len, _ptr(self.cursor),
                                        self.rank, self.rflags, _ptr(self.counters), _ptr(self.opcodes),
                                        _ptr(self.patch), _s()), "refill_plan")
            return
        check(_L.hkv_wl_refill(_ptr(self.ops), self.W, LOCAL, self.op, self.sizes.st_value, self.sizes.shift,
                               _ptr(self.trace_key), _ptr(self.trace_op), None, self.trace_len, _ptr(self.cursor),
                               self.rank, int(first), self.rflags, _ptr(self.counters), _ptr(self.opcodes), None,
                               _s()), "refill")
        if first:
            init_mirrors(self.ops, self.op, self.states)

    def local(self, cap: int | None = None):
        """Local batch, then this round's INVs, packed (inv_pack; worker w at inv_off[w]); at most `cap` of
        them (the rest keep their state and go out in a later round, counted in held[0])."""
        if self.failed:
            self.inv_count.zero_()
            self.inv_off.zero_()
            self.inv_maxc.zero_()
            return
        self.kvs.batch(L.BatchType.local_ops, self.ops, self.W, LOCAL, self.op, self.mb, state_out=self.states,
                       opcode_in=self.opcodes, patch=self.patch)
        check(_L.hkv_wl_marshal_invs_packed(_ptr(self.ops), self.W, LOCAL, self.op, _ptr(self.states), self.C,
                                            self.W * self.C if cap is None else int(cap), _ptr(self.inv_pack),
                                            _ptr(self.inv_off), _ptr(self.inv_sendable), _ptr(self.inv_count),
                                            self.rank, _ptr(self.held), _s()), "marshal_invs_packed")
        torch.amax(self.inv_count, dim=0, keepdim=True, out=self.inv_maxc)
        if self.count_elems:
            self.inv_total += self.inv_off[self.W]

    # -- the slabs each collective moves: (receive, send) views at the round's width
    def inv_total_io(self):
        return self.inv_totals, self.inv_off[self.W:]

    def round_shape(self) -> tuple[int, int]:
        """After the totals are gathered (host synchronisation): the round's width (the largest
        INV total of any rank) and this rank's ACK batch stride ((N-1) x its largest per-worker
        INV count: a worker gets at most one ACK per INV from every peer). Also keeps this rank's
        own INV total (own_total) for the per-peer ACK launches."""
        v = torch.cat([self.inv_totals.max().view(1), self.inv_maxc, self.inv_off[self.W:]]).cpu().tolist()
        self.own_total = int(v[2])
        return max(1, int(v[0])), max(1, (self.N - 1) * int(v[1]))

    def inv_io(self, width: int):
        n = width * self.op
        return self.inv_recv[:self.N * n], self.inv_pack[:n]

    def ack_io(self, width: int):
        n = self.N * width * self.ack_size
        return self.ack_recv[:n], self.ack_slab[:n]

    def val_total_io(self):
        return self.val_totals, self.val_off[self.W:]

    def val_io(self, width: int):
        n = width * L.OP_META_SIZE
        return self.val_recv[:self.N * n], self.val_pack[:n]

    # steady rounds (WidthPlan): each slab is one slot wider than the INV cap and carries its rank's
    # total in that spare slot, so the totals travel with the slabs (two collectives per round fewer)
    def _put_total(self, pack, width: int, size: int, off) -> None:
        a = (width - 1) * size
        pack[a:a + 4].view(torch.int32).copy_(off[self.W:])

    def _take_totals(self, recv, width: int, size: int, out) -> None:
        a = (width - 1) * size
        out.copy_(recv[:self.N * width * size].view(self.N, width * size)[:, a:a + 4].view(torch.int32).view(-1))

    def inv_io_total(self, width: int):
        """inv_io, the spare slot (width - 1) of the send slab holding this rank's INV total"""
        self._put_total(self.inv_pack, width, self.op, self.inv_off)
        return self.inv_io(width)

    def take_inv_totals(self, width: int) -> None:
        """inv_totals from the spare slots of the gathered INV slabs"""
        self._take_totals(self.inv_recv, width, self.op, self.inv_totals)

    def val_io_total(self, width: int):
        self._put_total(self.val_pack, width, L.OP_META_SIZE, self.val_off)
        return self.val_io(width)

    def take_val_totals(self, width: int) -> None:
        self._take_totals(self.val_recv, width, L.OP_META_SIZE, self.val_totals)

    def invs(self, width: int):
        """Apply the gathered INVs of the peers ([N][width], row p: inv_totals[p] INVs) as N
        batches; their ACKs go into ack_slab in the positions of the INVs they answer."""
        self.inv_totals[self.rank:self.rank + 1].zero_()   # (an indexed store from the host would synchronise)
        if self.failed:   # no ACKs from a failed replica
            self.ack_slab[:self.N * width * self.ack_size].view(-1, self.ack_size)[:, 8] = int(L.Bucket.EMPTY)
            return
        if self.count_elems:
            self.elem_totals[0] += self.inv_totals.sum()
        # one launch per peer, in rank order: a peer's slab holds at most one INV per key (one write in
        # flight per key and coordinator), so each applies in one pass (HKV_BATCH_UNIQUE)
        for p in range(self.N):
            if p != self.rank:
                self._inv_launch(p, width)
        if not self.fused_acks:
            check(_L.hkv_wl_marshal_acks_aligned(_ptr(self.inv_recv), _ptr(self.inv_totals), self.N, width, self.op,
                                                 _ptr(self.ack_slab), self.ack_size, self.rank, _s()), "marshal_acks")
            return
        n, na = width * self.op, width * self.ack_size   # this rank's own row: all empty slots
        check(_L.hkv_wl_marshal_acks_aligned(_ptr(self.inv_recv[self.rank * n:]), _ptr(self.inv_totals[self.rank:]), 1,
                                             width, self.op, _ptr(self.ack_slab[self.rank * na:]), self.ack_size,
                                             self.rank, _s()), "marshal_acks")

    def _inv_launch(self, p: int, width: int):
        """peer p's row of inv_recv as one unique-key launch; with fused_acks it also writes the ACKs
        answering them into ack_slab's row p, lined up with the INVs (positions past the row's total
        are never read: the peer's ACK launch stops at its own total)"""
        n = width * self.op
        if self.fused_acks:
            self.kvs.batch(L.BatchType.invs, self.inv_recv[p * n:], 1, width, self.op, self.mb,
                           counts=self.inv_totals[p:p + 1], unique=True,
                           ack_out=self.ack_slab[p * width * self.ack_size:], ack_out_size=self.ack_size)
        else:
            self.kvs.batch(L.BatchType.invs, self.inv_recv[p * n:], 1, width, self.op, self.mb,
                           counts=self.inv_totals[p:p + 1], unique=True)

    # -- per-peer exchanges (ReplicaGroupRound with p2p): each peer's INV slab is sent and received on
    # its own, applied as soon as it is there, and its ACK row goes back right after
    def inv_row_io(self, p: int, width: int):
        """(send, receive) of the INV exchange with peer p: this rank's packed slab, p's row"""
        n = width * self.op
        return self.inv_pack[:n], self.inv_recv[p * n:(p + 1) * n]

    def ack_row_io(self, p: int, width: int):
        """(send, receive) of the ACK exchange with peer p: the answers to p's INVs, p's answers to ours"""
        n = width * self.ack_size
        return self.ack_slab[p * n:(p + 1) * n], self.ack_recv[p * n:(p + 1) * n]

    def invs_begin(self, width: int):
        """Before the per-peer INV launches: this rank's own row carries nothing, and the ACK row it
        'receives' from itself is all empty slots (the ACK phase reads every row)"""
        self.inv_totals[self.rank:self.rank + 1].zero_()
        n, na = width * self.op, width * self.ack_size
        check(_L.hkv_wl_marshal_acks_aligned(_ptr(self.inv_recv[self.rank * n:]), _ptr(self.inv_totals[self.rank:]), 1,
                                             width, self.op, _ptr(self.ack_recv[self.rank * na:]), self.ack_size,
                                             self.rank, _s()), "marshal_acks")
        if self.failed:   # no ACKs from a failed replica
            self.ack_slab[:self.N * na].view(-1, self.ack_size)[:, 8] = int(L.Bucket.EMPTY)

    def invs_peer(self, p: int, width: int, fold: bool):
        """Peer p's INVs (its row of inv_recv, just arrived) as one unique-key launch, then the ACK row
        answering them. fold: p's total rides in the row's spare slot (steady rounds)"""
        n = width * self.op
        if fold:
            a = p * n + (width - 1) * self.op
            self.inv_totals[p:p + 1].copy_(self.inv_recv[a:a + 4].view(torch.int32))
        if self.failed:
            return
        self._inv_launch(p, width)
        if not self.fused_acks:
            check(_L.hkv_wl_marshal_acks_aligned(_ptr(self.inv_recv[p * n:]), _ptr(self.inv_totals[p:]), 1, width,
                                                 self.op, _ptr(self.ack_slab[p * width * self.ack_size:]), self.ack_size,
                                                 self.rank, _s()), "marshal_acks")

    def invs_end(self, width: int):
        if self.count_elems and not self.failed:
            self.elem_totals[0] += self.inv_totals.sum()

    def acks(self, width: int, stride: int):
        """Apply the ACKs returned by the peers (ack_recv [N][width], row p from rank p, lined up
        with inv_pack), regrouped per worker ([W][stride]); the VALs of completed writes, packed
        (val_pack)."""
        N, W, C = self.N, self.W, self.C
        if self.failed:
            self.val_off[W:].zero_()
            return
        if self.unique_acks:
            # row p of ack_recv: peer p's ACKs lined up with inv_pack, worker w's at [inv_off[w], inv_off[w+1]);
            # without the total read back, the launch spans the width and ends at inv_off[W]
            T = self.own_total if self.own_total is not None else width
            if T and self.ack_rows:
                self.kvs.batch(L.BatchType.acks, self.ack_recv, W, T, self.ack_size, self.mb, rw=self.ops,
                               rw_stride_bytes=LOCAL * self.op, offsets=self.inv_off, rw_state=self.states,
                               unique=True, rows=(N, width, self.rank), rw_opcodes=self._rwo())
            elif T:
                for p in range(N):
                    if p != self.rank:
                        self.kvs.batch(L.BatchType.acks, self.ack_recv[p * width * self.ack_size:], W, T, self.ack_size,
                                       self.mb, rw=self.ops, rw_stride_bytes=LOCAL * self.op, offsets=self.inv_off,
                                       rw_state=self.states, unique=True, rw_opcodes=self._rwo())
            if self.count_elems:
                self.elem_totals[1] += (N - 1) * self.inv_off[W]
            check(_L.hkv_wl_collect_vals_rows(_ptr(self.ack_recv), W, N, width, self.ack_size, _ptr(self.val_slab), C,
                                              _ptr(self.val_count), self.rank, _ptr(self.held[1:]), _ptr(self.inv_off),
                                              _s()), "collect_vals_rows")
            check(_L.hkv_wl_pack_rows(_ptr(self.val_slab), _ptr(self.val_count), W, C, L.OP_META_SIZE,
                                      _ptr(self.val_pack), _ptr(self.val_off), _s()), "pack vals")
            return
        check(_L.hkv_wl_regroup_aligned(_ptr(self.ack_recv), N, width, _ptr(self.inv_off), _ptr(self.inv_count), W,
                                        self.ack_size, _ptr(self.ack_batch), stride, _ptr(self.ack_batch_count),
                                        _s()), "regroup")
        if self.count_elems:
            self.elem_totals[1] += self.ack_batch_count.sum()
        self.kvs.batch(L.BatchType.acks, self.ack_batch, W, stride, self.ack_size, self.mb,
                       counts=self.ack_batch_count, rw=self.ops, rw_stride_bytes=LOCAL * self.op, rw_state=self.states,
                       rw_opcodes=self._rwo())
        check(_L.hkv_wl_collect_vals(_ptr(self.ack_batch), _ptr(self.ack_batch_count), W, stride, self.ack_size,
                                     _ptr(self.val_slab), C, _ptr(self.val_count), self.rank,
                                     _ptr(self.held[1:]), None, _s()), "collect_vals")
        check(_L.hkv_wl_pack_rows(_ptr(self.val_slab), _ptr(self.val_count), W, C, L.OP_META_SIZE,
                                  _ptr(self.val_pack), _ptr(self.val_off), _s()), "pack vals")

    def _rwo(self):
        """the opcode mirror the ACK launches complete from"""
        return self.opcodes

    def vals(self, width: int):
        """Apply the gathered VALs of the peers ([N][width], row p: val_totals[p] VALs)."""
        if self.failed:
            return
        self.val_totals[self.rank:self.rank + 1].zero_()
        if self.count_elems:
            self.elem_totals[2] += self.val_totals.sum()
        self.kvs.batch(L.BatchType.vals, self.val_recv, self.N, width, L.OP_META_SIZE, self.mb,
                       counts=self.val_totals)

    def membership_change(self, peer: int | None = None, membership: bytes | None = None):
        """The group drops `peer` (group_membership_update, inline-util.h:26-43), or takes the
        spacetime_group_membership Hades agreed on (`membership`). Every worker runs the
        after-membership-change batch over its ops (hermes_worker.c:526-542); the VALs of the
        writes and replays it completed are packed into val_pack for one more VAL exchange
        (memb_change_* callbacks, hermes_worker.c:163-203). A failed replica, or one whose
        membership did not change (both None), sends none."""
        W, C = self.W, self.C
        if self.failed or (peer is None and membership is None):
            self.val_off[W:].zero_()
            return
        if membership is not None:
            g = membership[1]
            if bin(g).count("1") < self.N // 2:   # inline-util.h:39-42: "Majority is down!"
                raise MajorityLost(f"replica {self.rank}: membership {g:#04x} of {self.N}")
            self.mb = bytes(membership[:3]) + bytes(5)
        else:
            g = self.mb[1] & ~(1 << peer) & 0xFF
            self.mb = L.membership(0, self.rank, alive=g)
        self.kvs.batch(L.BatchType.local_ops_after_membership_change, self.ops, W, LOCAL, self.op, self.mb,
                       state_out=self.states)
        check(_L.hkv_wl_marshal_memb_vals(_ptr(self.ops), W, LOCAL, self.op, _ptr(self.val_slab), C,
                                          _ptr(self.val_count), self.rank, _ptr(self.states), _s()), "marshal_memb_vals")
        check(_L.hkv_wl_pack_rows(_ptr(self.val_slab), _ptr(self.val_count), W, C, L.OP_META_SIZE,
                                  _ptr(self.val_pack), _ptr(self.val_off), _s()), "pack memb vals")

    def val_width(self) -> int:
        """After the VAL totals are gathered (host synchronisation): the largest of them"""
        return max(1, int(self.val_totals.max().item()))

    def fold_counters(self) -> torch.Tensor:
        """counters[0..4] brought up to date (refill leaves per-worker-group partial sums)"""
        check(_L.hkv_wl_fold_counters(_ptr(self.counters), _s()), "fold_counters")
        return self.counters

    def stats(self) -> dict:
        c = self.fold_counters()[:3].cpu().tolist()
        h = self.held.cpu().tolist()
        return {"committed": c[0], "misses": c[1], "writes_completed": c[2], "invs_held": h[0], "vals_dropped": h[1]}


class WidthPlan:
    """The slab width of a replica group's rounds without a host read per round. Every
    `calib_every`-th round (and the first) reads the round's largest INV total back, as before; the
    rounds in between use width = slack x that total + pad and cap each rank's INVs at it (the rest
    are held in PUT_SUCCESS, like credit-held INVs, and go out later). Every rank reads the same
    all-gathered totals, so every rank picks the same width. A round with a failure, Hades or the
    regrouped ACK path always reads back."""

    def __init__(self):
        self.calib_every = int(os.environ.get("HKV_GROUP_CALIB", "16"))
        self.slack = float(os.environ.get("HKV_GROUP_WIDTH_SLACK", "1.25"))
        self.pad = 256
        # the totals ride in one spare slot of each slab (HKV_GROUP_FOLD_TOTALS=0: their own all-gathers)
        self.fold = os.environ.get("HKV_GROUP_FOLD_TOTALS", "1") != "0"
        self.width = None
        self.k = 0

    def steady(self, special: bool) -> bool:
        """whether this round runs at the planned width (call once per round)"""
        k, self.k = self.k, self.k + 1
        return (self.calib_every > 0 and self.width is not None and not special and k % self.calib_every != 0)

    def calibrate(self, width: int, cap: int) -> None:
        """cap: the slab capacity in slots (one is kept for the spare slot)"""
        self.width = min(cap - 1, int(width * self.slack) + self.pad)

    def slab_width(self) -> int:
        """slots per slab in a steady round: the INV cap, plus the spare slot when the totals ride in it"""
        return self.width + 1 if self.fold else self.width


class _HostStaged:
    """a gloo exchange staged through host buffers: wait() ends the exchange and copies the received row
    to the device tensor (on the current stream)"""

    def __init__(self, works, host_rcv, rcv, host_snd):
        self.works, self.host_rcv, self.rcv, self.host_snd = works, host_rcv, rcv, host_snd

    def wait(self):
        for w in self.works:
            w.wait()
        self.rcv.copy_(self.host_rcv)


def _timed(events, name, fn, only=None):
    if events is None or (only is not None and name not in only):
        fn()
        return
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    events.setdefault(name, []).append((a, b))


class ReplicaGroupRound:
    """One replica per process; the exchanges are RCCL collectives (torch.distributed "nccl",
    or any backend whose all_gather_into_tensor / all_to_all_single take these tensors)."""

    LOCAL = LOCAL

    def __init__(self, kvs: HermesKV | None, n_workers: int, zipf: HkvZipf | None, write_permille: int = 200, *,
                 seed: int = 0x5EED, world: int, rank: int, group=None, replica=None, hades: bool = False,
                 comm=None, p2p: bool | None = None, **kw):
        """`replica`: drive an existing ReplicaRound-shaped object instead of building one.
        `hades`: the membership comes from Hades agreement over heartbeats exchanged every round
        (a failed rank is expelled when the survivors agree), instead of a host-driven drop.
        `comm`: an object with gather(out, inp), gather_async(out, inp) -> work (.wait()), a2a(out, inp)
        and p2p(pairs) -> {peer: [work]} to use instead of torch.distributed (tests: ranks as threads of
        one process). `p2p` (default: HKV_GROUP_P2P, on): the INV slabs and ACK rows go peer by peer
        (grouped isend/irecv per peer) instead of one all-gather and one all-to-all, so each peer's INV
        launch waits only for that peer's slab and its ACK row leaves right after it."""
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.comm = comm
        self.p2p = (os.environ.get("HKV_GROUP_P2P", "1") != "0") if p2p is None else p2p
        self.r = replica if replica is not None else ReplicaRound(kvs, n_workers, world, rank, zipf,
                                                                  write_permille, seed=seed, **kw)
        self.hades = hades
        self.world = world
        if hades:
            self.r.hades_start()
            self._hades_bootstrap()
        self.R = world - 1
        self.rstride = self.r.C * self.R
        self.counters = self.r.counters
        self.fold_counters = self.r.fold_counters
        self.plan = WidthPlan() if getattr(self.r, "packed_marshal", False) else None
        self.inv_total = self.r.inv_total
        self.elem_totals = self.r.elem_totals

    @property
    def count_elems(self) -> bool:
        return self.r.count_elems

    @count_elems.setter
    def count_elems(self, v: bool) -> None:
        self.r.count_elems = v

    def _gather(self, out, inp):
        if self.comm is not None:
            return self.comm.gather(out, inp)
        self.dist.all_gather_into_tensor(out, inp, group=self.group)

    def _gather_async(self, out, inp):
        """the same all-gather, returned unwaited: the collective runs on the backend's stream (RCCL's
        own) while torch's stream goes on; work.wait() orders the consumer after it"""
        if self.comm is not None:
            return self.comm.gather_async(out, inp)
        return self.dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)

    def _a2a(self, out, inp):
        if self.comm is not None:
            return self.comm.a2a(out, inp)
        self.dist.all_to_all_single(out, inp, group=self.group)

    def _p2p(self, pairs) -> dict:
        """pairs: (peer, send, receive), peers ascending. One grouped isend/irecv per peer, returned
        unwaited: {peer: [work]}. Every rank walks its peers in ascending order, which is one global
        order of the rank pairs, so the exchanges cannot wait on each other in a cycle."""
        if self.comm is not None:
            return self.comm.p2p(pairs)
        d = self.dist
        if pairs and pairs[0][1].is_cuda and d.get_backend(self.group) != "nccl":
            # gloo (tests: ranks sharing one GPU): its point-to-point ops move host memory and are not
            # ordered on the CUDA stream, so the rows are staged through host buffers
            out = {}
            for p, snd, rcv in pairs:
                sc, rc = snd.cpu(), torch.empty(rcv.shape, dtype=rcv.dtype)
                ws = d.batch_isend_irecv([d.P2POp(d.isend, sc, p, self.group), d.P2POp(d.irecv, rc, p, self.group)])
                out[p] = [_HostStaged(ws, rc, rcv, sc)]
            return out
        return {p: d.batch_isend_irecv([d.P2POp(d.isend, snd, p, self.group), d.P2POp(d.irecv, rcv, p, self.group)])
                for p, snd, rcv in pairs}

    def _views(self, changed: bool) -> bytes:
        """one heartbeat exchange: all ranks' rows gathered (row = sender), this rank polls its
        column. Returns the gathered table."""
        r, n = self.r, self.world
        row = torch.tensor(list(r.hades_row(changed)), dtype=torch.uint8, device=r.ops.device)
        out = torch.empty(n * row.numel(), dtype=torch.uint8, device=r.ops.device)
        self._gather(out, row)
        table = bytes(out.cpu().tolist())
        if not r.failed:
            w = 4 * n + 4
            r.hades.receive_column(b"".join(table[s * w:s * w + 4 * n] for s in range(n)))
        return table

    def _trailers(self, table: bytes) -> list[bytes]:
        w = 4 * self.world + 4
        return [table[s * w + 4 * self.world:(s + 1) * w] for s in range(self.world)]

    def _hades_bootstrap(self, max_periods: int = 16):
        """spin_until_all_nodes_are_in_membership (hermes_worker.c:245-259): heartbeat periods
        until every rank's membership is the whole group"""
        for _ in range(max_periods):
            self.r.hades.update()
            if all(t[1] for t in self._trailers(self._views(False))):
                return
        raise RuntimeError("Hades bootstrap did not reach the full membership")

    def _hades_period(self):
        """update_view_and_issue_hbs + group_membership_update + poll_for_remote_views
        (hermes_worker.c:262-291); when any rank's membership changed, the ranks whose membership
        changed run the after-membership-change batch and every rank joins one VAL exchange"""
        r = self.r
        changed, mb = False, None
        if not r.failed:
            changed, mb, _ = r.hades.update()
        table = self._views(changed)
        if any(t[0] for t in self._trailers(table)):
            r.membership_change(membership=mb if changed else None)
            self._gather(*r.val_total_io())
            w2 = r.val_width()
            self._gather(*r.val_io(w2))
            r.vals(w2)

    def step(self, events: dict | None = None, timed_batches=None, drop: int | None = None):
        """One protocol round. `drop`: that rank fails once its INVs of this round are out (no
        ACKs or VALs from it); the round ends with a membership change and one more VAL
        exchange for the writes it completes -- or, with Hades, the failed rank stops
        heartbeating and the survivors expel it when they agree (two periods later)."""
        r = self.r
        p2p = self.p2p and hasattr(r, "invs_peer")
        steady = self.plan is not None and self.plan.steady(drop is not None or self.hades or not r.unique_acks)
        fold = steady and self.plan.fold
        if steady:   # no host read: the planned width, each rank's INVs capped at it
            width, stride = self.plan.slab_width(), None
            r.own_total = None
            _timed(events, "local", lambda: r.local(cap=self.plan.width), timed_batches)
            if fold and p2p:
                r.inv_io_total(width)          # the total into the slab's spare slot; the rows go peer by peer
            elif fold:
                self._gather(*r.inv_io_total(width))
                r.take_inv_totals(width)
            else:
                self._gather(*r.inv_total_io())
        else:
            _timed(events, "local", r.local, timed_batches)
            self._gather(*r.inv_total_io())
            width, stride = r.round_shape()  # host synchronisation: this round's exact width
            if self.plan is not None:
                self.plan.calibrate(width, r.W * r.C)
        if p2p:
            peers = [p for p in range(self.world) if p != r.rank]
            inv_w = self._p2p([(p, *r.inv_row_io(p, width)) for p in peers])
        elif not fold:
            self._gather(*r.inv_io(width))
        if drop is not None:
            r.peer_failing()
            if drop == r.rank:
                r.fail()
        if p2p:
            ack_w = {}

            def invs():
                r.invs_begin(width)
                for p in peers:   # each peer's launch waits for that peer's slab only
                    for w in inv_w[p]:
                        w.wait()
                    r.invs_peer(p, width, fold)
                    ack_w.update(self._p2p([(p, *r.ack_row_io(p, width))]))
                r.invs_end(width)
            _timed(events, "invs", invs, timed_batches)
            for p in peers:
                for w in ack_w[p]:
                    w.wait()
        else:
            _timed(events, "invs", lambda: r.invs(width), timed_batches)
            self._a2a(*r.ack_io(width))
        _timed(events, "acks", lambda: r.acks(width, stride), timed_batches)
        if not self.hades and drop is None:
            # the VAL exchange overlaps the refill: the refill touches only this replica's op slab and
            # its mirrors, the VAL batch only the table, so their order does not matter
            if fold:
                w_val = self._gather_async(*r.val_io_total(width))
                r.refill()
                w_val.wait()
                r.take_val_totals(width)
            else:
                w_tot = self._gather_async(*r.val_total_io())
                w_val = self._gather_async(*r.val_io(width))
                r.refill()
                w_tot.wait()
                w_val.wait()
            _timed(events, "vals", lambda: r.vals(width), timed_batches)
            return
        self._gather(*r.val_total_io())
        self._gather(*r.val_io(width))
        _timed(events, "vals", lambda: r.vals(width), timed_batches)
        if self.hades:
            self._hades_period()
        elif drop is not None:
            r.membership_change(drop)
            self._gather(*r.val_total_io())
            w2 = r.val_width()
            self._gather(*r.val_io(w2))
            r.vals(w2)
        r.refill()

    def stats(self) -> dict:
        return self.r.stats()


class LoopbackGroup:
    """N replicas driven phase by phase in one process; the collectives are tensor copies with
    exactly the layouts the RCCL driver produces (all-gather: row p = rank p's slab;
    all-to-all: row p of the output = row `rank` of rank p's input)."""

    def __init__(self, rounds: list[ReplicaRound], hades: bool = False, p2p: bool | None = None):
        """p2p (default: HKV_GROUP_P2P, on, as ReplicaGroupRound): INV slabs and ACK rows move peer by
        peer (row copies, `_rows`) and each replica applies its peers' INVs through the per-peer phases
        (invs_begin / invs_peer / invs_end) instead of the all-gather and all-to-all layouts."""
        self.rounds = rounds
        self.N = len(rounds)
        self.hades = hades
        self.p2p = (os.environ.get("HKV_GROUP_P2P", "1") != "0") if p2p is None else p2p
        self.plan = WidthPlan() if all(getattr(r, "packed_marshal", False) for r in rounds) else None
        self.hades_changes = []        # (round, rank, membership) of every agreed change
        self.clock = 0
        if hades:
            for r in rounds:
                r.hades_start()
            full = (1 << self.N) - 1
            for _ in range(16):        # spin_until_all_nodes_are_in_membership
                for r in rounds:
                    r.hades.update()
                exchange_views([r.hades for r in rounds])
                if all(r.hades.state()[0] == full for r in rounds):
                    break
            else:
                raise RuntimeError("Hades bootstrap did not reach the full membership")

    def _hades_period(self):
        rs = self.rounds
        res = {}
        for r in rs:
            if not r.failed:
                res[r.rank] = r.hades.update()
        exchange_views([None if r.failed else r.hades for r in rs])
        if any(ch for ch, _, _ in res.values()):
            for r in rs:
                ch, mb, _ = res.get(r.rank, (False, None, False))
                if ch:
                    self.hades_changes.append((self.clock, r.rank, mb))
                r.membership_change(membership=mb if ch else None)
            self._gather_io([r.val_total_io() for r in rs])
            w2 = max(r.val_width() for r in rs)
            self._gather_io([r.val_io(w2) for r in rs])
            for r in rs:
                r.vals(w2)

    @staticmethod
    def _gather(outs, ins):
        for o in outs:
            torch.cat([x.to(o.device) for x in ins], out=o)

    def _a2a(self, outs, ins):
        N = self.N
        for q, o in enumerate(outs):
            ov = o.view(N, -1)
            for p, x in enumerate(ins):
                ov[p].copy_(x.view(N, -1)[q])

    def _gather_io(self, ios):
        self._gather([o for o, _ in ios], [i for _, i in ios])

    @staticmethod
    def _rows(pairs):
        """pairs: (send, receive) of the per-peer exchanges, each receive the send's copy"""
        for snd, rcv in pairs:
            rcv.copy_(snd)

    def _a2a_io(self, ios):
        self._a2a([o for o, _ in ios], [i for _, i in ios])

    def step(self, drop: int | None = None, observer=None):
        """One round of every replica. observer(phase), when given, runs after each phase has
        finished on every replica ("local", "invs", "acks", "vals", "end"): property checks of
        the group's state between phases (tests)."""
        rs = self.rounds
        seen = observer or (lambda phase: None)
        steady = self.plan is not None and self.plan.steady(drop is not None or self.hades or
                                                            not all(r.unique_acks for r in rs))
        fold = steady and self.plan.fold
        for r in rs:
            if steady:
                r.own_total = None
                r.local(cap=self.plan.width)
            else:
                r.local()
        seen("local")
        if fold and self.p2p:   # the totals ride in the slabs' spare slots, taken per peer (invs_peer)
            width = self.plan.slab_width()
            shapes = [(width, None)] * len(rs)
            for r in rs:
                r.inv_io_total(width)
        elif fold:
            width = self.plan.slab_width()
            shapes = [(width, None)] * len(rs)
            self._gather_io([r.inv_io_total(width) for r in rs])
            for r in rs:
                r.take_inv_totals(width)
        elif steady:
            self._gather_io([r.inv_total_io() for r in rs])
            width = self.plan.slab_width()
            shapes = [(width, None)] * len(rs)
        else:
            self._gather_io([r.inv_total_io() for r in rs])
            shapes = [r.round_shape() for r in rs]
            width = shapes[0][0]                 # the same on every replica (max of the same totals)
            if self.plan is not None:
                self.plan.calibrate(width, rs[0].W * rs[0].C)
        N = self.N
        if self.p2p:   # row p of replica q's INVs: peer p's slab
            self._rows([(rs[p].inv_row_io(q, width)[0], rs[q].inv_row_io(p, width)[1])
                        for q in range(N) for p in range(N) if p != q])
        elif not fold:
            self._gather_io([r.inv_io(width) for r in rs])
        if drop is not None:
            for r in rs:
                r.peer_failing()
            rs[drop].fail()
        if self.p2p:
            for q, r in enumerate(rs):
                r.invs_begin(width)
                for p in range(N):
                    if p != q:
                        r.invs_peer(p, width, fold)
                r.invs_end(width)
        else:
            for r in rs:
                r.invs(width)
        seen("invs")
        if self.p2p:   # row p of replica q's ACKs: peer p's answers to q's INVs
            self._rows([(rs[p].ack_row_io(q, width)[0], rs[q].ack_row_io(p, width)[1])
                        for q in range(N) for p in range(N) if p != q])
        else:
            self._a2a_io([r.ack_io(width) for r in rs])
        for r, (_, stride) in zip(rs, shapes):
            r.acks(width, stride)
        seen("acks")
        if fold:
            self._gather_io([r.val_io_total(width) for r in rs])
            for r in rs:
                r.take_val_totals(width)
        else:
            self._gather_io([r.val_total_io() for r in rs])
            self._gather_io([r.val_io(width) for r in rs])
        for r in rs:
            r.vals(width)
        seen("vals")
        if self.hades:
            self._hades_period()
        elif drop is not None:
            for r in rs:
                r.membership_change(drop)
            self._gather_io([r.val_total_io() for r in rs])
            w2 = rs[0].val_width()
            self._gather_io([r.val_io(w2) for r in rs])
            for r in rs:
                r.vals(w2)
        for r in rs:
            r.refill()
        seen("end")
        self.clock += 1
