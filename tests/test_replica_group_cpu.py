"""The replica-group exchange choreography over torch.distributed, on CPU with gloo
(world_size 2 and 3): ReplicaGroupRound.step() and LoopbackGroup.step() drive a stand-in
replica whose phases tag every packed-slab element with (origin rank, worker, slot) and check, in
the next phase, that each element arrived in the row and position the kernels assume
(all-gather at the round's width: row p = rank p's packed slab; all-to-all: row p = what rank p
addressed to this rank, in the positions of the INVs it answers).
The HIP phases themselves run in tests/test_replica_group_gpu.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hermes_amd.replica_group import LoopbackGroup, ReplicaGroupRound, slots_per_worker


def _tag(kind, a, b, w, j):
    return (((kind * 16 + a) * 16 + b) * 4096 + w) * 256 + j


class TagReplica:
    """Stand-in for ReplicaRound with the same exchange interface (int64 tags for elements)."""

    def __init__(self, world, rank, W=5, C=7, drop=None):
        self.N, self.rank, self.W, self.C = world, rank, W, C
        self.drop = drop        # (rank, round): that rank fails in that round after its INVs (checks only)
        self.failed = False
        self.in_memb = False
        N = world
        z = lambda *s: torch.zeros(*s, dtype=torch.int64)  # noqa: E731
        zi = lambda *s: torch.zeros(*s, dtype=torch.int32)  # noqa: E731
        self.inv_pack, self.inv_off, self.inv_totals = z(W * C), zi(W + 1), zi(N)
        self.inv_recv = z(N * W * C)
        self.ack_slab, self.ack_recv = z(N * W * C), z(N * W * C)
        self.val_pack, self.val_off, self.val_totals = z(W * C), zi(W + 1), zi(N)
        self.val_recv = z(N * W * C)
        self.counters = z(4)
        self.fold_counters = lambda: self.counters
        self.inv_total = z(1)
        self.elem_totals = z(3)
        self.count_elems = True
        self.checked = 0
        self.round = 0
        self.pending = 0

    def dead(self, p, after=False):
        """p has failed by this round (after=True: before this round's INVs)"""
        return self.drop is not None and p == self.drop[0] and self.round >= self.drop[1] + int(after)

    def count(self, origin, w):
        if self.in_memb:
            return 0 if self.dead(origin) else (origin + w) % 3
        return 0 if self.dead(origin, after=True) else (origin + w + self.round) % self.C

    def _pack(self, slab, off, kind):
        k = 0
        for w in range(self.W):
            off[w] = k
            for j in range(self.count(self.rank, w)):
                slab[k] = _tag(kind, self.rank, 0, w, j)
                k += 1
        off[self.W] = k

    def _rows(self, origin):
        """(w, j) of origin's packed slab, in order"""
        return [(w, j) for w in range(self.W) for j in range(self.count(origin, w))]

    def local(self):
        # the refill may run before the round's VAL batch (ReplicaGroupRound overlaps it with the
        # VAL exchange): the next round starts here
        self.round += self.pending
        self.pending = 0
        self.in_memb = False
        self._pack(self.inv_pack, self.inv_off, 1)

    def fail(self):
        assert self.drop == (self.rank, self.round)
        self.failed = True

    def peer_failing(self):
        assert self.drop is not None and self.drop[1] == self.round

    def membership_change(self, peer):
        assert self.drop == (peer, self.round)
        self.in_memb = True
        if self.failed:
            self.val_off.zero_()
            return
        self._pack(self.val_pack, self.val_off, 4)

    def val_width(self):
        return max(1, int(self.val_totals.max()))

    def inv_total_io(self):
        return self.inv_totals, self.inv_off[self.W:]

    def inv_io(self, width):
        return self.inv_recv[:self.N * width], self.inv_pack[:width]

    def round_shape(self):
        return max(1, int(self.inv_totals.max())), (self.N - 1) * self.C

    def ack_io(self, width):
        return self.ack_recv[:self.N * width], self.ack_slab[:self.N * width]

    def val_total_io(self):
        return self.val_totals, self.val_off[self.W:]

    def val_io(self, width):
        return self.val_recv[:self.N * width], self.val_pack[:width]

    def invs(self, width):
        self.inv_totals[self.rank] = 0
        rv, av = self.inv_recv[:self.N * width].view(self.N, width), self.ack_slab[:self.N * width].view(self.N, width)
        av.fill_(-1)                                     # ST_EMPTY where no ACK
        if self.failed:
            return
        for p in range(self.N):
            self._inv_row(p, width)

    def _inv_row(self, p, width):
        rv, av = self.inv_recv[:self.N * width].view(self.N, width), self.ack_slab[:self.N * width].view(self.N, width)
        n = int(self.inv_totals[p])
        rows = self._rows(p)
        assert n == (0 if p == self.rank else len(rows)) and len(rows) <= width
        for k in range(n):
            w, j = rows[k]
            assert int(rv[p, k]) == _tag(1, p, 0, w, j)
            av[p, k] = _tag(2, self.rank, p, w, j)   # ACK from me to coordinator p, INV's position
            self.checked += 1

    # the per-peer exchange (ReplicaGroupRound's p2p path): the same rows, one peer at a time
    def inv_row_io(self, p, width):
        return self.inv_pack[:width], self.inv_recv[p * width:(p + 1) * width]

    def ack_row_io(self, p, width):
        return self.ack_slab[p * width:(p + 1) * width], self.ack_recv[p * width:(p + 1) * width]

    def invs_begin(self, width):
        self.inv_totals[self.rank] = 0
        self.ack_slab[:self.N * width].fill_(-1)
        self.ack_recv[self.rank * width:(self.rank + 1) * width].fill_(-1)   # nothing from itself
        self.p2p_peers = []

    def invs_peer(self, p, width, fold):
        assert not fold and p != self.rank and p not in self.p2p_peers
        self.p2p_peers.append(p)
        if not self.failed:
            self._inv_row(p, width)

    def invs_end(self, width):
        assert self.p2p_peers == [p for p in range(self.N) if p != self.rank]
        self.p2p_rounds = getattr(self, "p2p_rounds", 0) + 1

    def acks(self, width, stride):
        rv = self.ack_recv[:self.N * width].view(self.N, width)
        if self.failed:
            self.val_off.zero_()
            return
        mine = self._rows(self.rank)
        for p in range(self.N):
            for k in range(width):
                if p != self.rank and k < len(mine) and not self.dead(p):
                    w, j = mine[k]
                    assert int(rv[p, k]) == _tag(2, p, self.rank, w, j)
                    self.checked += 1
                else:
                    assert int(rv[p, k]) == -1
        self._pack(self.val_pack, self.val_off, 3)

    def vals(self, width):
        if self.failed:
            return
        self.val_totals[self.rank] = 0
        rv = self.val_recv[:self.N * width].view(self.N, width)
        for p in range(self.N):
            n = int(self.val_totals[p])
            rows = self._rows(p)
            assert n == (0 if p == self.rank or self.dead(p) else len(rows))
            for k in range(n):
                w, j = rows[k]
                assert int(rv[p, k]) == _tag(4 if self.in_memb else 3, p, 0, w, j)
                self.checked += 1

    def refill(self):
        self.pending += 1


def _worker(rank, world, port, rounds, q, drop=None, p2p=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = TagReplica(world, rank, drop=drop)
        drv = ReplicaGroupRound(None, rep.W, None, world=world, rank=rank, replica=rep, p2p=p2p)
        for k in range(rounds):
            drv.step(drop=drop[0] if drop is not None and k == drop[1] else None)
        assert getattr(rep, "p2p_rounds", 0) == (rounds if p2p else 0)
        q.put((rank, rep.checked, None))
    except Exception as e:  # surfaced by the parent
        q.put((rank, 0, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,drop,p2p", [(2, None, True), (3, None, True), (3, (2, 1), True), (4, (1, 1), True),
                                            (3, None, False), (4, (1, 1), False)])
def test_rccl_choreography_gloo(world, drop, p2p):
    """drop = (rank, round): that rank fails in that round once its INVs are out; the others
    see no ACKs or VALs from it, the membership-change VAL exchange, and no INVs from it later.
    p2p: the INV slabs and ACK rows exchanged peer by peer (grouped isend/irecv, the default), or
    as one all-gather and one all-to-all."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rounds = 4 if drop else 3
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rounds, q, drop, p2p)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, checked, err in res:
        assert err is None, f"rank {rank}: {err}"
        assert checked > 0


@pytest.mark.parametrize("drop", [None, (2, 1)])
def test_loopback_matches_choreography(drop):
    world = 3
    reps = [TagReplica(world, r, drop=drop) for r in range(world)]
    grp = LoopbackGroup(reps)
    for k in range(4):
        grp.step(drop=drop[0] if drop is not None and k == drop[1] else None)
    assert all(r.checked > 0 for r in reps)


def test_slots_per_worker():
    assert slots_per_worker(200) == 104          # 50 +- 6.3 writes per 250-op batch
    assert slots_per_worker(0) == 8
    assert slots_per_worker(1000) == 250
    assert 125 < slots_per_worker(500) <= 250


class HadesReplica:
    """Stand-in for ReplicaRound in Hades mode: only heartbeats, membership changes and the
    VAL exchange that follows one (every rank joins it; ranks without a change send nothing)."""

    from hermes_amd.replica_group import ReplicaRound as _RR
    hades_start = _RR.hades_start
    hades_row = _RR.hades_row

    def __init__(self, world, rank, W=3):
        self.N, self.rank, self.W, self.C = world, rank, W, 1
        self.failed = False
        z = torch.zeros
        self.counters, self.inv_total, self.elem_totals = z(4), z(1), z(3)
        self.fold_counters = lambda: self.counters
        self.ops = torch.zeros(1, dtype=torch.uint8)
        self.val_off = torch.zeros(W + 1, dtype=torch.int32)
        self.val_totals = torch.zeros(world, dtype=torch.int32)
        self.val_pack = torch.zeros(16, dtype=torch.int64)
        self.val_recv = torch.zeros(world * 16, dtype=torch.int64)
        self.changes = []       # (period, g) of this rank's membership changes
        self.memb_exchanges = 0
        self.period = 0

    def membership_change(self, peer=None, membership=None):
        if self.failed or membership is None:
            self.val_off.zero_()
            return
        self.changes.append((self.period, membership[1]))
        self.val_off[self.W] = 1 + self.rank
        self.val_pack[:1 + self.rank] = 100 + self.rank

    def val_total_io(self):
        return self.val_totals, self.val_off[self.W:]

    def val_width(self):
        return max(1, int(self.val_totals.max()))

    def val_io(self, width):
        return self.val_recv[:self.N * width], self.val_pack[:width]

    def vals(self, width):
        self.memb_exchanges += 1


def _hades_worker(rank, world, port, periods, dead, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = HadesReplica(world, rank)
        drv = ReplicaGroupRound(None, rep.W, None, world=world, rank=rank, replica=rep, hades=True)
        assert rep.hades.state()[0] == (1 << world) - 1       # bootstrap: the whole group
        for p in range(periods):
            rep.period = p
            if rank == dead[0] and p == dead[1]:
                rep.failed = True
            drv._hades_period()
        q.put((rank, rep.changes, rep.memb_exchanges, rep.hades.state(), None))
    except Exception as e:  # surfaced by the parent
        q.put((rank, None, 0, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dead", [(3, (2, 2)), (4, (1, 3))])
def test_hades_membership_over_gloo(world, dead):
    """ReplicaGroupRound(hades=True): heartbeats all-gathered every round, a failed rank stops
    sending them, and the survivors agree on its expulsion in the same period with a new epoch;
    every rank (the failed one with nothing to send) joins the one VAL exchange that follows"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    periods = 8
    procs = [ctx.Process(target=_hades_worker, args=(r, world, port, periods, dead, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, changes, exch, state, err in res:
        assert err is None, f"rank {rank}: {err}"
    want = ((1 << world) - 1) & ~(1 << dead[0])
    live = [x for x in res if x[0] != dead[0]]
    assert all(len(x[1]) == 1 and x[1][0][1] == want for x in live), res
    assert len({x[1][0][0] for x in live}) == 1 and live[0][1][0][0] <= dead[1] + 2, res
    assert len({x[3] for x in live}) == 1                      # same membership and epoch
    assert all(x[2] == 1 for x in res), res                     # one VAL exchange, joined by all


class _NullReplica:
    """Stand-in for ReplicaRound with the exchange interface and no data: ReplicaGroupRound's order of
    exchanges depends on the phase sequence only, not on what the slabs hold."""

    def __init__(self, world, rank, W=4, C=5):
        self.N, self.rank, self.W, self.C = world, rank, W, C
        self.failed = False
        z = lambda n: torch.zeros(n, dtype=torch.int64)  # noqa: E731
        self.inv_pack, self.val_pack = z(W * C), z(W * C)
        self.inv_recv, self.ack_slab, self.ack_recv, self.val_recv = (z(world * W * C) for _ in range(4))
        self.inv_totals, self.val_totals = z(world), z(world)
        self.inv_off, self.val_off = z(W + 1), z(W + 1)
        self.counters, self.inv_total, self.elem_totals = z(4), z(1), z(3)
        self.fold_counters = lambda: self.counters
        self.count_elems = False
        self.packed_marshal = True
        self.unique_acks = True
        self.own_total = None
        self.kind = {}                # data_ptr of a send buffer -> exchange kind

    def _k(self, kind, t):
        self.kind[t.data_ptr()] = kind
        return t

    def local(self, cap=None):
        pass

    def inv_total_io(self):
        return self.inv_totals, self.inv_off[self.W:]

    def round_shape(self):
        return self.W * self.C - 1, (self.N - 1) * self.C

    def inv_io(self, width):
        return self.inv_recv[:self.N * width], self.inv_pack[:width]

    def inv_io_total(self, width):
        return self.inv_io(width)

    def take_inv_totals(self, width):
        pass

    def inv_row_io(self, p, width):
        return self._k("inv", self.inv_pack[:width]), self.inv_recv[p * width:(p + 1) * width]

    def ack_row_io(self, p, width):
        return self._k("ack", self.ack_slab[p * width:(p + 1) * width]), self.ack_recv[p * width:(p + 1) * width]

    def ack_io(self, width):
        return self.ack_recv[:self.N * width], self.ack_slab[:self.N * width]

    def invs(self, width):
        pass

    def invs_begin(self, width):
        pass

    def invs_peer(self, p, width, fold):
        pass

    def invs_end(self, width):
        pass

    def acks(self, width, stride):
        pass

    def val_total_io(self):
        return self.val_totals, self.val_off[self.W:]

    def val_io(self, width):
        return self.val_recv[:self.N * width], self.val_pack[:width]

    def val_io_total(self, width):
        return self.val_io(width)

    def take_val_totals(self, width):
        pass

    def val_width(self):
        return 1

    def vals(self, width):
        pass

    def refill(self):
        pass

    def peer_failing(self):
        pass

    def fail(self):
        self.failed = True

    def membership_change(self, peer=None, membership=None):
        pass


class _RecordingComm:
    """comm= for ReplicaGroupRound that moves nothing and records every exchange in issue order"""

    class _Done:
        def wait(self):
            pass

    def __init__(self, rank, rep, log):
        self.rank, self.rep, self.log = rank, rep, log

    def gather(self, out, inp):
        self.log.append(("gather",))

    def gather_async(self, out, inp):
        self.log.append(("gather",))
        return self._Done()

    def a2a(self, out, inp):
        self.log.append(("a2a",))

    def p2p(self, pairs):
        for p, snd, _ in pairs:
            self.log.append(("p2p", self.rep.kind[snd.data_ptr()], min(self.rank, p), max(self.rank, p)))
        return {p: [self._Done()] for p, _, _ in pairs}


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("drop_round", [None, 3])
def test_p2p_exchanges_follow_one_global_pair_order(world, drop_round):
    """ReplicaGroupRound's per-peer exchanges (batch_isend_irecv with each peer) cannot
    wait on one another in a cycle. Every rank's exchanges, in issue order, are recorded at world sizes
    2-8 over 20 rounds (steady rounds at the planned width and calibrating ones, with and without a
    failure): (1) within a round each rank's sequence of (phase, rank pair) is a subsequence of ONE
    global order -- all INV pairs, then all ACK pairs, pairs ascending -- so the globally first pending
    exchange is at the head of both its ranks' queues; (2) both ranks of a pair issue their exchanges of
    that pair in the same order; (3) every rank issues the same sequence of collectives."""
    from hermes_amd.replica_group import ReplicaGroupRound
    rounds = 20
    logs = {}
    for rank in range(world):
        rep = _NullReplica(world, rank)
        log = []
        drv = ReplicaGroupRound(None, rep.W, None, world=world, rank=rank, replica=rep, p2p=True,
                                comm=_RecordingComm(rank, rep, log))
        per_round = []
        for k in range(rounds):
            start = len(log)
            drop = world - 1 if drop_round is not None and k == drop_round and world > 2 else None
            drv.step(drop=drop)
            per_round.append(log[start:])
        logs[rank] = per_round
    pairs = sorted((a, b) for a in range(world) for b in range(a + 1, world))
    global_order = [("p2p", kind, a, b) for kind in ("inv", "ack") for a, b in pairs]
    pos = {e: i for i, e in enumerate(global_order)}
    for k in range(rounds):
        colls = {r: [e for e in logs[r][k] if e[0] != "p2p"] for r in range(world)}
        assert all(colls[r] == colls[0] for r in range(world)), (k, colls)
        for r in range(world):
            seq = [e for e in logs[r][k] if e[0] == "p2p"]
            idx = [pos[e] for e in seq]
            assert idx == sorted(idx) and len(set(idx)) == len(idx), (k, r, seq)
            # every pair of this rank exchanged once per phase
            assert sorted(e[2:] for e in seq if e[1] == "inv") == [p for p in pairs if r in p]
            assert sorted(e[2:] for e in seq if e[1] == "ack") == [p for p in pairs if r in p]
        for a, b in pairs:
            sa = [e[1] for e in logs[a][k] if e[0] == "p2p" and e[2:] == (a, b)]
            sb = [e[1] for e in logs[b][k] if e[0] == "p2p" and e[2:] == (a, b)]
            assert sa == sb, (k, a, b, sa, sb)
