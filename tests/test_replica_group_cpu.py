"""The replica-group exchange choreography over torch.distributed, on CPU with gloo
(world_size 2 and 3): ReplicaGroupRound.step() and LoopbackGroup.step() drive a stand-in
replica whose phases tag every slab element with (origin rank, worker, slot) and check, in the
next phase, that each element arrived in the row and slot the kernels assume
(all-gather: row p = rank p's slab; all-to-all: row p = what rank p addressed to this rank).
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
    """Stand-in for ReplicaRound with the same tensors (int64 tags for bytes)."""

    def __init__(self, world, rank, W=5, C=7):
        self.N, self.rank, self.W, self.C = world, rank, W, C
        N = world
        z = lambda *s: torch.zeros(*s, dtype=torch.int64)  # noqa: E731
        zi = lambda *s: torch.zeros(*s, dtype=torch.int32)  # noqa: E731
        self.inv_slab, self.inv_count = z(W * C), zi(W)
        self.inv_recv, self.inv_recv_count = z(N * W * C), zi(N * W)
        self.ack_slab, self.ack_slab_count = z(N * W * C), zi(N * W)
        self.ack_recv, self.ack_recv_count = z(N * W * C), zi(N * W)
        self.val_slab, self.val_count = z(W * C), zi(W)
        self.val_recv, self.val_recv_count = z(N * W * C), zi(N * W)
        self.counters = z(4)
        self.inv_total = z(1)
        self.elem_totals = z(3)
        self.checked = 0
        self.round = 0

    def count(self, origin, w):
        return (origin + w + self.round) % self.C

    def local(self):
        v = self.inv_slab.view(self.W, self.C)
        v.fill_(-1)
        for w in range(self.W):
            n = self.count(self.rank, w)
            self.inv_count[w] = n
            for j in range(n):
                v[w, j] = _tag(1, self.rank, 0, w, j)

    def invs(self):
        N, W, C = self.N, self.W, self.C
        rv, rc = self.inv_recv.view(N, W, C), self.inv_recv_count.view(N, W)
        av, ac = self.ack_slab.view(N, W, C), self.ack_slab_count.view(N, W)
        rc[self.rank].zero_()
        for p in range(N):
            for w in range(W):
                n = int(rc[p, w])
                assert n == (0 if p == self.rank else self.count(p, w))
                for j in range(n):
                    assert int(rv[p, w, j]) == _tag(1, p, 0, w, j)
                    av[p, w, j] = _tag(2, self.rank, p, w, j)   # ACK from me to coordinator p
                    self.checked += 1
                ac[p, w] = n

    def acks(self):
        N, W, C = self.N, self.W, self.C
        rv, rc = self.ack_recv.view(N, W, C), self.ack_recv_count.view(N, W)
        vv = self.val_slab.view(W, C)
        for p in range(N):
            for w in range(W):
                n = int(rc[p, w])
                assert n == (0 if p == self.rank else self.count(self.rank, w))
                for j in range(n):
                    assert int(rv[p, w, j]) == _tag(2, p, self.rank, w, j)
                    self.checked += 1
        for w in range(W):
            n = self.count(self.rank, w)
            self.val_count[w] = n
            for j in range(n):
                vv[w, j] = _tag(3, self.rank, 0, w, j)

    def vals(self):
        N, W, C = self.N, self.W, self.C
        rv, rc = self.val_recv.view(N, W, C), self.val_recv_count.view(N, W)
        rc[self.rank].zero_()
        for p in range(N):
            for w in range(W):
                n = int(rc[p, w])
                for j in range(n):
                    assert int(rv[p, w, j]) == _tag(3, p, 0, w, j)
                    self.checked += 1

    def refill(self):
        self.round += 1


def _worker(rank, world, port, rounds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = TagReplica(world, rank)
        drv = ReplicaGroupRound(None, rep.W, None, world=world, rank=rank, replica=rep)
        for _ in range(rounds):
            drv.step()
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


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_choreography_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rounds = 3
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, checked, err in res:
        assert err is None, f"rank {rank}: {err}"
        assert checked > 0



def test_loopback_matches_choreography():
    world = 3
    reps = [TagReplica(world, r) for r in range(world)]
    grp = LoopbackGroup(reps)
    for _ in range(3):
        grp.step()
    assert all(r.checked > 0 for r in reps)


def test_slots_per_worker():
    assert slots_per_worker(200) == 104          # 50 +- 6.3 writes per 250-op batch
    assert slots_per_worker(0) == 8
    assert slots_per_worker(1000) == 250
    assert 125 < slots_per_worker(500) <= 250
