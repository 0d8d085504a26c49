"""N-replica Hermes groups on one GPU (hermes_amd.replica_group.LoopbackGroup): the phases,
kernels and slab layouts of the RCCL group, with the collectives done by tensor copies.

Two checks per round:
* every batch launch of every replica is mirrored into an oracle table of the same replica
  (same input bytes, same counts, same read_write_ops) and the outputs -- elements,
  read_write_ops and the whole index + log -- must be bit-exact. This is the reference's
  batch functions under real cross-replica traffic: conflicting writes from several
  coordinators, cid tie-breaks, ACK quorums from real peers.
* at the end of each round every key is VALID on every replica with the same timestamp and
  value (Hermes' invariant after all INV/ACK/VAL exchanges of a round have been applied).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402
from oracle.oracle import OracleKVS, gen_keys  # noqa: E402
from tests.helpers import Mirror  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _key_images(g, o, keys):
    """(state, cid, version, value) of every key's log entry, via the oracle's index."""
    log = g.log_bytes()
    e = g.sizes.entry
    rows = []
    for k in keys:
        off = o.lookup(int(k))
        if off is None:
            rows.append(None)
            continue
        ent = log[off:off + e]
        rows.append((int(ent[18]), int(ent[23]), int(ent[24:28].view(np.uint32)[0]), ent[33:33 + g.sizes.st_value].tobytes()))
    return rows


@pytest.mark.parametrize("n_rep,workers,write_pm,rounds,retry,skew,fold,p2p", [
    (2, 24, 300, 4, False, 0, True, True), (3, 16, 400, 4, False, 0, True, True), (4, 8, 500, 3, False, 0, True, True),
    (8, 16, 200, 3, False, 0, True, True), (8, 16, 200, 4, True, 3, True, True), (8, 16, 200, 4, True, 0, True, True),
    (3, 24, 400, 5, True, 3, True, True), (3, 24, 400, 5, True, 3, False, True), (8, 16, 200, 4, True, 3, True, False),
    (3, 24, 400, 5, True, 3, False, False)])
def test_loopback_group_parity_and_convergence(n_rep, workers, write_pm, rounds, retry, skew, fold, p2p, monkeypatch):
    """(8, 16, 200, 3) is BASELINE configs[3]'s group on one GPU: 8 replicas (the width of the
    membership vectors), 20 % writes, Zipf 0.99 -- every phase, kernel and slab layout of the RCCL
    run, with every launch of every replica mirrored into its oracle twin. retry / skew: the
    configuration bench.py --gpus N runs (refill_ops' retry, stalled ops keep their slots, and the
    reference's skew optimisations, config.h:79-80) and the reference's shipped one (skew 0). fold: the
    steady rounds' totals ride in a spare slot of each slab (WidthPlan.fold) or get their own gathers.
    p2p: INV slabs and ACK rows moved peer by peer (ReplicaGroupRound's default), or as the all-gather
    and all-to-all layouts."""
    monkeypatch.setenv("HKV_GROUP_FOLD_TOTALS", "1" if fold else "0")
    monkeypatch.setenv("HKV_GROUP_P2P", "1" if p2p else "0")
    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import LoopbackGroup, ReplicaRound
    from hermes_amd.workload import zipf_params

    n_keys, bkts, cap = 4000, 8192, 1 << 20
    z = zipf_params(n_keys, 0.99)
    reps, mirrors = [], []
    for r in range(n_rep):
        g = HermesKV(n_keys, bkts, cap, machine_id=r, skew=skew)
        o = OracleKVS(bkts, cap, r, skew=skew)
        o.populate(n_keys, L.DEFAULT.kvs_value)
        mirrors.append(Mirror(g, o, f"replica {r}"))
        reps.append(ReplicaRound(g, workers, n_rep, r, z, write_pm, seed=77 + r, trace_len=512, retry_stalled=retry))
    grp = LoopbackGroup(reps)
    keys = gen_keys(n_keys)
    for step in range(rounds):
        grp.step()
        torch.cuda.synchronize()
        imgs = [_key_images(m.g, m.o, keys) for m in mirrors]
        for i, k in enumerate(keys):
            base = imgs[0][i]
            if base is None:
                assert all(im[i] is None for im in imgs)
                continue
            assert base[0] == L.State.VALID, f"round {step}: key #{i} state {base[0]} on replica 0"
            for r in range(1, n_rep):
                assert imgs[r][i] == base, f"round {step}: key #{i} differs between replica 0 and {r}"
    for rep in reps:
        st = rep.stats()
        assert st["invs_held"] == 0 and st["vals_dropped"] == 0, st
        assert st["committed"] > 0 and st["writes_completed"] > 0, st
    # every write of the group was applied somewhere as an INV on every peer
    inv_sent = sum(int(r.inv_total.item()) for r in reps)
    inv_applied = sum(int(r.elem_totals[0].item()) for r in reps)
    assert inv_applied == inv_sent * (n_rep - 1)
    if retry:
        # stalled ops kept their slots (nothing dropped) and the skew flags' outcomes occurred
        stalls = sum(m.codes[(int(L.BatchType.local_ops), "out9", int(c))] for m in mirrors
                     for c in (L.Resp.GET_STALL, L.Resp.PUT_STALL))
        assert stalls > 0
        coalesced = sum(m.codes[(int(L.BatchType.local_ops), "out9", int(L.Resp.PUT_COMPLETE))] for m in mirrors)
        assert (coalesced > 0) == bool(skew & 2), coalesced


@pytest.mark.parametrize("n_rep", [3, 4])
def test_loopback_group_membership_change(n_rep):
    """BASELINE configs[4] in the replica group: the last replica fails in round 1 after its INVs
    are out (no ACKs, no VALs from it). The others drop it from the membership, run the
    after-membership-change batch and exchange the VALs of the writes it completes; later rounds
    replay the writes the failed replica left INVALID. Every launch is mirrored into the oracle;
    after every round the live replicas agree on every key (state, timestamp, value), and a key
    is either VALID or INVALID with the failed replica's write."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import LoopbackGroup, ReplicaRound
    from hermes_amd.workload import zipf_params

    n_keys, bkts, cap = 4000, 8192, 1 << 20
    z = zipf_params(n_keys, 0.99)
    reps, mirrors = [], []
    for r in range(n_rep):
        g = HermesKV(n_keys, bkts, cap, machine_id=r)
        o = OracleKVS(bkts, cap, r)
        o.populate(n_keys, L.DEFAULT.kvs_value)
        mirrors.append(Mirror(g, o, f"replica {r}"))
        reps.append(ReplicaRound(g, 16, n_rep, r, z, 400, seed=55 + r, trace_len=512))
    grp = LoopbackGroup(reps)
    keys = gen_keys(n_keys)
    dead = n_rep - 1
    invalid_after = []
    for step in range(5):
        grp.step(drop=dead if step == 1 else None)
        torch.cuda.synchronize()
        imgs = [_key_images(m.g, m.o, keys) for m in mirrors[:dead]]
        n_inv = 0
        for i in range(len(keys)):
            base = imgs[0][i]
            for r in range(1, dead):
                assert imgs[r][i] == base, f"round {step}: key #{i} differs between replica 0 and {r}"
            if base is None:
                continue
            if step < 1:
                assert base[0] == L.State.VALID
            else:
                assert base[0] in (L.State.VALID, L.State.INVALID), f"round {step}: key #{i} state {base[0]}"
                if base[0] == L.State.INVALID:
                    assert base[1] == dead, f"round {step}: key #{i} INVALID by {base[1]}"
                    n_inv += 1
        invalid_after.append(n_inv)
    assert invalid_after[1] > 0, invalid_after            # the failed replica's last writes
    assert invalid_after[-1] < invalid_after[1], invalid_after   # reads replayed some of them
    for rep in reps[:dead]:
        assert rep.mb[1] == ((1 << n_rep) - 1) & ~(1 << dead)
        st = rep.stats()
        assert st["invs_held"] == 0 and st["vals_dropped"] == 0 and st["writes_completed"] > 0, st


def test_loopback_group_hades_membership():
    """SURVEY 8(f) row 4 on the GPU: the membership comes from Hades agreement (hkv_hades_*) over
    heartbeats exchanged every round. Replica 3 of 4 fails in round 1 after its INVs; the others
    keep issuing writes that wait for its ACK until they agree to expel it (the same round on every
    survivor, within two periods, with a new epoch), run the after-membership-change batch under
    the agreed membership and exchange the VALs of the writes it completes. Every launch is
    mirrored into the oracle; once the change is in, the survivors agree on every key, and a key
    is either VALID or INVALID with the failed replica's write."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import LoopbackGroup, ReplicaRound
    from hermes_amd.workload import zipf_params

    n_rep, n_keys, bkts, cap = 4, 4000, 8192, 1 << 20
    z = zipf_params(n_keys, 0.99)
    reps, mirrors = [], []
    for r in range(n_rep):
        g = HermesKV(n_keys, bkts, cap, machine_id=r)
        o = OracleKVS(bkts, cap, r)
        o.populate(n_keys, L.DEFAULT.kvs_value)
        mirrors.append(Mirror(g, o, f"replica {r}"))
        reps.append(ReplicaRound(g, 16, n_rep, r, z, 400, seed=77 + r, trace_len=512))
    grp = LoopbackGroup(reps, hades=True)
    e0 = reps[0].hades.state()[1]
    keys = gen_keys(n_keys)
    dead = n_rep - 1
    for step in range(6):
        grp.step(drop=dead if step == 1 else None)
        torch.cuda.synchronize()
        changed = [c for c in grp.hades_changes]
        if not changed or changed[0][0] == step:
            continue            # writes may still wait for the failed replica's ACKs
        imgs = [_key_images(m.g, m.o, keys) for m in mirrors[:dead]]
        for i in range(len(keys)):
            base = imgs[0][i]
            for r in range(1, dead):
                assert imgs[r][i] == base, f"round {step}: key #{i} differs between replica 0 and {r}"
            if base is not None:
                assert base[0] in (L.State.VALID, L.State.INVALID), f"round {step}: key #{i} state {base[0]}"
                if base[0] == L.State.INVALID:
                    assert base[1] == dead, f"round {step}: key #{i} INVALID by {base[1]}"
    want = ((1 << n_rep) - 1) & ~(1 << dead)
    ch = grp.hades_changes
    assert sorted(c[1] for c in ch) == list(range(dead)), ch          # every survivor, once
    assert len({c[0] for c in ch}) == 1 and 1 <= ch[0][0] <= 3, ch     # together, within two periods
    for rep in reps[:dead]:
        g, e = rep.hades.state()
        assert g == want and e == e0 + 1 and rep.mb[1] == want and rep.mb[2] == ((~want | (1 << rep.rank)) & 0xFF)
        st = rep.stats()
        assert st["invs_held"] == 0 and st["vals_dropped"] == 0 and st["writes_completed"] > 0, st


class _HConsistent:
    """HConsistent (tla/Hermes.tla:53-56), checked between phases: every two live replicas whose
    copy of a key is VALID hold the same timestamp (version, cid) and value."""

    def __init__(self, mirrors, keys):
        o = mirrors[0].o
        self.mirrors = mirrors
        self.off = np.array([o.lookup(int(k)) for k in keys if o.lookup(int(k)) is not None], np.int64)
        self.checks = 0
        self.valid_pairs = 0

    def __call__(self, live, phase):
        import torch
        torch.cuda.synchronize()
        m0 = self.mirrors[0]
        sv = m0.g.sizes.st_value
        imgs = []
        for r in live:
            log = self.mirrors[r].g.log_bytes()
            ent = log[self.off[:, None] + np.arange(33 + sv)[None, :]]
            imgs.append((ent[:, 18], ent[:, 23], ent[:, 24:28].copy().view(np.uint32)[:, 0], ent[:, 33:33 + sv]))
        valid = np.stack([im[0] == int(L.State.VALID) for im in imgs])
        for a in range(len(live)):
            for b in range(a + 1, len(live)):
                both = valid[a] & valid[b]
                self.valid_pairs += int(both.sum())
                for f in range(3):
                    x, y = imgs[a][f][both], imgs[b][f][both]
                    assert np.array_equal(x, y), f"{phase}: replicas {live[a]} and {live[b]} VALID with different " \
                                                 f"{('cid', 'version', 'value')[f]} on {int((x != y).reshape(len(x), -1).any(1).sum())} keys"
        self.checks += 1


@pytest.mark.parametrize("n_rep,hades", [(4, True), (8, False)])
def test_loopback_group_hconsistent_between_phases(n_rep, hades):
    """The TLA+ invariant HConsistent (tla/Hermes.tla:53-56, THEOREM :263) as a property of the
    device replica group: after every phase of every round -- local batch, INVs, ACKs, VALs, round
    end -- no two live replicas hold a key VALID with different timestamps or values. With Hades,
    replica 3 fails in round 1 and the check also covers the rounds before its expulsion."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import LoopbackGroup, ReplicaRound
    from hermes_amd.workload import zipf_params

    n_keys, bkts, cap = 4000, 8192, 1 << 20
    z = zipf_params(n_keys, 0.99)
    reps, mirrors = [], []
    for r in range(n_rep):
        g = HermesKV(n_keys, bkts, cap, machine_id=r)
        o = OracleKVS(bkts, cap, r)
        o.populate(n_keys, L.DEFAULT.kvs_value)
        mirrors.append(Mirror(g, o, f"replica {r}"))
        reps.append(ReplicaRound(g, 16, n_rep, r, z, 400, seed=91 + r, trace_len=512))
    grp = LoopbackGroup(reps, hades=hades)
    inv = _HConsistent(mirrors, gen_keys(n_keys))
    dead = n_rep - 1 if hades else None
    for step in range(5):
        live = [r.rank for r in reps if not r.failed]
        grp.step(drop=dead if hades and step == 1 else None,
                 observer=lambda phase: inv([r.rank for r in reps if not r.failed], f"round {step} {phase}"))
    assert inv.checks == 5 * 5 and inv.valid_pairs > 0
    if hades:
        assert grp.hades_changes and all(c[2][1] == ((1 << n_rep) - 1) & ~(1 << dead) for c in grp.hades_changes)


def _dist_child(rank, world, port, q, drop=None, retry=False, skew=0):
    import os

    import torch.distributed as dist

    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import ReplicaGroupRound
    from hermes_amd.workload import zipf_params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n_keys = 4000
        g = HermesKV(n_keys, 8192, 1 << 20, machine_id=rank, skew=skew)
        drv = ReplicaGroupRound(g, 16, zipf_params(n_keys, 0.99), 400, seed=99, world=world, rank=rank,
                                trace_len=512, retry_stalled=retry)
        for k in range(4 if drop is not None else 3):
            drv.step(drop=drop if k == 1 else None)
        torch.cuda.synchronize()
        log = g.log_bytes()
        imgs = []
        for k in gen_keys(n_keys):
            off = g.lookup_offset(int(k))
            if off is None:
                imgs.append(None)
                continue
            ent = log[off:off + g.sizes.entry]
            imgs.append((int(ent[18]), int(ent[23]), int(ent[24:28].view(np.uint32)[0]), ent[33:64].tobytes()))
        q.put((rank, imgs, drv.stats(), int(g.take_error_flags()), None))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, None, None, 0, repr(e)))


@pytest.mark.parametrize("world,drop,retry,skew", [(2, None, False, 0), (3, None, False, 0), (3, 2, False, 0),
                                                   (3, None, True, 3)])
def test_dist_group_driver_one_gpu(world, drop, retry, skew):
    """ReplicaGroupRound itself (the driver bench.py runs over RCCL), with `world` processes
    sharing one GPU over gloo (which takes CUDA tensors): every key converges across ranks; also
    under bench.py's configuration (retry + skew flags 3)."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_child, args=(r, world, port, q, drop, retry, skew)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    for rank, imgs, st, flags, err in res:
        assert err is None, f"rank {rank}: {err}"
        assert flags == 0
        assert st["invs_held"] == 0 and st["vals_dropped"] == 0 and st["writes_completed"] > 0, st
    live = [x for x in res if x[0] != drop]     # a failed rank's table no longer follows the group
    base = live[0][1]
    for i, b in enumerate(base):
        if b is None:
            continue
        if drop is None:
            assert b[0] == L.State.VALID, f"key #{i} state {b[0]}"
        else:   # INVALID only where the failed rank's last write was never validated
            assert b[0] == L.State.VALID or (b[0] == L.State.INVALID and b[1] == drop), f"key #{i} {b[:3]}"
        for rank, imgs, *_ in live[1:]:
            assert imgs[i] == b, f"key #{i} differs between rank {live[0][0]} and rank {rank}"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world,config", [(2, "cfg2"), (3, "cfg5")])
def test_bench_multi_rank_over_gloo(world, config):
    """bench.py's N > 1 branch end to end (what the driver runs on 8 GPUs over RCCL): torchrun with
    `world` ranks sharing this GPU over gloo, small tables. cfg5 drops the last rank in the middle
    of the timed steps. The JSON line must report every rank's committed ops, no consistency flags,
    and (cfg5) the shrunken membership."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--steps", "4", "--warmup", "1", "--keys", "30000", "--workers", "48",
           "--config", config, "--dist-backend", "gloo", "--cpu-seconds", "0", "--host-api-seconds", "0"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == world and d["value"] > 0 and d["detail"]["error_flags"] == 0, d
    conv = d["detail"]["convergence"]
    assert conv["live_ranks_agree"], conv          # every live replica holds the same keys
    if config == "cfg2":
        assert conv["not_valid"] == [0] * world, conv
        assert d["config"]["refill"] == "retry" and d["config"]["skew_flags"] == 3
    assert d["config"]["parallelism"] == f"replicas{world}"
    assert d["roofline"]["launches"]["invs"]["elements"] > 0
    if config == "cfg5":
        g = d["detail"]["membership"]["g_membership_after"]
        assert g == ((1 << world) - 1) & ~(1 << (world - 1)), d["detail"]["membership"]


class _ThreadComm:
    """The collectives of `n` ranks run as threads of one process on one GPU: each rank leaves its
    input, and after a barrier copies what it receives on the shared (null) stream -- the producers
    of every input were enqueued before the barrier, so stream order makes the copies correct without
    any host synchronisation."""

    class _Rank:
        def __init__(self, hub, rank):
            self.hub, self.rank = hub, rank

        def gather(self, out, inp):
            h = self.hub
            h.slots[self.rank] = inp
            h.bar.wait()
            ov = out.view(h.n, -1)
            for p, x in enumerate(h.slots):
                ov[p].copy_(x.reshape(-1))
            h.bar.wait()

        def gather_async(self, out, inp):
            self.gather(out, inp)
            return type("Done", (), {"wait": lambda self: None})()

        def a2a(self, out, inp):
            h = self.hub
            h.slots[self.rank] = inp
            h.bar.wait()
            ov = out.view(h.n, -1)
            for p, x in enumerate(h.slots):
                ov[p].copy_(x.view(h.n, -1)[self.rank])
            h.bar.wait()

        def p2p(self, pairs):
            """per-peer exchanges through a mailbox: every send of the call is posted first, then each
            receive waits for its peer's matching send (the k-th message between two ranks) and copies it
            on the shared stream, behind the sender's producers"""
            h = self.hub
            with h.cv:
                for p, snd, _ in pairs:
                    k = h.sent.get((self.rank, p), 0)
                    h.sent[(self.rank, p)] = k + 1
                    h.mail[(self.rank, p, k)] = snd
                    h.p2p_calls += 1
                h.cv.notify_all()
            for p, _, rcv in pairs:
                k = h.got.get((p, self.rank), 0)
                h.got[(p, self.rank)] = k + 1
                with h.cv:
                    if not h.cv.wait_for(lambda: (p, self.rank, k) in h.mail, timeout=60):
                        raise TimeoutError(f"rank {self.rank}: no message {k} from {p}")
                    snd = h.mail.pop((p, self.rank, k))
                rcv.copy_(snd)
            done = type("Done", (), {"wait": lambda self: None})()
            return {p: [done] for p, _, _ in pairs}

    def __init__(self, n):
        import threading
        self.n = n
        self.bar = threading.Barrier(n, timeout=60)
        self.slots = [None] * n
        self.cv = threading.Condition()
        self.mail, self.sent, self.got = {}, {}, {}
        self.p2p_calls = 0

    def rank(self, r):
        return self._Rank(self, r)


@pytest.mark.parametrize("world", [2, 4])
def test_group_rounds_without_host_sync(world):
    """ReplicaGroupRound's steady rounds (bench.py --gpus N's configuration: retry + skew flags 3)
    make no host synchronisation: after the first round calibrates the slab width (WidthPlan), 10
    rounds run under torch.cuda.set_sync_debug_mode("error") -- a .item(), .cpu() or synchronize in
    any of them raises. The ranks are threads of this process with a thread-barrier comm; afterwards
    every rank's table has converged (same state, timestamp and value of every key, all VALID)."""
    import faulthandler
    import os
    import threading

    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import ReplicaGroupRound
    from hermes_amd.workload import zipf_params
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    dump = open(os.path.join(root, "gpurun_out", f"sync_test_stacks_{world}.txt"), "w")
    faulthandler.dump_traceback_later(90, exit=False, file=dump)   # every thread's stack if it hangs
    n_keys = 20000
    hub = _ThreadComm(world)
    z = zipf_params(n_keys, 0.99)
    tables = [HermesKV(n_keys, 1 << 15, 1 << 22, machine_id=r, skew=3) for r in range(world)]
    errs, drivers = [], [None] * world
    phase = threading.Barrier(world + 1, timeout=120)

    def note(msg):
        dump.write(msg + "\n")
        dump.flush()

    def run(r):
        try:
            note(f"rank {r} start")
            drivers[r] = drv = ReplicaGroupRound(tables[r], 64, z, 200, seed=123, world=world, rank=r,
                                                 trace_len=1024, retry_stalled=True, comm=hub.rank(r))
            note(f"rank {r} built")
            drv.step()            # calibrates the width (host read)
            note(f"rank {r} calibrated, width {drv.plan.width}")
            phase.wait()          # the main thread arms the sync check
            phase.wait()
            for k in range(10):
                drv.step()
                note(f"rank {r} step {k}")
            phase.wait()          # the main thread disarms it
        except Exception as e:   # noqa: BLE001 -- reported below
            errs.append((r, repr(e)))
            hub.bar.abort()
            phase.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    try:
        phase.wait()
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode("error")
        phase.wait()
        phase.wait()
    except threading.BrokenBarrierError:
        pass
    finally:
        torch.cuda.set_sync_debug_mode(0)
        for t in ts:
            t.join(timeout=120)
        faulthandler.cancel_dump_traceback_later()
        dump.close()
    assert not errs, errs
    # the per-peer exchanges (ReplicaGroupRound's p2p default): per rank and round, its INV slab to each
    # peer and an ACK row back to each, over the calibrating round and the 10 checked ones
    assert hub.p2p_calls == world * 11 * 2 * (world - 1), hub.p2p_calls
    torch.cuda.synchronize()
    for d in drivers:
        st = d.stats()
        assert st["committed"] > 0 and st["writes_completed"] > 0, st
        assert d.plan is not None and d.plan.width is not None
    assert all(t.take_error_flags() == 0 for t in tables)
    # state, timestamp (cid, version) and value of every key (last_local_write_ts is each replica's own)
    keys = gen_keys(n_keys)
    base = None
    for g in tables:
        log = g.log_bytes()
        img = []
        for k in keys:
            off = g.lookup_offset(int(k))
            img.append(None if off is None else (int(log[off + 18]), log[off + 23:off + 28].tobytes(),
                                                 log[off + 33:off + 64].tobytes()))
        if base is None:
            base = img
            bad = sum(1 for x in img if x is not None and x[0] != L.State.VALID)
            assert bad == 0, f"{bad} keys not VALID"
        else:
            diff = sum(1 for x, y in zip(img, base) if x != y)
            assert diff == 0, f"{diff} keys differ between replicas"
