"""The N=1 bench round (hermes_amd.workload.Round, virtual peers) on the GPU: every batch launch
of a Round over more than kLookupHead (8192) local elements -- so the split lookup, the
absorbing-state shortcut, the INV/ACK rounds and the fallback all run as in bench.py -- is
mirrored into an oracle table and must be bit-exact (elements, read_write_ops, index, log).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402
from oracle.oracle import OracleKVS  # noqa: E402
from tests.helpers import Mirror  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("theta,workers,cfg3,fused,retry", [
    (0.99, 40, False, None, False), (0.0, 40, False, None, False), (0.99, 160, False, None, False),
    (0.99, 40, True, None, False), (0.99, 40, True, False, False), (0.99, 40, True, True, True)])
def test_bench_round_mirrored(theta, workers, cfg3, fused, retry):
    """cfg3: bench.py --config cfg3 (RMWs on, big objects, 25 % PUT + 25 % RMW): the rounds engine,
    op-sized ACKs from the virtual peers, RMW completions. Its refills are planned as patches that the
    local launch's in-place resolve writes (patch_in_resolve), or with fused=False refilled in place
    (hkv_wl_refill_st); retry: refill_ops' policy (planned only when asked, fused=True), so patched and
    kept (stalled) ops share launches."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts = 60_000, 1 << 16
    cap = 1 << 25 if cfg3 else 1 << 23
    steps = 3                         # 10,000 / 40,000 local elements per launch
    g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0)
    o = OracleKVS(bkts, cap, 0, cfg3, cfg3, 4 if cfg3 else 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "bench round")
    r = Round(g, workers, L.membership(3, 0), [1, 2], zipf_params(n_keys, theta), 500 if cfg3 else 200,
              500 if cfg3 else 0, seed=0x5EED, max_steps=8, trace_len=1024, fused_refill=fused, retry_stalled=retry)
    assert r.fused == (fused is not False)   # (cfg3 under retry plans only when asked: fused=True)
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    # local, the peers' INVs (one launch per peer), their ACKs (one rows launch; cfg3: one per peer), VAL
    assert m.launches == steps * (6 if cfg3 else 5)
    st = r.stats()
    assert st["committed"] > 0 and (st["writes_completed"] > 0 or retry), st
    assert g.take_error_flags() == 0
    # the virtual peers write with the keys' live timestamps: some of their INVs beat local writes
    # in flight on the cid tie-break (WRITE -> INVALID_WRITE / INVALID), and the ACK completes them
    assert m.codes[(int(L.BatchType.invs), "out8", int(L.Resp.INV_SUCCESS))] > 0
    if cfg3 and not retry:
        # configs[2]'s conflicts: peers INV-abort local RMWs their own write beats (received in the
        # ACK batch), the local replica INV-aborts peer RMWs below its key's timestamp, and the
        # aborted RMWs end as RMW_ABORT in the next local batch (hermesKV.c:372-394)
        assert m.codes[(int(L.BatchType.acks), "in8", int(L.Resp.OP_INV_ABORT))] > 0, m.codes
        assert m.codes[(int(L.BatchType.invs), "out8", int(L.Resp.OP_INV_ABORT))] > 0, m.codes
        assert m.codes[(int(L.BatchType.local_ops), "out9", int(L.Resp.RMW_ABORT))] > 0, m.codes
        assert st["rmw_aborts"] > 0, st


@pytest.mark.parametrize("cfg3", [False, True])
def test_merged_plan_peer_ts_equals_split(cfg3):
    """hkv_wl_refill_plan_peer_ts (the refill plan and the next round's virtual-peer timestamps in one
    launch at the end of Round.step) against hkv_wl_refill_plan at the end of the step and hkv_wl_peer_ts_at
    at the start of the next: two rounds from the same seed, one forced to the split calls, must hold the
    same ops, patches, cursors, counters, the round's peer slabs and table bytes after every step."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts = 60_000, 1 << 16
    cap = 1 << 25 if cfg3 else 1 << 23
    rounds = []
    for split in (False, True):
        g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0)
        r = Round(g, 40, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 500 if cfg3 else 200,
                  500 if cfg3 else 0, seed=0x5EED, max_steps=8, trace_len=1024)
        assert r.fused
        if split:
            refill = r.refill
            r.refill = lambda first=False, next_round=False, _f=refill: _f(first)
        rounds.append((g, r))
    for step in range(5):
        for _, r in rounds:
            r.step()
        torch.cuda.synchronize()
        (ga, a), (gb, b) = rounds
        # (peer_ts, the RMW peers' write per entry and peer, is stamped a round ahead by the merged launch
        # like the slabs below; the ops and the table show its use)
        for name in ("ops", "patch", "cursor", "states", "opcodes"):
            x, y = getattr(a, name), getattr(b, name)
            assert (x is None and y is None) or torch.equal(x, y), f"step {step}: {name} differs"
        # the peers' INV / VAL slabs of the round just run (the merged launch has already stamped the next
        # round's; the split calls stamp them when that round starts)
        n = len(a.remote_packed)
        k = step % n
        if n > 1:
            for j, (x, y) in enumerate(zip(a.remote_packed[k], b.remote_packed[k])):
                if isinstance(x, torch.Tensor):
                    assert torch.equal(x, y), f"step {step}: remote slab {k}.{j} differs"
        assert np.array_equal(ga.index_bytes(), gb.index_bytes()) and np.array_equal(ga.log_bytes(), gb.log_bytes())
    assert rounds[0][1].stats() == rounds[1][1].stats() and rounds[0][1].stats()["committed"] > 0
    for g, _ in rounds:
        assert g.take_error_flags() == 0


@pytest.mark.parametrize("skew,rmw", [(0, True), (3, True), (3, False)])
def test_big_patches_applied_in_resolve(skew, rmw):
    """Refill patches of 312-B ops applied by the local launch itself (hkv_batch.hip patch_in_resolve:
    k_lookup reads each patch beside the op header, k_resolve0_direct runs the exec functions on a patched
    copy and writes the op once), against the oracle on the ops as the patches make them: every patch
    flavour of include/hermeskv.h (GETs, PUTs, RMWs; a value fill byte or none, also on a GET; the ts
    reset), invalid patches beside valid ones, patched elements past their batch's count (patched, not
    run), random bytes in the pad after each value (kept), skewed keys over several launches. With RMWs off
    an element after its key's first mutation resolves against S_1, whose kind (WRITE with version + 2, or
    REPLAY) the skew flags take from that first element's opcode -- its patch's, as the op is not yet written."""
    from hermes_amd.kvs import HermesKV
    from oracle.oracle import gen_keys
    from tests import gen
    n_keys, bkts, cap = 3000, 512, 1 << 21
    g = HermesKV(n_keys, bkts, cap, machine_id=1, rmw=rmw, big_objects=True, extra_cache_lines=4, skew=skew)
    o = OracleKVS(bkts, cap, 1, rmw, True, 4, skew=skew)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "big patches")
    sz = g.sizes
    rng = np.random.default_rng(4242 + skew)
    keys = gen_keys(n_keys)
    tsp = gen.TsPool(rng)
    mb = L.membership(3, 1)
    W, S = 40, 250                       # 10,000 elements: the multi-kernel engine
    vend = L.OP_VALUE_OFF + sz.st_value
    assert 0 < sz.op - vend <= 8
    hits = 0
    for rnd in range(4):
        pool = gen.key_pool(rng, keys, hot=40 if rnd % 2 else 400)
        loc = gen.local_ops(rng, pool, W * S, sz, rmw, tsp)
        raw = loc.view(np.uint8).reshape(W * S, sz.op)
        raw[:, vend:] = rng.integers(0, 256, size=(W * S, sz.op - vend))
        p = np.zeros((W * S, 16), np.uint8)
        valid = rng.random(W * S) < 0.7
        pk = gen.draw_keys(rng, pool, W * S)
        p[:, 0:8] = pk.view(np.uint8).reshape(-1, 8)
        p[:, 8] = rng.choice([int(L.Op.GET), int(L.Op.PUT), int(L.Op.RMW)], size=W * S,
                             p=[0.5, 0.3, 0.2] if rmw else [0.6, 0.4, 0.0])
        p[:, 9] = rng.integers(0, 256, size=W * S)
        p[:, 10:12] = rng.integers(0, 256, size=(W * S, 2))
        fill = rng.integers(1, 256, size=W * S)
        getp = p[:, 8] == int(L.Op.GET)
        p[:, 12] = np.where(getp, np.where(rng.random(W * S) < 0.1, fill, 0),
                            np.where(rng.random(W * S) < 0.9, fill, 0))
        p[:, 13] = rng.random(W * S) < 0.3
        p[:, 14] = valid
        p[~valid, 8:14] = rng.integers(0, 256, size=(int((~valid).sum()), 6))   # ignored bytes of invalid patches
        counts = rng.integers(S // 2, S + 1, size=W).astype(np.int32)
        ops = torch.from_numpy(raw.reshape(-1).copy()).cuda()
        patch = torch.from_numpy(p.reshape(-1)).cuda()
        state_out = torch.zeros(W * S, dtype=torch.uint8, device="cuda")
        m.batch(L.BatchType.local_ops, ops, W, S, sz.op, mb, counts=torch.from_numpy(counts).cuda(), patch=patch,
                state_out=state_out)
        got = ops.cpu().numpy().reshape(W * S, sz.op)
        hits += int(np.isin(got[:, 9], [int(L.Resp.GET_COMPLETE), int(L.Resp.PUT_SUCCESS),
                                         int(L.Resp.RMW_SUCCESS)]).sum())
        # a patched element past its batch's count is patched, not run
        past = (np.arange(S)[None, :] >= counts[:, None]).reshape(-1) & valid
        assert past.any() and (got[past, 9] == int(L.Bucket.NEW)).all()
    assert hits > 1000 and m.launches == 4


@pytest.mark.parametrize("skew,hot", [(0, False), (3, False), (3, True)])
def test_retry_round_mirrored(skew, hot):
    """The bench round under refill_ops' retry policy (stalled ops keep their slots), alone and with
    the reference's skew optimisations (skew_flags 3: read completion and write coalescing, GET
    timestamps reset by the refill) and hot-request coalescing: every launch mirrored into an
    oracle table with the same flags, bit-exact; with the flags, local batches complete stalled
    GETs and PUTs (PUT_COMPLETE straight out of a local batch exists only through coalescing)."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 23
    g = HermesKV(n_keys, bkts, cap, machine_id=0, skew=skew)
    o = OracleKVS(bkts, cap, 0, skew=skew)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "retry round")
    r = Round(g, 40, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 200, seed=0x5EED, max_steps=8,
              trace_len=1024, retry_stalled=True, coalesce_hot=hot)
    steps = 5
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    assert m.launches == steps * 5      # local, the peers' INVs (one launch each), their ACKs (one rows launch), VAL
    st = r.stats()
    assert st["committed"] > 0 and st["dropped"] == 0, st
    # the ACK rows launch made the VALs of the writes it completed (checked against val_callbacks per launch)
    assert (m.codes[(int(L.BatchType.acks), "vals_sent", 0)] > 0) == r.fused_vals, m.codes
    assert g.take_error_flags() == 0
    coalesced = m.codes[(int(L.BatchType.local_ops), "out9", int(L.Resp.PUT_COMPLETE))]
    assert (coalesced > 0) == bool(skew & 2), m.codes
    if hot:   # some committed ops were coalesced requests
        assert st["committed"] > 0
    else:
        # the per-outcome breakdown bench.py reports (CommitAudit): it adds up to the refill's own
        # commit count, and the value-less GETs / coalesced PUTs exist only under their skew flag
        a = r.audit_rounds(3)
        assert a["consistent"], a
        pr = a["per_round"]
        assert pr["get_value"] > 0 and pr["put_own"] > 0, a
        if not skew & 1:
            assert pr["get_no_value"] == 0, a
        if not skew & 2:
            assert pr["put_coalesced_recorded"] + pr["put_coalesced_inherited"] + pr["put_coalesced_unknown"] == 0, a
        if skew == 3:
            assert pr["get_no_value"] + pr["put_coalesced_recorded"] + pr["put_coalesced_inherited"] > 0, a
        assert g.take_error_flags() == 0


class _DeviceBytes:
    """A device byte range as a torch tensor, without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


@pytest.mark.parametrize("cfg3", [False, True])
def test_full_size_round_invariants(cfg3):
    """BASELINE configs[1] at full size (100M keys, 16384 virtual workers: the bench's round), and
    configs[2] (the same keys in 320-B entries, RMWs, fresh batches: its refills planned as patches that
    the local launch writes): properties that hold at any size. After every round each key is VALID again
    (every local write was ACKed by both virtual peers and completed, every INV's VAL applied, no
    membership change), no INV was held back, writes completed, and the engine's consistency flags are
    clear."""
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params
    n_keys = 100_000_000
    sizes = L.Sizes(True, 4) if cfg3 else L.DEFAULT
    bkts, cap = sized_geometry(n_keys, sizes)
    g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0)
    r = Round(g, 16384, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 500 if cfg3 else 200,
              500 if cfg3 else 0, seed=0x5EED, max_steps=4)
    assert r.fused
    entry = g.sizes.entry
    assert g.log_head == n_keys * entry       # populate wrote entries 0..n-1 back to back
    log = torch.as_tensor(_DeviceBytes(g.device_log(), n_keys * entry), device="cuda")
    state = log.view(n_keys, entry)[:, 18]    # object meta byte 0: state
    assert int((state != int(L.State.VALID)).sum()) == 0
    for step in range(3):
        r.step()
        torch.cuda.synchronize()
        bad = int((state != int(L.State.VALID)).sum())
        assert bad == 0, f"round {step}: {bad} keys not VALID"
    st = r.stats()
    assert st["invs_held"] == 0 and st["committed"] > 4_000_000 and st["writes_completed"] > 600_000, st
    assert g.take_error_flags() == 0


def _round_launches(r, k: int, sent: int, alive: int, changes: int) -> int:
    """Launches one Round.step makes: the local batch, one INV launch per live peer with INVs in round
    index k, the ACK rows launch (when any peer answers and the round sent INVs), the VAL batch, and one
    after-membership-change batch per membership change in the round"""
    n_inv = sum(1 for _, n, _ in r.remote_packed[k][5][:sent] if n)
    acks = (1 if (not r.fit or r.inv_round) else 0) if alive else 0
    return 1 + n_inv + acks + 1 + changes


@pytest.mark.parametrize("machines", [3, 8])
def test_membership_change_round_mirrored(machines):
    """BASELINE configs[4] on one GPU: the last virtual peer fails in round 2 after sending its
    INVs (no ACKs, no VALs from it), the group drops it and every worker runs the
    after-membership-change batch (hermes_worker.c:526-542); later rounds replay the writes it
    left INVALID. Every launch, including the after-change batch, is mirrored into the oracle."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 23
    g = HermesKV(n_keys, bkts, cap, machine_id=0)
    o = OracleKVS(bkts, cap, 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "membership round")
    peers = list(range(1, machines))
    r = Round(g, 40, L.membership(machines, 0), peers, zipf_params(n_keys, 0.99), 200, seed=0x5EED,
              max_steps=8, trace_len=1024, remote_per_peer=20)
    op = g.sizes.op
    replays = []
    marshal = r.marshal_invs

    def counting_marshal():
        replays.append(int((r.ops.view(-1, op)[:, 9] == int(L.Resp.REPLAY_SUCCESS)).sum()))
        marshal()
    r.marshal_invs = counting_marshal
    for step in range(6):
        drop = peers[-1] if step == 2 else None
        k, sent, before = r.clock % len(r.remote_inv), r.alive, m.launches
        r.step(drop=drop)
        torch.cuda.synchronize()
        want = _round_launches(r, k, sent, sent - (drop is not None), int(drop is not None))
        assert m.launches - before == want, (step, m.launches - before, want)
    assert r.mb[1] == ((1 << machines) - 1) & ~(1 << peers[-1]) and r.alive == machines - 2
    st = r.stats()
    assert st["committed"] > 0 and st["writes_completed"] > 0, st
    assert sum(replays[3:]) > 0, replays
    assert g.take_error_flags() == 0


@pytest.mark.parametrize("machines", [3, 8])
def test_hades_membership_round_mirrored(machines):
    """SURVEY 8(f) row 4 on one GPU: this replica and its virtual peers run the Hades agreement
    (hkv_hades_*) over heartbeats every round. The last peer fails in round 2 after its INVs; the
    writes waiting for its ACK stay in flight until the survivors agree to expel it (every live
    node in the same period, within two periods, with a new epoch); then the after-membership-change
    batch runs under the agreed membership and later reads replay what it left INVALID. Every
    launch is mirrored into the oracle."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 23
    g = HermesKV(n_keys, bkts, cap, machine_id=0)
    o = OracleKVS(bkts, cap, 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "hades round")
    peers = list(range(1, machines))
    r = Round(g, 40, L.membership(machines, 0), peers, zipf_params(n_keys, 0.99), 200, seed=0x5EED,
              max_steps=10, trace_len=1024, remote_per_peer=20, hades=True)
    e0 = r.hades[0].state()[1]
    op = g.sizes.op
    replays = []
    marshal = r.marshal_invs

    def counting_marshal():
        replays.append(int((r.ops.view(-1, op)[:, 9] == int(L.Resp.REPLAY_SUCCESS)).sum()))
        marshal()
    r.marshal_invs = counting_marshal
    steps = 8
    for step in range(steps):
        drop = peers[-1] if step == 2 else None
        k, sent, before, nch = r.clock % len(r.remote_inv), r.alive, m.launches, len(r.hades_changes)
        r.step(drop=drop)
        torch.cuda.synchronize()
        want = _round_launches(r, k, sent, sent - (drop is not None), len(r.hades_changes) - nch)
        assert m.launches - before == want, (step, m.launches - before, want)
    want = ((1 << machines) - 1) & ~(1 << peers[-1])
    assert len(r.hades_changes) == 1 and r.hades_changes[0][1] == want, r.hades_changes
    at = r.hades_changes[0][0]
    assert 2 <= at <= 4, r.hades_changes
    assert r.mb[1] == want and r.mb[2] == (~want | 1) & 0xFF
    for i, h in r.hades.items():
        if i != peers[-1]:
            assert h.state() == (want, e0 + 1), (i, h.state())
    st = r.stats()
    assert st["committed"] > 0 and st["writes_completed"] > 0, st
    assert sum(replays[at + 1:]) > 0, replays
    assert g.take_error_flags() == 0


def test_rmw_semantics_invariant_cfg3():
    """HRSemanticsRMW (tla/HermesRMWs.tla:31-37) on the RMW-heavy round: across every round, no
    two RMWs committed on a key with the same version (and different tie-breakers), and no RMW
    committed with the version of a committed write or the one just below it. Commits are read
    from the op buffers before each refill (RMW_COMPLETE / PUT_COMPLETE with the op's timestamp)."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 25
    g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=True, big_objects=True, extra_cache_lines=4)
    r = Round(g, 40, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 500, 500, seed=0x5EED, max_steps=10,
              trace_len=1024)
    op = g.sizes.op
    rmws, writes = {}, {}
    refill = r.refill

    def recording_refill(*args, **kw):
        ops = r.ops.view(-1, op).cpu().numpy()
        st = ops[:, 9]
        for kind, code in (("rmw", int(L.Resp.RMW_COMPLETE)), ("put", int(L.Resp.PUT_COMPLETE))):
            for x in ops[st == code]:
                key = int(x[:8].view(np.uint64)[0])
                ver, cid = int(x[12:16].view(np.uint32)[0]), int(x[11])
                (rmws if kind == "rmw" else writes).setdefault(key, []).append((ver, cid))
        refill(*args, **kw)
    r.refill = recording_refill
    for _ in range(8):
        r.step()
    torch.cuda.synchronize()
    n_rmw = sum(len(v) for v in rmws.values())
    assert n_rmw > 0 and sum(len(v) for v in writes.values()) > 0
    for key, rv in rmws.items():
        wv = {v for v, _ in writes.get(key, [])}
        seen = {}
        for ver, cid in rv:
            assert ver not in wv and ver + 1 not in wv, (key, ver, sorted(wv))
            assert seen.setdefault(ver, cid) == cid, (key, ver)
    assert g.take_error_flags() == 0


@pytest.mark.parametrize("credits,cfg3", [(3, False), (6, True)])
def test_val_credits_round_mirrored(credits, cfg3):
    """VALs under credits and the outstanding-VAL gate (hermes_worker.c:479-503).
    With a few VAL credits per round, workers carry VALs, stop polling their ACKs while they do
    (the ACKs wait in their queue, holding INV credits) and send the carried VALs first. Every
    batch launch is mirrored into the oracle; every round's VALs are checked against a model of
    the queues (carried first, then the applied queue's LAST_ACK_SUCCESS elements in queue order,
    at most `credits` sent), and every VAL produced is sent exactly once or still carried."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts = 60_000, 1 << 16
    cap = 1 << 25 if cfg3 else 1 << 23
    g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0)
    o = OracleKVS(bkts, cap, 0, cfg3, cfg3, 4 if cfg3 else 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "val credits round")
    W = 40
    r = Round(g, W, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 500 if cfg3 else 200,
              500 if cfg3 else 0, seed=0x5EED, max_steps=8, trace_len=1024, val_credits=credits)
    asz, q = r.ack_size, r.ack_stride
    seen = {"gated": 0, "carried_rounds": 0, "produced": 0}
    vals_credit = r.vals_under_credits

    def checked_vals():
        torch.cuda.synchronize()
        carried = r.vq.view(W, r.C, 16).cpu().numpy().copy()
        vq_n = r.vq_n.cpu().numpy().copy()
        acnt = r.ack_count.cpu().numpy().copy()
        aq = r.acks.view(W, q, asz).cpu().numpy().copy()
        vals_credit()
        torch.cuda.synchronize()
        out = r.val_out.view(W, -1, 16).cpu().numpy()
        vc, vq_n2 = r.val_count.cpu().numpy(), r.vq_n.cpu().numpy()
        vq2, aq_n2 = r.vq.view(W, r.C, 16).cpu().numpy(), r.aq_n.cpu().numpy()
        for w in range(W):
            src = [carried[w, j] for j in range(vq_n[w])]
            assert acnt[w] == 0 or vq_n[w] == 0, "ACKs applied while VALs were outstanding"
            skip = (int(L.Resp.ACK_SUCCESS), int(L.Op.MEMBERSHIP_CHANGE), int(L.Bucket.EMPTY))
            new = [j for j in range(acnt[w]) if aq[w, j, 8] not in skip]   # val_skip_or_get_sender_id
            seen["produced"] += len(new)
            for j in new:
                v = aq[w, j, :16].copy()
                v[8], v[9] = int(L.Op.VAL), 0
                src.append(v)
            send = min(len(src), credits)
            assert vc[w] == send and vq_n2[w] == len(src) - send, (w, vc[w], vq_n2[w], len(src))
            for j in range(send):
                assert np.array_equal(out[w, j], src[j]), (w, j)
            for j in range(len(src) - send):
                assert np.array_equal(vq2[w, j], src[send + j]), (w, j)
            if acnt[w]:
                assert aq_n2[w] == 0
            seen["gated"] += int(vq_n[w] > 0)
        seen["carried_rounds"] += int((vq_n2 > 0).any())
    r.vals_under_credits = checked_vals
    steps = 6
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    # local, the peers' INVs (one launch per peer), ACK (one packed launch), VAL
    assert m.launches == steps * 5
    st = r.stats()
    assert g.take_error_flags() == 0
    assert seen["gated"] > 0 and seen["carried_rounds"] > 0, seen
    assert st["gated_worker_rounds"] == seen["gated"], (st, seen)
    assert st["vals_sent"] + st["vals_carried"] == seen["produced"], (st, seen)
    assert st["val_overflow"] == 0 and st["writes_completed"] > 0, st
    if not cfg3:   # queued ACKs held INV credits back (cfg3's slots rarely bind: most ops stall on RMW conflicts)
        assert st["invs_held"] > 0, st
    assert m.codes[(int(L.BatchType.acks), "out8", int(L.Resp.LAST_ACK_SUCCESS))] == seen["produced"]


# PUT/RMW/REPLAY_SUCCESS, IN_PROGRESS_PUT/RMW/REPLAY, PUT/RMW/REPLAY_COMPLETE_SEND_VALS, membership
# change: a fresh-batch refill keeps these (their keys point at the slot through op_buffer_index)
IN_FLIGHT = (122, 135, 123, 143, 148, 144, 133, 149, 147, 118)


def _refill_ref(ops, W, S, osz, st_value, shift, tkey, top, tlen, cursor, mid, first, flags, tid=None, hot=None):
    """refill_ops (inline-util.h:149-303) as hkv_wl_refill applies it, in numpy: per worker, walk
    the op buffer in order; a completed op (every op on the first pass; with REFILL_ALL also a
    stalled one) is counted (committed ops: no_coales of them under hot-request coalescing, else
    one) and takes the next trace command. READ_TS_RESET zeroes a new GET's timestamp
    (:268-272). COALESCE_HOT (:237-257): while the next command is a GET/PUT on an id below 100
    and the worker's pointer for that id and opcode class names a slot whose opcode equals the
    command's, that slot's no_coales grows and the command is consumed; the slot then inserted
    becomes the pointer. hot: [W][200] slot indexes (255 = NULL), updated in place."""
    ops = ops.copy().reshape(W, S, osz)
    cursor = cursor.copy()
    cnt = np.zeros(5, dtype=np.int64)
    done_states = (130, 128, 138, 137, 119, 121)
    refill_all, ts_reset, coalesce = flags & 1, flags & 2, flags & 4

    def no_coales(o):
        return (int(o[16]) | int(o[17]) << 8) >> 1

    for w in range(W):
        it = 0
        for i in range(S):
            o = ops[w, i]
            st = int(o[9])
            complete = st in done_states
            drop = bool(refill_all) and not first and not complete and st not in IN_FLIGHT
            if not first and complete:
                cnt[0] += (no_coales(o) if coalesce else 1) if st not in (130, 138) else 0
                cnt[1] += st == 130
                cnt[2] += st == 128
            cnt[3] += drop
            cnt[4] += (not first) and st == 138
            if not (first or complete or drop):
                continue
            if not first:
                o[8] = o[9] = 140          # reset op bucket: opcode = state = ST_EMPTY
            if coalesce and int(top[w * tlen + (int(cursor[w]) + it) % tlen]) != 113:
                while True:
                    t = w * tlen + (int(cursor[w]) + it) % tlen
                    kid, oc = int(tid[t]), int(top[t])
                    col = 0 if oc == 111 else 100
                    p = int(hot[w, col + kid]) if kid < 100 else 255
                    if p != 255 and int(ops[w, p, 8]) == oc:
                        v = int(ops[w, p, 16]) | int(ops[w, p, 17]) << 8
                        v = (v & 1) | ((((v >> 1) + 1) & 0x7FFF) << 1)
                        ops[w, p, 16], ops[w, p, 17] = v & 0xFF, v >> 8
                        it += 1
                    else:
                        break
                if kid < 100:
                    hot[w, col + kid] = i
            t = w * tlen + (int(cursor[w]) + it) % tlen
            it += 1
            oc = int(top[t])
            o[0:8] = np.frombuffer(np.uint64(tkey[t]).tobytes(), dtype=np.uint8)
            o[8], o[9] = oc, 141
            o[10] = 0 if oc == 111 else (st_value >> shift) & 0xFF
            if oc == 111 and ts_reset:
                o[11:16] = 0
            fl = (1 if oc == 113 else 0) | (0 if first else 2)
            o[16], o[17] = fl & 0xFF, fl >> 8
            if oc != 111:
                o[18:18 + st_value] = ord("a") + mid
        cursor[w] = (int(cursor[w]) + it) % tlen
    return ops.reshape(-1), cursor, cnt


@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("flags", [0, 1, 2, 4, 6, 5])
def test_refill_kernel_matches_numpy(big, flags):
    """hkv_wl_refill (LDS-staged for 56-B ops, in place for 312-B ops, the sequential walk for
    hot-request coalescing) against a numpy restatement: slab bytes, trace cursors, the
    committed / miss / PUT_COMPLETE / dropped counters and the hot-key pointers. flags: 1 fresh
    batches (ops in flight keep their slots), 2 GET timestamps reset, 4 hot-request coalescing
    (56-B ops only), several passes so pointers carry over."""
    from hermes_amd import workload as WL
    if big and flags & 4:
        pytest.skip("hot-request coalescing stages the slab in LDS: 56-B ops")
    sz = L.BIG if big else L.DEFAULT
    W, S, osz, tlen, mid = 37, 250, sz.op, 300, 2
    rng = np.random.default_rng(11 + big + 2 * flags)
    states = np.array([130, 128, 138, 137, 119, 121, 131, 132, 136, 140, 141, *IN_FLIGHT], dtype=np.uint8)
    ops = rng.integers(0, 256, size=W * S * osz, dtype=np.uint8)
    ops.reshape(W, S, osz)[:, :, 9] = rng.choice(states, size=(W, S))
    # opcodes as the refill leaves them, so pointers find live GET/PUT slots
    ops.reshape(W, S, osz)[:, :, 8] = rng.choice(np.array([111, 112, 113], dtype=np.uint8), size=(W, S))
    tkey = rng.integers(0, 2**63, size=W * tlen, dtype=np.int64)
    top = rng.choice(np.array([111, 111, 111, 112, 113], dtype=np.uint8), size=W * tlen)
    tid = np.where(rng.random(W * tlen) < 0.6, rng.integers(0, 12, W * tlen),
                   rng.integers(0, 400, W * tlen)).astype(np.int32)
    cursor = rng.integers(0, tlen, size=W, dtype=np.int32)
    hot = np.full((W, 200), 255, np.uint8)
    d_ops = torch.from_numpy(ops.copy()).cuda()
    d_tkey, d_top = torch.from_numpy(tkey).cuda(), torch.from_numpy(top).cuda()
    d_tid = torch.from_numpy(tid).cuda()
    d_cur = torch.from_numpy(cursor.copy()).cuda()
    d_cnt = torch.zeros(4096, dtype=torch.int64, device="cuda")
    d_opc = torch.zeros(W * S, dtype=torch.uint8, device="cuda")
    d_hot = torch.from_numpy(hot.reshape(-1).copy()).cuda()
    passes = 3 if flags & 4 else 1
    exp_ops, exp_cur = ops, cursor
    exp_cnt = np.zeros(5, np.int64)
    for p in range(passes):
        if p:   # between passes: some ops complete, some stall, as a round would leave them
            exp_ops = exp_ops.copy()
            exp_ops.reshape(W, S, osz)[:, :, 9] = rng.choice(states, size=(W, S))
            d_ops.copy_(torch.from_numpy(exp_ops))
        exp_ops, exp_cur, c = _refill_ref(exp_ops, W, S, osz, sz.st_value, sz.shift, tkey.view(np.uint64), top, tlen,
                                          exp_cur, mid, False, flags, tid, hot)
        exp_cnt += c
        WL.check(WL._L.hkv_wl_refill(WL._ptr(d_ops), W, S, osz, sz.st_value, sz.shift, WL._ptr(d_tkey),
                                     WL._ptr(d_top), WL._ptr(d_tid), tlen, WL._ptr(d_cur), mid, 0, flags,
                                     WL._ptr(d_cnt), WL._ptr(d_opc), WL._ptr(d_hot), None), "refill")
    WL.check(WL._L.hkv_wl_fold_counters(WL._ptr(d_cnt), None), "fold")
    torch.cuda.synchronize()
    if flags & 4:
        assert np.array_equal(d_hot.cpu().numpy().reshape(W, 200), hot), "hot-key pointers differ"
    got = d_ops.cpu().numpy()
    if not np.array_equal(got, exp_ops):
        bad = np.nonzero(got != exp_ops)[0]
        pytest.fail(f"slab differs at {len(bad)} bytes: ops {np.unique(bad // osz)[:8]}, offsets {np.unique(bad % osz)[:16]}")
    assert np.array_equal(d_cur.cpu().numpy(), exp_cur)
    assert d_cnt[:5].cpu().tolist() == exp_cnt.tolist()
    # the opcode mirror (hkv_batch_desc.d_opcode_in) is every op's opcode byte after the refill
    assert np.array_equal(d_opc.cpu().numpy(), exp_ops.reshape(W * S, osz)[:, 8])


def _apply_patches(ops, patch, osz, st_value):
    """d_patch applied in numpy (include/hermeskv.h: the 16-B layout and what applying does)"""
    ops = ops.copy().reshape(-1, osz)
    p = patch.reshape(-1, 16)
    for i in np.nonzero(p[:, 14])[0]:
        o = ops[i]
        o[0:8] = p[i, 0:8]
        o[8], o[9], o[10] = p[i, 8], 141, p[i, 9]
        if p[i, 13]:
            o[11:16] = 0
        o[16:18] = p[i, 10:12]
        if p[i, 12]:
            o[18:18 + st_value] = p[i, 12]
    return ops.reshape(-1)


@pytest.mark.parametrize("flags", [0, 1, 2])
def test_refill_plan_matches_refill(flags):
    """hkv_wl_refill_plan + the next local launch's patches give exactly what hkv_wl_refill gives:
    the numpy refill restatement's ops after applying the plan's patches (numpy), the same cursors,
    counters and opcode mirror; non-refilled ops get invalid patches."""
    from hermes_amd import workload as WL
    sz = L.DEFAULT
    W, S, osz, tlen, mid = 37, 250, sz.op, 300, 2
    rng = np.random.default_rng(77 + flags)
    states = np.array([130, 128, 138, 137, 119, 121, 131, 132, 136, 140, 141, *IN_FLIGHT], dtype=np.uint8)
    ops = rng.integers(0, 256, size=W * S * osz, dtype=np.uint8)
    ops.reshape(W, S, osz)[:, :, 9] = rng.choice(states, size=(W, S))
    tkey = rng.integers(0, 2**63, size=W * tlen, dtype=np.int64)
    top = rng.choice(np.array([111, 112, 113], dtype=np.uint8), size=W * tlen)
    cursor = rng.integers(0, tlen, size=W, dtype=np.int32)
    exp_ops, exp_cur, exp_cnt = _refill_ref(ops, W, S, osz, sz.st_value, sz.shift, tkey.view(np.uint64), top, tlen,
                                            cursor, mid, False, flags)
    d_st = torch.from_numpy(ops.reshape(W * S, osz)[:, 9].copy()).cuda()
    d_tkey, d_top = torch.from_numpy(tkey).cuda(), torch.from_numpy(top).cuda()
    d_cur = torch.from_numpy(cursor.copy()).cuda()
    d_cnt = torch.zeros(4096, dtype=torch.int64, device="cuda")
    opc0 = ops.reshape(W * S, osz)[:, 8].copy()
    d_opc = torch.from_numpy(opc0.copy()).cuda()
    d_patch = torch.full((W * S * 16,), 0xAB, dtype=torch.uint8, device="cuda")   # stale bytes get overwritten
    WL.check(WL._L.hkv_wl_refill_plan(WL._ptr(d_st), W, S, sz.st_value, sz.shift, WL._ptr(d_tkey), WL._ptr(d_top),
                                      tlen, WL._ptr(d_cur), mid, flags, WL._ptr(d_cnt), WL._ptr(d_opc),
                                      WL._ptr(d_patch), None), "refill_plan")
    WL.check(WL._L.hkv_wl_fold_counters(WL._ptr(d_cnt), None), "fold")
    torch.cuda.synchronize()
    patch = d_patch.cpu().numpy()
    assert set(np.unique(patch.reshape(-1, 16)[:, 14]).tolist()) <= {0, 1}
    got = _apply_patches(ops, patch, osz, sz.st_value)
    assert np.array_equal(got, exp_ops), "patched ops differ from the refill"
    assert np.array_equal(d_cur.cpu().numpy(), exp_cur)
    assert d_cnt[:5].cpu().tolist() == exp_cnt.tolist()
    assert np.array_equal(d_opc.cpu().numpy(), exp_ops.reshape(W * S, osz)[:, 8])
    # the plan reads the state mirror and leaves it as it was (the local launch writes the new states)
    assert np.array_equal(d_st.cpu().numpy(), ops.reshape(W * S, osz)[:, 9])


@pytest.mark.parametrize("mirror", [False, True])
@pytest.mark.parametrize("big", [False, True])
def test_marshal_invs_kernel_matches_numpy(big, mirror):
    """hkv_wl_marshal_invs_cap (per-thread 16-B copies for 56-B ops, one wave-wide copy per op for
    312-B ops) against a numpy restatement of inv_skip_or_get_sender_id /
    inv_copy_and_modify_elem / inv_modify_elem_after_send (hermes_worker.c:12-65) with C credits;
    with the state mirror, it is read instead of the ops and follows their new states."""
    from hermes_amd import workload as WL
    sz = L.BIG if big else L.DEFAULT
    W, S, osz, C, mid = 29, 250, sz.op, 40, 3
    rng = np.random.default_rng(5 + big)
    states = np.array([122, 135, 123, 118, 121, 131, 130, 143], dtype=np.uint8)
    ops = rng.integers(0, 256, size=W * S * osz, dtype=np.uint8)
    ops.reshape(W, S, osz)[:, :, 9] = rng.choice(states, size=(W, S), p=[.3, .05, .05, .02, .3, .1, .1, .08])
    exp_ops = ops.copy().reshape(W, S, osz)
    exp_out = np.zeros((W, C, osz), dtype=np.uint8)
    exp_cnt = np.zeros(W, dtype=np.int32)
    held = 0
    after = {122: 143, 135: 148, 123: 144, 118: 119}
    for w in range(W):
        r = 0
        for i in range(S):
            st = int(exp_ops[w, i, 9])
            if st not in after:
                continue
            if r < C:
                exp_out[w, r] = exp_ops[w, i]
                exp_out[w, r, 8], exp_out[w, r, 9] = 114, mid
                exp_ops[w, i, 9] = after[st]
            r += 1
        exp_cnt[w] = min(r, C)
        held += max(0, r - C)
    d_ops = torch.from_numpy(ops.copy()).cuda()
    d_out = torch.zeros(W * C * osz, dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(W, dtype=torch.int32, device="cuda")
    d_held = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_st = torch.from_numpy(ops.reshape(W * S, osz)[:, 9].copy()).cuda() if mirror else None
    WL.check(WL._L.hkv_wl_marshal_invs_cap(WL._ptr(d_ops), W, S, osz, WL._ptr(d_out), C, WL._ptr(d_cnt), mid,
                                           WL._ptr(d_held), WL._ptr(d_st), None), "marshal_invs")
    torch.cuda.synchronize()
    if mirror:
        assert np.array_equal(d_st.cpu().numpy(), exp_ops.reshape(W * S, osz)[:, 9]), "state mirror differs"
    cnt = d_cnt.cpu().numpy()
    assert np.array_equal(cnt, exp_cnt)
    out = d_out.cpu().numpy().reshape(W, C, osz)
    for w in range(W):
        assert np.array_equal(out[w, :cnt[w]], exp_out[w, :cnt[w]]), f"worker {w}: INV rows differ"
    assert np.array_equal(d_ops.cpu().numpy(), exp_ops.reshape(-1)), "op states differ"
    assert int(d_held.item()) == held


def test_big_op_refill_from_state_mirror():
    """configs[2]'s refill three ways over the same rounds: planned as patches that the next local launch
    writes into the 312-B ops (patch_in_resolve; the default under fresh batches, asked for here), in place deciding from the state mirror
    (hkv_wl_refill_st, fused_refill=False) and in place from each op's state byte (hkv_wl_refill). After
    every round the mirrors equal the ops' state and opcode bytes, and the ops -- the planned round's with
    its patches applied (numpy) -- the cursors and the counters are the same byte for byte."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 25
    rounds = []
    for mode in ("plan", "mirror", "ops"):
        g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=True, big_objects=True, extra_cache_lines=4, skew=3)
        r = Round(g, 40, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 500, 500, seed=0x5EED,
                  max_steps=8, trace_len=1024, retry_stalled=True, fused_refill=mode == "plan")
        r.st_refill = mode == "mirror" and r.st_refill
        rounds.append((g, r))
    assert rounds[0][1].fused and rounds[1][1].st_refill, "configs[2] rounds plan their refills, else use the mirror"
    for _ in range(6):
        for _, r in rounds:
            r.step()
        torch.cuda.synchronize()
        p, a, b = rounds[0][1], rounds[1][1], rounds[2][1]
        ops = a.ops.view(-1, a.op)
        assert torch.equal(a.states, ops[:, 9]), "state mirror differs from the ops' state bytes"
        assert torch.equal(a.opcodes, ops[:, 8]), "opcode mirror differs from the ops' opcodes"
        assert torch.equal(a.ops, b.ops), "refill from the mirror differs from the refill from the ops"
        planned = _apply_patches(p.ops.cpu().numpy(), p.patch.cpu().numpy(), p.op, p.sizes.st_value)
        assert np.array_equal(planned, b.ops.cpu().numpy()), "planned refill differs from the refill in place"
        assert torch.equal(p.opcodes, b.ops.view(-1, b.op)[:, 8]), "planned opcode mirror differs"
        assert torch.equal(a.cursor, b.cursor) and torch.equal(p.cursor, b.cursor)
    assert rounds[0][1].stats() == rounds[1][1].stats() == rounds[2][1].stats()
    assert rounds[0][1].stats()["committed"] > 0
    for g, _ in rounds:
        assert g.take_error_flags() == 0
