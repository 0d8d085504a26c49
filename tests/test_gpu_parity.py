"""Parity of the device path (libhermeskv.so on an MI355X) with the oracle, bit for bit.

Every comparison is on the reference's byte images: element arrays, read_write_ops buffers,
node_suspected, and the whole MICA index + log after every batch. The oracle is the CPU
restatement pinned in tests/test_oracle.py.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402
from oracle.oracle import OracleKVS, gen_keys  # noqa: E402
from tests import gen  # noqa: E402
from tests.helpers import load_golden, run_known_answers  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(params=["engine", "small"], autouse=True)
def engine_path(request):
    """Every parity test runs on both device engines: the multi-kernel engine and the
    single-workgroup kernel that launches of at most 4096 elements take by default."""
    from hermes_amd import kvs
    kvs.HermesKV.default_flags = kvs.BATCH_ENGINE if request.param == "engine" else kvs.BATCH_SMALL
    yield request.param
    kvs.HermesKV.default_flags = 0


def _kvs():
    from hermes_amd.kvs import HermesKV
    return HermesKV


def make_pair(n_keys, num_bkts, log_cap, rmw=False, big=False, machine_id=0, skew=0):
    sizes = L.BIG if big else L.DEFAULT
    ecl = 4 if big else 0
    g = _kvs()(n_keys, num_bkts, log_cap, machine_id, rmw, big, ecl, skew=skew)
    o = OracleKVS(num_bkts, log_cap, machine_id, rmw, big, ecl, skew=skew)
    o.populate(n_keys, sizes.kvs_value)
    return g, o, sizes


def assert_tables_equal(g, o, what=""):
    gi, oi = g.index_bytes(), o.index_bytes()
    if not np.array_equal(gi, oi):
        bad = np.nonzero(gi != oi)[0]
        pytest.fail(f"{what}: index differs at {len(bad)} bytes, first {bad[:8]}")
    gl, ol = g.log_bytes(), o.log_bytes()[: g.cfg.log_cap]
    if not np.array_equal(gl, ol):
        bad = np.nonzero(gl != ol)[0]
        e = g.sizes.entry
        pytest.fail(f"{what}: log differs at {len(bad)} bytes; entries {np.unique(bad // e)[:8]} "
                    f"offsets-in-entry {np.unique(bad % e)[:16]}")
    assert g.log_head == o.log_head(), what
    assert g.take_error_flags() == 0, f"{what}: device consistency flags raised"


def assert_elems_equal(a, b, what):
    av, bv = a.view(np.uint8).reshape(len(a), -1), b.view(np.uint8).reshape(len(b), -1)
    if not np.array_equal(av, bv):
        rows = np.nonzero((av != bv).any(axis=1))[0]
        cols = np.nonzero((av != bv).any(axis=0))[0]
        r = rows[0]
        pytest.fail(f"{what}: {len(rows)} elems differ (first {rows[:8]}), byte columns {cols[:16]}; "
                    f"gpu {av[r][:20]} oracle {bv[r][:20]}")


# ------------------------------------------------------------------ populate
@pytest.mark.parametrize("n_keys,num_bkts,log_cap,big", [
    (20000, 2048, 1 << 21, False),     # ~10 keys per bucket: evictions + same-tag overwrites
    (3000, 4096, 1 << 17, False),      # log wraps (3000 x 64 B > 128 KiB)
    (1500, 256, 1 << 20, True),        # big objects, 320-byte entries
    (2000, 1024, 1 << 18, True),       # big objects whose log wraps past a non-multiple of 320
])
def test_populate_bit_exact(n_keys, num_bkts, log_cap, big):
    g, o, _ = make_pair(n_keys, num_bkts, log_cap, big=big, rmw=big)
    assert_tables_equal(g, o, "populate")
    assert g.evictions == o.evictions()


def test_populate_reference_default_geometry_lookups():
    """spacetime_init geometry (1M keys, 2^21 buckets): all keys but the survey's three hit."""
    ka = load_golden("known_answers.json")
    c = ka["config"]
    g = _kvs()(c["num_keys"], c["num_bkts"], c["log_cap"], machine_id=0)
    keys = gen_keys(c["num_keys"])
    n = len(keys)
    ops = np.zeros(n, dtype=L.op_dtype())
    ops["key"] = keys
    ops["opcode"] = int(L.Op.GET)
    ops["state"] = int(L.Bucket.NEW)
    stride = 250
    nb = (n + stride - 1) // stride
    padded = np.zeros(nb * stride, dtype=ops.dtype)
    padded[:n] = ops
    counts = np.full(nb, stride, dtype=np.int32)
    counts[-1] = n - (nb - 1) * stride
    g.batch_host(L.BatchType.local_ops, padded, L.membership(3, 0), n_batches=nb, stride=stride, counts=counts)
    st = padded["state"][:n]
    assert np.nonzero(st == int(L.Resp.MISS))[0].tolist() == ka["always_miss_ids"]
    ok = st == int(L.Resp.GET_COMPLETE)
    assert ok.sum() == n - 3
    ids = np.arange(n)
    assert (padded["value"][:n][ok, 0] == ord("a") + ids[ok] % 20).all()
    assert (padded["val_len"][:n][ok] == 30).all()


# ------------------------------------------------------------------ known answers
class _GpuEngine:
    def __init__(self, kvs):
        self.kvs = kvs

    def batch(self, btype, elems, mb, rw=None):
        self.kvs.batch_host(btype, elems, mb, rw=rw)

    def entry(self, key):
        return self.kvs.entry(key)


def test_known_answers_device_path():
    c = load_golden("known_answers.json")["config"]
    g = _kvs()(c["num_keys"], c["num_bkts"], c["log_cap"], machine_id=c["machine_id"])
    run_known_answers(_GpuEngine(g), gen_keys(c["num_keys"]))


class _RefApiEngine:
    """Drives the exported reference entry points (spacetime_init + hermes_batch_ops_to_KVS)."""

    def __init__(self, kvs_mod):
        self.m = kvs_mod

    def batch(self, btype, elems, mb, rw=None):
        ns = [-1]
        full = None
        if rw is not None:  # the reference's read_write_ops holds max_batch_size (250) ops
            full = np.zeros(250, dtype=rw.dtype)
            full[: len(rw)] = rw
        self.m.hermes_batch_ops_to_KVS(btype, elems, len(elems), elems.dtype.itemsize, mb, ns, full, 0)
        if rw is not None:
            rw[:] = full[: len(rw)]

    def entry(self, key):
        return _kvs().default_table().entry(key)


def test_known_answers_reference_entry_points():
    from hermes_amd import kvs
    kvs.spacetime_init(0)
    run_known_answers(_RefApiEngine(kvs), gen_keys(1_000_000))


def _oracle_from_device(kvs, skew):
    """An oracle table holding the device table's current image (index, log, head)"""
    from oracle.oracle import lib as olib
    c = kvs.cfg
    o = OracleKVS(c.num_bkts, c.log_cap, c.machine_id, bool(c.rmw_enabled), bool(c.big_objects), c.extra_cache_lines,
                  skew=skew)
    o.index_bytes()[:] = kvs.index_bytes()
    used = min(kvs.log_head, c.log_cap)
    o.log_bytes()[:used] = kvs.log_bytes(0, used)
    olib().hko_set_log_head.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    olib().hko_set_log_head(o.h, kvs.log_head)
    return o


@pytest.mark.parametrize("skew", [0, 3])
def test_random_rounds_reference_entry_points(skew):
    """Randomized protocol rounds through the drop-in entry point itself (spacetime_init +
    hermes_batch_ops_to_KVS on the default 1M-key table), one call per worker batch as the
    reference's workers make them (hermes_worker.c:451-509): local ops, INVs (with membership-change
    INVs: node_suspected), ACKs against the worker's own op buffer as read_write_ops, VALs, and the
    after-membership-change batch. Small calls take the partitioned launch (k_hpart: one workgroup
    per key partition); a call piling more than a partition's capacity on one key (the hot round's
    900-element batches) takes the single-workgroup kernel. Each call is replayed on an oracle copy
    of the table; elements, read_write_ops, node_suspected and the touched keys' entries must match."""
    from hermes_amd import kvs as K
    K.spacetime_init(0)
    d = K.HermesKV.default_table()
    d.set_skew(skew)
    try:
        o = _oracle_from_device(d, skew)
        keys = gen_keys(1_000_000)
        rng = np.random.default_rng(20261017 + skew)
        tsp = gen.TsPool(rng)
        sizes = L.DEFAULT
        mb_full, mb_fail = L.membership(5, 0), L.membership(5, 0, alive=0b01111)
        W = 4

        def call(btype, e, mb, rw=None, what=""):
            eo = gen.bytecopy(e)
            rwo = gen.bytecopy(rw) if rw is not None else None
            ns_g, ns_o = [-1], None
            K.hermes_batch_ops_to_KVS(btype, e, len(e), e.dtype.itemsize, mb, ns_g, rw, 0)
            ns_o = o.batch(btype, eo, mb, rw=rwo)
            assert_elems_equal(e, eo, what)
            if rw is not None:
                assert_elems_equal(rw, rwo, what + " rw")
            assert ns_g[0] == ns_o, f"{what}: node_suspected {ns_g[0]} vs {ns_o}"

        def entries_equal(pool, what):
            for k in pool:
                off = o.lookup(int(k))
                if off is None:
                    continue
                assert np.array_equal(d.log_bytes(off, 64), o.log_bytes()[off:off + 64]), f"{what}: entry of {int(k):#x}"

        for rnd in range(12):
            hot = rnd in (5, 11)
            pool = keys[[rng.integers(0, 1_000_000)]] if hot else gen.key_pool(rng, keys, hot=24 if rnd % 2 else 300)
            mb = mb_fail if rnd >= 8 else mb_full
            n_loc, n_msg = (250, 900) if hot else (int(rng.integers(100, 251)), int(rng.integers(20, 200)))
            bufs = []
            for w in range(W):
                loc = gen.local_ops(rng, pool, n_loc, sizes, False, tsp)
                if skew:
                    z = rng.random(n_loc) < 0.3
                    loc["ts_ver"][z] = 0
                    loc["ts_cid"][z & (loc["opcode"] == int(L.Op.GET))] = 0
                call(L.BatchType.local_ops, loc, mb, what=f"round {rnd} worker {w} local")
                gen.harvest_ts(tsp, loc)
                rw = np.zeros(250, dtype=L.op_dtype())
                rw[:n_loc] = loc
                bufs.append(rw)
            for w in range(W):
                call(L.BatchType.invs, gen.invs(rng, pool, n_msg, sizes, False, tsp), mb, what=f"round {rnd} invs {w}")
            for w in range(W):
                call(L.BatchType.acks, gen.acks(rng, pool, n_msg, sizes, False, tsp), mb, rw=bufs[w],
                     what=f"round {rnd} acks {w}")
            for w in range(W):
                call(L.BatchType.vals, gen.vals(rng, pool, n_msg, sizes, False, tsp), mb, what=f"round {rnd} vals {w}")
            if rnd >= 8:
                call(L.BatchType.local_ops_after_membership_change, gen.memb_ops(rng, pool, n_loc, sizes, False, tsp),
                     mb_fail, what=f"round {rnd} membership")
            entries_equal(pool, f"round {rnd}")
        assert d.take_error_flags() == 0
    finally:
        d.set_skew(0)


# ------------------------------------------------------------------ randomized protocol rounds
CONFIGS = [
    pytest.param(dict(rmw=False, big=False), id="default"),
    pytest.param(dict(rmw=False, big=True), id="big"),
    pytest.param(dict(rmw=True, big=False), id="rmw"),
    pytest.param(dict(rmw=True, big=True), id="big_rmw"),
    # the reference's skew optimisations (hkv_config.skew_flags, config.h:79-80): stalled GETs and
    # PUTs complete once the key's version moved on
    pytest.param(dict(rmw=False, big=False, skew=3), id="skew"),
    pytest.param(dict(rmw=False, big=True, skew=3), id="big_skew"),
    pytest.param(dict(rmw=True, big=False, skew=3), id="rmw_skew"),
]


def _run_both(g, o, btype, elems_g, elems_o, mb, n_batches, stride, counts, rw_g=None, rw_o=None,
              rw_stride=0, ns_g=None, ns_o=None, packed=False):
    """packed: the device gets the batches back to back (HKV_BATCH_PACKED), the oracle in rows;
    elems_g then holds the rows again afterwards (empty slots untouched)"""
    if packed:
        cnt = np.full(n_batches, stride, np.int32) if counts is None else counts
        live = (np.arange(stride)[None, :] < cnt[:, None]).reshape(-1)
        off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        flat = elems_g[live].copy()
        g.batch_host(btype, flat, mb, rw=rw_g, n_batches=n_batches, node_suspected=ns_g, offsets=off,
                     rw_stride_elems=rw_stride)
        elems_g[live] = flat
    else:
        g.batch_host(btype, elems_g, mb, rw=rw_g, n_batches=n_batches, stride=stride, counts=counts,
                     rw_stride_elems=rw_stride, node_suspected=ns_g)
    o.batch_multi(btype, elems_o, n_batches, stride, counts, mb, rw=rw_o, rw_stride_elems=rw_stride,
                  node_suspected=ns_o)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_random_protocol_rounds(cfg):
    rng = np.random.default_rng(20261015)
    rmw, big, skew = cfg["rmw"], cfg["big"], cfg.get("skew", 0)
    n_keys, num_bkts = 3000, 512
    sizes = L.BIG if big else L.DEFAULT
    log_cap = 1 << max(16, (n_keys * sizes.entry + 1024).bit_length())
    g, o, sizes = make_pair(n_keys, num_bkts, log_cap, rmw=rmw, big=big, machine_id=0, skew=skew)
    assert_tables_equal(g, o, "populate")
    keys = gen_keys(n_keys)
    tsp = gen.TsPool(rng)
    mb_full = L.membership(5, 0)
    mb_fail = L.membership(5, 0, alive=0b01111)     # node 4 dropped
    W, S, M = 5, 48, 96                              # workers, local stride, message stride
    for rnd in range(14):
        pool = gen.key_pool(rng, keys, hot=24 if rnd % 2 else 200)
        mb = mb_fail if rnd >= 9 else mb_full
        # local ops
        loc = gen.local_ops(rng, pool, W * S, sizes, rmw, tsp)
        if skew:   # refilled GETs carry (0, 0) (inline-util.h:268-272); some PUTs version 0
            z = rng.random(W * S) < 0.3
            loc["ts_ver"][z] = 0
            loc["ts_cid"][z & (loc["opcode"] == int(L.Op.GET))] = 0
        counts = rng.integers(S // 2, S + 1, size=W).astype(np.int32)
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, W, S, counts)
        assert_elems_equal(loc, loc_o, f"round {rnd} local")
        gen.harvest_ts(tsp, loc)
        assert_tables_equal(g, o, f"round {rnd} local")
        rw_g, rw_o = gen.bytecopy(loc), gen.bytecopy(loc)   # each worker's op buffer is its read_write_ops
        # invs
        inv = gen.invs(rng, pool, W * M, sizes, rmw, tsp)
        counts = rng.integers(0, M + 1, size=W).astype(np.int32)
        ns_g = np.full(W, -1, np.int32)
        ns_o = ns_g.copy()
        inv_o = gen.bytecopy(inv)
        _run_both(g, o, L.BatchType.invs, inv, inv_o, mb, W, M, counts, ns_g=ns_g, ns_o=ns_o, packed=rnd % 2 == 1)
        assert_elems_equal(inv, inv_o, f"round {rnd} invs")
        np.testing.assert_array_equal(ns_g, ns_o)
        assert_tables_equal(g, o, f"round {rnd} invs")
        # acks (read_write_ops = the local buffers)
        ack = gen.acks(rng, pool, W * M, sizes, rmw, tsp)
        counts = rng.integers(M // 2, M + 1, size=W).astype(np.int32)
        ack_o = gen.bytecopy(ack)
        _run_both(g, o, L.BatchType.acks, ack, ack_o, mb, W, M, counts, rw_g, rw_o, rw_stride=S, packed=rnd % 2 == 0)
        assert_elems_equal(ack, ack_o, f"round {rnd} acks")
        assert_elems_equal(rw_g, rw_o, f"round {rnd} acks rw")
        assert_tables_equal(g, o, f"round {rnd} acks")
        # vals
        val = gen.vals(rng, pool, W * M, sizes, rmw, tsp)
        val_o = gen.bytecopy(val)
        _run_both(g, o, L.BatchType.vals, val, val_o, mb, W, M, None, packed=rnd % 3 == 1)
        assert_elems_equal(val, val_o, f"round {rnd} vals")
        assert_tables_equal(g, o, f"round {rnd} vals")
        # completion after a membership change
        if rnd >= 9:
            mem = gen.memb_ops(rng, pool, W * S, sizes, rmw, tsp)
            mem_o = gen.bytecopy(mem)
            _run_both(g, o, L.BatchType.local_ops_after_membership_change, mem, mem_o, mb_fail, W, S, None)
            assert_elems_equal(mem, mem_o, f"round {rnd} membership")
            assert_tables_equal(g, o, f"round {rnd} membership")


def test_empty_and_all_miss_batches():
    g, o, sizes = make_pair(500, 256, 1 << 16)
    keys = gen_keys(500)
    mb = L.membership(3, 0)
    # zero-length batches are no-ops
    e = np.zeros(4, dtype=L.op_dtype())
    g.batch_host(L.BatchType.local_ops, e, mb, n_batches=4, stride=1, counts=np.zeros(4, np.int32))
    assert (e["state"] == 0).all()
    # elements whose keys are absent: ST_MISS in byte 9 of every element type
    rng = np.random.default_rng(3)
    for bt, msg in ((L.BatchType.local_ops, False), (L.BatchType.invs, False), (L.BatchType.acks, True),
                    (L.BatchType.vals, True)):
        a = np.zeros(64, dtype=L.msg_dtype() if msg else L.op_dtype())
        a["key"] = rng.integers(1, 2**63, size=64, dtype=np.int64).astype(np.uint64)
        a["opcode"] = {0: 111, 2: 114, 3: 115, 4: 116}[int(bt)]
        b = gen.bytecopy(a)
        g.batch_host(bt, a, mb)
        o.batch(bt, b, mb)
        assert_elems_equal(a, b, f"miss {bt}")
        assert (a.view(np.uint8).reshape(64, -1)[:, 9] == int(L.Resp.MISS)).all()
    assert_tables_equal(g, o, "misses")
    del keys, sizes


@pytest.mark.parametrize("cfg", CONFIGS)
def test_max_size_batches_single_hot_key(cfg):
    """Maximum batch sizes (250 local / 900 msg per worker) all on one or two keys: every batch
    type goes through the hot-key workgroup engine (segments far longer than kShortSeg)."""
    rmw, big = cfg["rmw"], cfg["big"]
    g, o, sizes = make_pair(1000, 1024, 1 << 19 if big else 1 << 17, rmw=rmw, big=big)
    keys = gen_keys(1000)
    rng = np.random.default_rng(7)
    tsp = gen.TsPool(rng)
    mb = L.membership(3, 0)
    W = 8
    for rnd, pool in enumerate((keys[[17]], keys[[17, 18]], keys[[17]])):
        loc = gen.local_ops(rng, pool, W * 250, sizes, rmw, tsp)
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, W, 250, None)
        assert_elems_equal(loc, loc_o, f"hot local {rnd}")
        gen.harvest_ts(tsp, loc)
        inv = gen.invs(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        inv_o = gen.bytecopy(inv)
        ns_g = np.full(W, -1, np.int32)
        ns_o = ns_g.copy()
        _run_both(g, o, L.BatchType.invs, inv, inv_o, mb, W, 900, None, ns_g=ns_g, ns_o=ns_o)
        assert_elems_equal(inv, inv_o, f"hot invs {rnd}")
        np.testing.assert_array_equal(ns_g, ns_o)
        ack = gen.acks(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        ack_o = gen.bytecopy(ack)
        rw_g, rw_o = gen.bytecopy(loc), gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.acks, ack, ack_o, mb, W, 900, None, rw_g, rw_o, rw_stride=250)
        assert_elems_equal(ack, ack_o, f"hot acks {rnd}")
        assert_elems_equal(rw_g, rw_o, f"hot rw {rnd}")
        val = gen.vals(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        val_o = gen.bytecopy(val)
        _run_both(g, o, L.BatchType.vals, val, val_o, mb, W, 900, None)
        assert_elems_equal(val, val_o, f"hot vals {rnd}")
        mem = gen.memb_ops(rng, pool, W * 250, sizes, rmw, tsp)
        mem_o = gen.bytecopy(mem)
        _run_both(g, o, L.BatchType.local_ops_after_membership_change, mem, mem_o,
                  L.membership(3, 0, alive=0b011), W, 250, None)
        assert_elems_equal(mem, mem_o, f"hot membership {rnd}")
        assert_tables_equal(g, o, f"hot {rnd}")


@pytest.mark.parametrize("cfg", CONFIGS)
def test_tag_collisions_in_segments(cfg):
    """Keys absent from the table whose bucket and tag equal a present key's: the reference
    finds the present key's slot, fails the 8-byte compare and reports ST_MISS. The device
    defers that compare to the segment engines, so these elements sit inside the present key's
    segments (short and hot) and must come out ST_MISS without touching the entry."""
    rmw, big = cfg["rmw"], cfg["big"]
    g, o, sizes = make_pair(1000, 1024, 1 << 19 if big else 1 << 17, rmw=rmw, big=big)
    keys = gen_keys(1000)
    rng = np.random.default_rng(11)
    tsp = gen.TsPool(rng)
    mb = L.membership(3, 0)
    W = 6
    hot = keys[[21, 22]]
    fake = np.array([int(k) ^ (1 << 40) for k in hot] + [int(hot[0]) ^ (1 << 33)], dtype=np.uint64)
    assert all(o.lookup(int(f)) is None for f in fake)
    for rnd, pool in enumerate((np.concatenate([hot, fake]), np.concatenate([keys[100:400], fake]),
                                np.concatenate([hot[:1], fake[:1]]))):
        loc = gen.local_ops(rng, pool, W * 250, sizes, rmw, tsp)
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, W, 250, None)
        assert_elems_equal(loc, loc_o, f"collide local {rnd}")
        gen.harvest_ts(tsp, loc)
        inv = gen.invs(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        inv_o = gen.bytecopy(inv)
        ns_g = np.full(W, -1, np.int32)
        ns_o = ns_g.copy()
        _run_both(g, o, L.BatchType.invs, inv, inv_o, mb, W, 900, None, ns_g=ns_g, ns_o=ns_o)
        assert_elems_equal(inv, inv_o, f"collide invs {rnd}")
        ack = gen.acks(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        ack_o = gen.bytecopy(ack)
        rw_g, rw_o = gen.bytecopy(loc), gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.acks, ack, ack_o, mb, W, 900, None, rw_g, rw_o, rw_stride=250)
        assert_elems_equal(ack, ack_o, f"collide acks {rnd}")
        assert_elems_equal(rw_g, rw_o, f"collide rw {rnd}")
        val = gen.vals(rng, pool, W * 900, sizes, rmw, tsp, machine_num=3)
        val_o = gen.bytecopy(val)
        _run_both(g, o, L.BatchType.vals, val, val_o, mb, W, 900, None)
        assert_elems_equal(val, val_o, f"collide vals {rnd}")
        miss = np.isin(loc["key"], fake)
        assert (loc["state"][miss] == int(L.Resp.MISS)).sum() > miss.sum() // 2  # the rest were skipped
        assert_tables_equal(g, o, f"collide {rnd}")


def test_adversarial_inv_alternating_equal_timestamps():
    """Equal-timestamp INVs from alternating senders: every one rewrites last_writer_id, so the
    hot-key engine has one candidate per element (its slowest case) and must stay exact."""
    g, o, sizes = make_pair(500, 512, 1 << 16)
    keys = gen_keys(500)
    mb = L.membership(3, 0)
    n = 4 * 900
    inv = np.zeros(n, dtype=L.op_dtype())
    inv["key"] = keys[3]
    inv["opcode"] = int(L.Op.INV)
    inv["state"] = np.arange(n) % 3
    inv["ts_ver"] = 2 * (1 + (np.arange(n) // 1000))
    inv["ts_cid"] = 1
    inv["val_len"] = 31
    inv["value"] = (np.arange(n) % 251)[:, None]
    inv_o = gen.bytecopy(inv)
    _run_both(g, o, L.BatchType.invs, inv, inv_o, mb, 4, 900, None)
    assert_elems_equal(inv, inv_o, "alternating invs")
    assert_tables_equal(g, o, "alternating invs")


def test_hash_ids_matches_oracle():
    from hermes_amd.kvs import hash_ids
    ids = np.concatenate([np.arange(0, 5000), np.array([631343, 2**31 - 1, 99_999_999])]).astype(np.int32)
    got = hash_ids(torch.from_numpy(ids).cuda()).cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got[:5000], gen_keys(5000))
    from oracle.oracle import cityhash128
    for k, i in enumerate(ids[5000:]):
        assert got[5000 + k] == cityhash128(int(i).to_bytes(4, "little"))[1]


@pytest.mark.parametrize("big", [False, True])
def test_inv_direct_path_edge_cases(big):
    """The INV direct path (non-RMW INV launches: X/F/Y words, k_inv_resolve, k_inv_commit) against
    the oracle: timestamps below, equal to and above each key's (so OUT_OF_GROUP holds exactly up
    to the first raise while the key is in WRITE), repeated maxima from several senders (the last
    one's sender is the last writer), INV_ABORT / OUT_OF_GROUP / MEMBERSHIP_CHANGE input opcodes,
    hot and missing keys, ragged counts, and launches past the 8192-element lookup head."""
    g, o, sizes = make_pair(2000, 1024, 1 << 20 if big else 1 << 17, big=big)
    keys = gen_keys(2000)
    rng = np.random.default_rng(424242)
    tsp = gen.TsPool(rng)
    mb = L.membership(5, 0)
    e = sizes.entry
    W, M = 14, 900
    for rnd in range(6):
        pool = gen.key_pool(rng, keys, hot=12 if rnd % 2 else 150)
        loc = gen.local_ops(rng, pool, 8 * 250, sizes, False, tsp)   # leaves keys in WRITE / REPLAY
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, 8, 250, None)
        assert_elems_equal(loc, loc_o, f"round {rnd} local")
        inv = np.zeros(W * M, dtype=L.op_dtype(sizes))
        inv["key"] = gen.draw_keys(rng, pool, W * M)
        log = o.log_bytes()
        cur_v = np.zeros(W * M, np.uint32)
        cur_c = np.zeros(W * M, np.uint8)
        for i, k in enumerate(inv["key"]):
            off = o.lookup(int(k))
            if off is not None:
                cur_v[i] = log[off + 24:off + 28].view(np.uint32)[0]
                cur_c[i] = log[off + 23]
        kind = rng.choice(4, size=W * M, p=[0.2, 0.35, 0.3, 0.15])   # below, equal, +2, +4
        ver = cur_v.astype(np.int64) + np.select([kind == 0, kind == 2, kind == 3], [-2, 2, 4], 0)
        ver = np.maximum(ver, 0).astype(np.uint32)
        cid = np.where(kind == 1, cur_c, rng.integers(0, 3, size=W * M)).astype(np.uint8)
        inv["ts_ver"] = ver
        inv["ts_cid"] = cid
        inv["state"] = rng.integers(0, 5, size=W * M)                    # sender
        inv["opcode"] = rng.choice([int(L.Op.INV), int(L.Resp.OP_INV_ABORT), L.INV_OUT_OF_GROUP,
                                    int(L.Op.MEMBERSHIP_CHANGE)], size=W * M, p=[0.8, 0.08, 0.07, 0.05])
        inv["val_len"] = sizes.st_value >> sizes.shift
        inv["flags"] = rng.integers(0, 2, size=W * M)
        inv["value"] = rng.integers(0, 256, size=(W * M, sizes.st_value))
        counts = rng.integers(M // 2, M + 1, size=W).astype(np.int32)
        ns_g = np.full(W, -1, np.int32)
        ns_o = ns_g.copy()
        inv_o = gen.bytecopy(inv)
        _run_both(g, o, L.BatchType.invs, inv, inv_o, mb, W, M, counts, ns_g=ns_g, ns_o=ns_o, packed=rnd % 2 == 1)
        assert_elems_equal(inv, inv_o, f"round {rnd} invs")
        np.testing.assert_array_equal(ns_g, ns_o)
        assert_tables_equal(g, o, f"round {rnd} invs")
        out = inv["opcode"][inv["state"] != int(L.Resp.MISS)]
        assert (out == L.INV_OUT_OF_GROUP).any() and (out == int(L.Resp.INV_SUCCESS)).any()
        # VALs for some of the INVs bring keys back to VALID for the next round
        val = gen.vals(rng, pool, 8 * 250, sizes, False, tsp)
        val_o = gen.bytecopy(val)
        _run_both(g, o, L.BatchType.vals, val, val_o, mb, 8, 250, None)
        assert_elems_equal(val, val_o, f"round {rnd} vals")
    del e


@pytest.mark.parametrize("big", [False, True])
def test_ack_direct_path_edge_cases(big):
    """The ACK direct path (non-RMW ACK launches: epoch-tagged T words, F, k_ack_resolve) against the
    oracle: ACKs matching each key's pending write or not, duplicate and out-of-range (>= 8)
    senders, quorums reached at different elements or never, LAST_ACK_* input opcodes, a
    membership with a dropped node, ragged counts and read_write_ops completions."""
    g, o, sizes = make_pair(2000, 1024, 1 << 20 if big else 1 << 17, big=big)
    keys = gen_keys(2000)
    rng = np.random.default_rng(515151)
    tsp = gen.TsPool(rng)
    W, S, M = 10, 250, 400
    for rnd in range(6):
        mb = L.membership(5, 0) if rnd < 4 else L.membership(5, 0, alive=0b10111)
        pool = gen.key_pool(rng, keys, hot=16 if rnd % 2 else 300)
        loc = gen.local_ops(rng, pool, W * S, sizes, False, tsp)     # pending writes / replays
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, W, S, None)
        assert_elems_equal(loc, loc_o, f"round {rnd} local")
        rw_g, rw_o = gen.bytecopy(loc), gen.bytecopy(loc)
        ack = np.zeros(W * M, dtype=L.msg_dtype())
        ack["key"] = gen.draw_keys(rng, pool, W * M)
        log = o.log_bytes()
        lv = np.zeros(W * M, np.uint32)
        lc = np.zeros(W * M, np.uint8)
        for i, k in enumerate(ack["key"]):
            off = o.lookup(int(k))
            if off is not None:
                lc[i] = log[off + 28]
                lv[i] = int.from_bytes(bytes(log[off + 29:off + 33]), "little")
        match = rng.random(W * M) < 0.7
        ack["ts_ver"] = np.where(match, lv, lv + 2)
        ack["ts_cid"] = np.where(match, lc, rng.integers(0, 5, size=W * M))
        ack["sender"] = rng.choice(10, size=W * M, p=[0.22, 0.22, 0.22, 0.12, 0.1, 0.04, 0.02, 0.02, 0.02, 0.02])
        ack["opcode"] = rng.choice([int(L.Op.ACK), int(L.Resp.LAST_ACK_SUCCESS),
                                    int(L.Resp.LAST_ACK_NO_BCAST_SUCCESS), int(L.Resp.ACK_SUCCESS)],
                                   size=W * M, p=[0.8, 0.1, 0.05, 0.05])
        counts = rng.integers(M // 3, M + 1, size=W).astype(np.int32)
        ack_o = gen.bytecopy(ack)
        _run_both(g, o, L.BatchType.acks, ack, ack_o, mb, W, M, counts, rw_g, rw_o, rw_stride=S, packed=rnd % 2 == 0)
        assert_elems_equal(ack, ack_o, f"round {rnd} acks")
        assert_elems_equal(rw_g, rw_o, f"round {rnd} acks rw")
        assert_tables_equal(g, o, f"round {rnd} acks")
        live = np.concatenate([np.arange(b * M, b * M + counts[b]) for b in range(W)])
        assert (ack["opcode"][live] == int(L.Resp.LAST_ACK_SUCCESS)).sum() > 0
        val = gen.vals(rng, pool, W * S, sizes, False, tsp)
        val_o = gen.bytecopy(val)
        _run_both(g, o, L.BatchType.vals, val, val_o, mb, W, S, None)
        assert_elems_equal(val, val_o, f"round {rnd} vals")


@pytest.mark.parametrize("cfg", CONFIGS)
def test_scripted_rare_outcomes(cfg):
    """tests/scripted.py through the device path and the oracle side by side: every step's
    elements, read_write_ops, node_suspected and table image bit-exact, the scripted outcomes
    (OUT_OF_GROUP, INV-aborts both ways, RMW_ABORT, ST_EMPTY reads, LAST_ACK completions of PUTs,
    RMWs and GET replays, write replays, *_COMPLETE_SEND_VALS after membership changes) all
    produced, covering every outcome code the batch function can emit in the build."""
    from tests.scripted import required_outcomes, run_scripted
    rmw, big = cfg["rmw"], cfg["big"]
    g, o, sizes = make_pair(1000, 4096, 1 << 22, rmw=rmw, big=big)

    def runner(btype, elems, mb, rw=None, node_suspected=None):
        eo, rwo = gen.bytecopy(elems), (gen.bytecopy(rw) if rw is not None else None)
        ns_o = node_suspected.copy() if node_suspected is not None else None
        g.batch_host(btype, elems, mb, rw=rw, node_suspected=node_suspected)
        o.batch_multi(btype, eo, 1, len(eo), None, mb, rw=rwo, node_suspected=ns_o)
        assert_elems_equal(elems, eo, f"scripted type {int(btype)}")
        if rw is not None:
            assert_elems_equal(rw, rwo, f"scripted type {int(btype)} rw")
        if node_suspected is not None:
            np.testing.assert_array_equal(node_suspected, ns_o)
        assert_tables_equal(g, o, f"scripted type {int(btype)}")

    seen = run_scripted(runner, gen_keys(1000), sizes, rmw)
    missing = required_outcomes(rmw) - seen
    assert not missing, f"not produced: {sorted(missing, key=str)}"


@pytest.mark.parametrize("big", [False, True])
def test_scripted_skew_optimisations(big):
    """tests/scripted.py's skew scenario (skew_flags 3, config.h:79-80) through the device path and
    the oracle side by side: elements, read_write_ops and the table bit-exact, and the scripted
    read completions and coalesced writes produced -- after a key's first write in the same
    launch (S_1's timestamp), in REPLAY, and with the write path's 16-bit version."""
    from tests.scripted import run_scripted_skew
    g, o, sizes = make_pair(1000, 4096, 1 << 22, big=big, skew=3)

    def runner(btype, elems, mb, rw=None, node_suspected=None):
        eo, rwo = gen.bytecopy(elems), (gen.bytecopy(rw) if rw is not None else None)
        g.batch_host(btype, elems, mb, rw=rw)
        o.batch_multi(btype, eo, 1, len(eo), None, mb, rw=rwo)
        assert_elems_equal(elems, eo, f"skew type {int(btype)}")
        if rw is not None:
            assert_elems_equal(rw, rwo, f"skew type {int(btype)} rw")
        assert_tables_equal(g, o, f"skew type {int(btype)}")

    seen = run_scripted_skew(runner, gen_keys(1000), sizes)
    assert (0, int(L.Resp.PUT_COMPLETE)) in seen and (0, int(L.Resp.GET_COMPLETE)) in seen


def test_local_opcode_mirror(engine_path):
    """hkv_batch_desc.d_opcode_in: with a correct mirror the local launch gives the same bytes as
    without one (k_local_pre then reads only the PUTs' headers); a mirror that hides a PUT is
    reported as error flag bit 3."""
    if engine_path != "engine":
        pytest.skip("the mirror is read by the multi-kernel engine's direct local path")
    rng = np.random.default_rng(31)
    g, o, sizes = make_pair(3000, 512, 1 << 18)
    keys = gen_keys(3000)
    tsp = gen.TsPool(rng)
    W, S = 40, 200   # 8000 elements: several prepass blocks, so the launch-head filter runs too
    mb = L.membership(3, 0)
    for rnd in range(3):
        pool = gen.key_pool(rng, keys, hot=24 if rnd % 2 else 400)
        loc = gen.local_ops(rng, pool, W * S, sizes, False, tsp)
        loc_o = gen.bytecopy(loc)
        d = torch.from_numpy(loc.view(np.uint8).copy()).cuda()
        opc = torch.from_numpy(loc["opcode"].astype(np.uint8).copy()).cuda()
        g.batch(L.BatchType.local_ops, d, W, S, sizes.op, mb, opcode_in=opc)
        torch.cuda.synchronize()
        o.batch_multi(L.BatchType.local_ops, loc_o, W, S, None, mb)
        got = d.cpu().numpy()
        assert np.array_equal(got, loc_o.view(np.uint8).reshape(-1)), f"round {rnd}: elements differ"
        assert_tables_equal(g, o, f"round {rnd}")
        assert g.take_error_flags() == 0
    # hide every PUT from the mirror: the launch reports it
    loc = gen.local_ops(rng, gen.key_pool(rng, keys, hot=400), W * S, sizes, False, tsp)
    d = torch.from_numpy(loc.view(np.uint8).copy()).cuda()
    opc = torch.full((W * S,), int(L.Op.GET), dtype=torch.uint8, device="cuda")
    g.batch(L.BatchType.local_ops, d, W, S, sizes.op, mb, opcode_in=opc)
    assert g.take_error_flags() & 8


@pytest.mark.parametrize("rmw,big", [(False, False), (False, True), (True, True)], ids=["default", "big", "big_rmw"])
def test_unique_inv_launch_matches_oracle(engine_path, rmw, big):
    """HKV_BATCH_UNIQUE INV launches (one pass, each element straight onto its entry; big objects:
    element and entry staged in LDS, k_unique_big): a peer's slab with one INV per key -- raises,
    equal and smaller timestamps, keys in WRITE (OUT_OF_GROUP), RMW INVs answered with INV-aborts,
    membership-change INVs (node_suspected), ragged counts and misses -- against the oracle; a slab
    with a repeated key raises error flag bit 4 (HKV_CHECK_UNIQUE, set by conftest)."""
    import os
    assert os.environ.get("HKV_CHECK_UNIQUE") == "1"
    rng = np.random.default_rng(4242)
    g, o, sizes = make_pair(4000, 1024, 1 << 21 if big else 1 << 18, rmw=rmw, big=big)
    keys = gen_keys(4000)
    tsp = gen.TsPool(rng)
    mb = L.membership(5, 0)
    for rnd in range(6):
        # local writes first, so some keys sit in WRITE with a pending timestamp
        loc = gen.local_ops(rng, gen.key_pool(rng, keys, hot=300), 2000, sizes, rmw, tsp)
        loc_o = gen.bytecopy(loc)
        _run_both(g, o, L.BatchType.local_ops, loc, loc_o, mb, 8, 250, None)
        gen.harvest_ts(tsp, loc)
        ids = rng.choice(4000, size=3000, replace=False)
        pool = np.concatenate([keys[ids], rng.integers(1, 2**63, size=16, dtype=np.int64).astype(np.uint64)])
        rng.shuffle(pool)
        inv = gen.invs(rng, pool, len(pool), sizes, rmw, tsp)
        inv["key"] = pool                           # every key once
        W, M = 4, len(pool) // 4
        counts = rng.integers(M // 2, M + 1, size=W).astype(np.int32)
        inv_o = gen.bytecopy(inv)
        ns_g, ns_o = np.full(W, -1, np.int32), np.full(W, -1, np.int32)
        g.batch_host(L.BatchType.invs, inv, mb, n_batches=W, stride=M, counts=counts, node_suspected=ns_g,
                     unique=True)
        o.batch_multi(L.BatchType.invs, inv_o, W, M, counts, mb, node_suspected=ns_o)
        assert_elems_equal(inv, inv_o, f"round {rnd} unique invs")
        np.testing.assert_array_equal(ns_g, ns_o)
        assert_tables_equal(g, o, f"round {rnd} unique invs")
    if engine_path == "engine":   # the check runs in the one-pass kernel
        dup = gen.invs(rng, keys[:64], 512, sizes, rmw, tsp)
        dup["opcode"] = int(L.Op.INV)
        g.batch_host(L.BatchType.invs, dup, mb, n_batches=1, stride=512, unique=True)
        assert g.take_error_flags() & 16
