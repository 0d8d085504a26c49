"""Pins the CPU restatement (oracle/) before it is trusted as the parity checker.

1. CityHash128 against vectors produced by the reference's own city.c (tests/golden/cityhash_ref.json,
   made by tools/make_golden.py from oracle/_ref), and live against oracle/_ref when it is built.
2. hermes_batch_ops_to_KVS semantics against the reference outputs recorded in SURVEY.md section 4
   (tests/golden/known_answers.json).
"""
import numpy as np
import pytest

from hermes_amd import layout as L
from oracle import oracle as O
from tests.helpers import load_golden, run_known_answers


def test_cityhash_matches_reference_vectors():
    g = load_golden("cityhash_ref.json")
    for v in g["key_ids_le32"]:
        f, s = O.cityhash128(int(v["id"]).to_bytes(4, "little"))
        assert (f, s) == (int(v["first"]), int(v["second"])), v["id"]
    for v in g["short_strings"]:
        f, s = O.cityhash128(bytes.fromhex(v["hex"]))
        assert (f, s) == (int(v["first"]), int(v["second"])), v["hex"]


def test_cityhash_live_reference_when_built():
    r = O.reference_cityhash128(b"\x05\x00\x00\x00")
    if r is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(1)
    for i in rng.integers(0, 2**31, size=2000):
        b = int(i).to_bytes(4, "little")
        assert O.cityhash128(b) == O.reference_cityhash128(b)


def test_gen_keys_matches_scalar():
    keys = O.gen_keys(1000)
    for i in (0, 1, 5, 999):
        assert keys[i] == O.cityhash128(i.to_bytes(4, "little"))[1]


class _OracleEngine:
    def __init__(self, kv):
        self.kv = kv

    def batch(self, btype, elems, mb, rw=None):
        self.kv.batch(btype, elems, mb, rw=rw)

    def entry(self, key):
        off = self.kv.lookup(int(key))
        assert off is not None
        return self.kv.log_bytes()[off:off + L.DEFAULT.entry].view(L.entry_dtype())[0]


@pytest.fixture(scope="module")
def table_1m():
    ka = load_golden("known_answers.json")["config"]
    kv = O.OracleKVS(ka["num_bkts"], ka["log_cap"], machine_id=ka["machine_id"])
    kv.populate(ka["num_keys"], ka["val_len"])
    return kv, O.gen_keys(ka["num_keys"])


def test_known_answers(table_1m):
    kv, keys = table_1m
    run_known_answers(_OracleEngine(kv), keys)


def test_exactly_three_misses_at_1m():
    ka = load_golden("known_answers.json")
    c = ka["config"]
    kv = O.OracleKVS(c["num_bkts"], c["log_cap"])
    kv.populate(c["num_keys"], c["val_len"])
    keys = O.gen_keys(c["num_keys"])
    ops = np.zeros(c["num_keys"], dtype=L.op_dtype())
    ops["key"] = keys
    ops["opcode"] = int(L.Op.GET)
    ops["state"] = int(L.Bucket.NEW)
    for b in range(0, len(ops), 250):
        kv.batch(L.BatchType.local_ops, ops[b:b + 250], L.membership(3, 0))
    miss = np.nonzero(ops["state"] == int(L.Resp.MISS))[0].tolist()
    assert miss == ka["always_miss_ids"]
    assert (ops["state"][ops["state"] != int(L.Resp.MISS)] == int(L.Resp.GET_COMPLETE)).all()
    # value = 'a' + id % 20 (spacetime.c:58), val_len 30 after populate
    ok = ops["state"] == int(L.Resp.GET_COMPLETE)
    ids = np.arange(c["num_keys"])
    assert (ops["value"][ok, 0] == (ord("a") + ids[ok] % 20)).all()
    assert (ops["val_len"][ok] == 30).all()


def test_big_object_val_len_quirks():
    """SURVEY 7 bit-exact quirks: uint8 val_len arithmetic with SHIFT_BITS 3 (spacetime.h:263-273)."""
    kv = O.OracleKVS(1 << 12, 1 << 24, big_objects=True, extra_cache_lines=4, rmw=True)
    sz = L.BIG
    kv.populate(1000, sz.kvs_value)
    keys = O.gen_keys(1000)
    ops = np.zeros(2, dtype=L.op_dtype(sz))
    ops["key"] = keys[[3, 4]]
    ops["opcode"] = int(L.Op.GET)
    ops["state"] = int(L.Bucket.NEW)
    kv.batch(L.BatchType.local_ops, ops, L.membership(3, 0))
    assert (ops["state"] == int(L.Resp.GET_COMPLETE)).all()
    assert (ops["val_len"] == 244).all()


@pytest.mark.parametrize("rmw,big", [(False, False), (True, False), (True, True)])
def test_scripted_rare_outcomes_oracle(rmw, big):
    """tests/scripted.py on the oracle alone: every branch outcome it expects (written out from
    hermesKV.c) happens, and together they cover every code the batch function can emit."""
    from tests.scripted import required_outcomes, run_scripted
    sz = L.BIG if big else L.DEFAULT
    kv = O.OracleKVS(1 << 12, 1 << 22, machine_id=0, rmw=rmw, big_objects=big, extra_cache_lines=4 if big else 0)
    kv.populate(1000, sz.kvs_value)

    def runner(btype, elems, mb, rw=None, node_suspected=None):
        if node_suspected is not None:
            node_suspected[0] = kv.batch(btype, elems, mb, rw=rw)
        else:
            kv.batch(btype, elems, mb, rw=rw)

    seen = run_scripted(runner, O.gen_keys(1000), sz, rmw)
    missing = required_outcomes(rmw) - seen
    assert not missing, f"not produced: {sorted(missing, key=str)}"


@pytest.mark.parametrize("big", [False, True])
def test_scripted_skew_optimisations_oracle(big):
    """tests/scripted.py's skew scenario on the oracle (skew_flags 3): read completion and write
    coalescing outcomes written out from hermesKV.c:196-356, incl. the 16-bit version of the
    write path and the REPLAY exception."""
    from tests.scripted import run_scripted_skew
    sz = L.BIG if big else L.DEFAULT
    kv = O.OracleKVS(1 << 12, 1 << 22, machine_id=0, big_objects=big, extra_cache_lines=4 if big else 0, skew=3)
    kv.populate(1000, sz.kvs_value)
    seen = run_scripted_skew(lambda bt, e, mb, rw=None, node_suspected=None: kv.batch(bt, e, mb, rw=rw),
                             O.gen_keys(1000), sz)
    assert (0, int(L.Resp.PUT_COMPLETE)) in seen and (0, int(L.Resp.GET_COMPLETE)) in seen


def test_skew_flags_off_keep_stalls_oracle():
    """The same first batch without the flags: every op behind the write stalls (the default build)."""
    from tests.scripted import SK, _sk_ops
    kv = O.OracleKVS(1 << 12, 1 << 22, machine_id=0)
    kv.populate(1000, L.DEFAULT.kvs_value)
    keys = O.gen_keys(1000)
    l1 = _sk_ops(L.DEFAULT, [("hot", L.Op.PUT, (0, 0)), ("hot", L.Op.GET, (0, 0)), ("hot", L.Op.PUT, (0, 0)),
                             ("hot", L.Op.GET, (0, 7))], keys)
    kv.batch(L.BatchType.local_ops, l1, L.membership(3, 0))
    assert [int(x) for x in l1["state"]] == [int(L.Resp.PUT_SUCCESS), int(L.Resp.GET_STALL), int(L.Resp.PUT_STALL),
                                             int(L.Resp.GET_STALL)]
    assert [int(x) for x in l1["ts_ver"]] == [2, 0, 0, 0]
    assert SK["hot"] < 1000
