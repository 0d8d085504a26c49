"""A scripted protocol scenario that drives hermes_batch_ops_to_KVS through its rare branches, with
the expected per-element outcome of every step written out (hermesKV.c line by line):

  OUT_OF_GROUP INVs, node_suspected, INV-aborts sent and received, RMW_ABORT, the ST_EMPTY read of
  an INVALID key whose write is still in flight, LAST_ACK_SUCCESS completing PUTs, RMWs and GET
  replays (read_write_ops -> PUT_COMPLETE / RMW_COMPLETE / ST_NEW), write replays after a member
  fails, and the after-membership-change completions PUT/RMW/REPLAY_COMPLETE_SEND_VALS.

`run_scripted(runner, keys, sizes, rmw)` applies every step through `runner(btype, elems, mb,
rw=None, node_suspected=None)` (in place) and checks the outcomes. tests/test_oracle.py runs it on
the oracle alone; tests/test_gpu_parity.py on the device path and the oracle side by side.
"""
from __future__ import annotations

import numpy as np

from hermes_amd import layout as L

R = L.Resp
B = L.Bucket
O = L.Op

# key ids (none of them is one of the 1M table's populate misses)
K = {n: 100 + 7 * i for i, n in enumerate(
    ["put_last", "get_ok", "put_memb", "put_oog", "rmw_memb", "rmw_abort", "rmw_last", "inv4",
     "inv_abort", "rmw_inv", "rmw_memb2", "replay_ack"])}
MISSING_KEY = 0x1234_5678_9ABC_DEF1


def _ops(sizes, rows, keys):
    a = np.zeros(len(rows), dtype=L.op_dtype(sizes))
    for i, r in enumerate(rows):
        name, oc = r[0], r[1]
        a[i]["key"] = MISSING_KEY if name is None else keys[K[name]]
        a[i]["opcode"] = int(oc)
        a[i]["state"] = int(r[2]) if len(r) > 2 else int(B.NEW)
        if len(r) > 3:
            a[i]["ts_ver"], a[i]["ts_cid"] = r[3]
        if oc in (O.PUT, O.RMW):
            a[i]["value"][:] = ord("p") + i
            a[i]["val_len"] = sizes.st_value >> sizes.shift
        if oc == O.RMW:
            a[i]["flags"] = 1
    return a


def _invs(sizes, rows, keys):
    a = np.zeros(len(rows), dtype=L.op_dtype(sizes))
    for i, (name, oc, sender, ts, rmw_flag) in enumerate(rows):
        a[i]["key"] = keys[K[name]]
        a[i]["opcode"] = int(oc)
        a[i]["state"] = sender
        a[i]["ts_ver"], a[i]["ts_cid"] = ts
        a[i]["val_len"] = sizes.st_value >> sizes.shift
        a[i]["flags"] = rmw_flag
        a[i]["value"][:] = ord("A") + i
    return a


def _acks(sizes, rmw, rows, keys):
    a = np.zeros(len(rows), dtype=L.op_dtype(sizes) if rmw else L.msg_dtype())
    for i, (name, oc, sender, ts) in enumerate(rows):
        a[i]["key"] = keys[K[name]]
        a[i]["opcode"] = int(oc)
        a[i]["state" if rmw else "sender"] = sender
        a[i]["ts_ver"], a[i]["ts_cid"] = ts
        if rmw:
            a[i]["val_len"] = sizes.st_value >> sizes.shift
            a[i]["value"][:] = ord("z")
            a[i]["flags"] = 1 if oc == R.OP_INV_ABORT else 0
    return a


def _check(what, got, want):
    got = [int(x) for x in got]
    want = [int(x) for x in want]
    assert got == want, f"{what}: got {got}, want {want}"


def run_scripted(runner, keys, sizes, rmw: bool) -> set:
    """Returns the set of (batch type, outcome code) the scenario produced."""
    seen = set()
    mb5 = L.membership(5, 0)                 # g 0x1F, w_ack_init 0xE1
    mb4 = L.membership(5, 0, alive=0x0F)     # node 4 failed
    mb3 = L.membership(5, 0, alive=0x07)     # nodes 3, 4 failed
    ts2 = (2, 0)                             # a fresh key's first local write (2 for RMWs and non-RMW builds)
    tsw = (4, 0) if rmw else (2, 0)          # a plain PUT in an RMW build steps by 4 (hermesKV.c:129-134)
    rmw_or_get = (lambda n: (n, O.RMW)) if rmw else (lambda n: ("get_ok", O.GET))

    # ---- 1. local batch (all 5 machines alive)
    l1 = _ops(sizes, [("put_last", O.PUT), ("put_last", O.GET), ("put_last", O.PUT), ("get_ok", O.GET),
                      ("put_memb", O.PUT), ("put_oog", O.PUT), (None, O.GET), rmw_or_get("rmw_memb"),
                      rmw_or_get("rmw_abort"), rmw_or_get("rmw_memb"), rmw_or_get("rmw_last"),
                      rmw_or_get("rmw_inv"), rmw_or_get("rmw_memb2")], keys)
    runner(L.BatchType.local_ops, l1, mb5)
    rmw_ok = R.RMW_SUCCESS if rmw else R.GET_COMPLETE
    _check("local 1", l1["state"], [R.PUT_SUCCESS, R.GET_STALL, R.PUT_STALL, R.GET_COMPLETE, R.PUT_SUCCESS,
                                    R.PUT_SUCCESS, R.MISS, rmw_ok, rmw_ok, R.RMW_STALL if rmw else R.GET_COMPLETE,
                                    rmw_ok, rmw_ok, rmw_ok])
    seen |= {(0, int(x)) for x in l1["state"]}
    # the worker broadcasts the INVs (inv_modify_elem_after_send, hermes_worker.c:30-50)
    l1["state"][l1["state"] == R.PUT_SUCCESS] = B.IN_PROGRESS_PUT
    l1["state"][l1["state"] == R.RMW_SUCCESS] = B.IN_PROGRESS_RMW

    # ---- 2. incoming INVs
    inv_rows = [("put_oog", O.INV, 1, tsw, 0),            # equal ts, key in WRITE -> OUT_OF_GROUP
                ("inv4", O.INV, 4, (2, 4), 0),            # VALID -> INVALID, last writer 4
                ("get_ok", O.MEMBERSHIP_CHANGE, 3, (0, 0), 0),   # skipped; node_suspected := value[0]
                ("replay_ack", O.INV, 4, (2, 4), 0)]
    if rmw:
        inv_rows += [("rmw_abort", O.INV, 3, (2, 3), 0),  # beats the in-flight RMW (2,0): INVALID
                     ("inv_abort", O.INV, 2, (0, 2), 1),  # RMW INV below (0,255): INV-abort
                     ("rmw_inv", O.INV, 4, (2, 4), 0)]    # in-flight RMW key -> INVALID, obi kept
    i1 = _invs(sizes, inv_rows, keys)
    i1["value"][2][0] = 4
    ns = np.full(1, -1, np.int32)
    runner(L.BatchType.invs, i1, mb5, node_suspected=ns)
    want = [L.INV_OUT_OF_GROUP, R.INV_SUCCESS, O.MEMBERSHIP_CHANGE, R.INV_SUCCESS]
    if rmw:
        want += [R.INV_SUCCESS, R.OP_INV_ABORT, R.INV_SUCCESS]
    _check("invs", i1["opcode"], want)
    assert int(ns[0]) == 4, f"node_suspected {int(ns[0])}"
    seen |= {(2, int(x)) for x in i1["opcode"]} | {("node_suspected", 4)}
    if rmw:   # the INV-abort carries the key's local state (hermes_local_state_to_op)
        ab = i1[5]
        assert (int(ab["ts_ver"]), int(ab["ts_cid"]), int(ab["state"])) == (0, 255, 2), ab
        assert int(ab["value"][0]) == ord("a") + K["inv_abort"] % 20

    # ---- 3. ACKs (read_write_ops = batch 1)
    ack_rows = [("put_last", O.ACK, s, tsw) for s in (1, 2, 3, 4)] + \
               [("put_memb", O.ACK, s, tsw) for s in (1, 2, 3)]
    if rmw:
        ack_rows += [("rmw_memb", O.ACK, s, ts2) for s in (1, 2, 3)] + \
                    [("rmw_last", O.ACK, s, ts2) for s in (1, 2, 3, 4)] + \
                    [("rmw_memb", R.OP_INV_ABORT, 2, (2, 2))] + \
                    [("rmw_memb2", O.ACK, s, ts2) for s in (1, 2, 3)]
    a1 = _acks(sizes, rmw, ack_rows, keys)
    runner(L.BatchType.acks, a1, mb5, rw=l1)
    want = [R.ACK_SUCCESS] * 3 + [R.LAST_ACK_SUCCESS] + [R.ACK_SUCCESS] * 3
    if rmw:
        want += [R.ACK_SUCCESS] * 3 + [R.ACK_SUCCESS] * 3 + [R.LAST_ACK_SUCCESS] + [R.ACK_SUCCESS] * 4
    _check("acks", a1["opcode"], want)
    seen |= {(3, int(x)) for x in a1["opcode"]}
    assert int(l1["state"][0]) == R.PUT_COMPLETE
    seen.add(("rw", int(l1["state"][0])))
    if rmw:
        assert int(l1["state"][10]) == R.RMW_COMPLETE
        seen.add(("rw", int(l1["state"][10])))

    # ---- 4. node 4 fails: after-membership-change batch over batch 1
    runner(L.BatchType.local_ops_after_membership_change, l1, mb4)
    want = [R.PUT_COMPLETE, R.GET_STALL, R.PUT_STALL, R.GET_COMPLETE, R.PUT_COMPLETE_SEND_VALS,
            B.IN_PROGRESS_PUT, R.MISS]
    if rmw:   # rmw_memb went INVALID through the INV-abort: it completes without VALs
        want += [R.RMW_COMPLETE, B.IN_PROGRESS_RMW, R.RMW_STALL, R.RMW_COMPLETE, B.IN_PROGRESS_RMW,
                 B.RMW_COMPLETE_SEND_VALS]
    else:
        want += [R.GET_COMPLETE] * 6
    _check("after membership change", l1["state"], want)
    seen |= {(1, int(x)) for x in l1["state"][[4, 7, 12]]}

    # ---- 5. local batch under the new membership: replays, RMW abort, EMPTY read
    l2 = _ops(sizes, [("inv4", O.GET), ("rmw_abort", O.RMW, B.IN_PROGRESS_RMW, ts2) if rmw else ("get_ok", O.GET),
                      ("rmw_inv", O.GET) if rmw else ("get_ok", O.GET), ("put_last", O.GET),
                      ("replay_ack", O.GET)], keys)
    runner(L.BatchType.local_ops, l2, mb4)
    _check("local 2", l2["state"], [R.REPLAY_SUCCESS, R.RMW_ABORT if rmw else R.GET_COMPLETE,
                                    B.EMPTY if rmw else R.GET_COMPLETE, R.GET_COMPLETE, R.REPLAY_SUCCESS])
    assert (int(l2["ts_ver"][0]), int(l2["ts_cid"][0])) == (2, 4)   # replays carry the key's ts
    seen |= {(0, int(x)) for x in l2["state"]}
    l2["state"][l2["state"] == R.REPLAY_SUCCESS] = B.IN_PROGRESS_REPLAY

    # ---- 6. ACKs of the replays: one completes (GET replay -> read_write_op NEW), one waits
    a2 = _acks(sizes, rmw, [("inv4", O.ACK, 1, (2, 4)), ("inv4", O.ACK, 2, (2, 4))] +
               [("replay_ack", O.ACK, s, (2, 4)) for s in (1, 2, 3)], keys)
    runner(L.BatchType.acks, a2, mb4, rw=l2)
    _check("acks 2", a2["opcode"], [R.ACK_SUCCESS] * 4 + [R.LAST_ACK_SUCCESS])
    assert int(l2["state"][4]) == B.NEW
    seen.add(("rw", int(l2["state"][4])))

    # ---- 7. node 3 fails too: the waiting replay completes
    runner(L.BatchType.local_ops_after_membership_change, l2, mb3)
    assert int(l2["state"][0]) == B.REPLAY_COMPLETE_SEND_VALS, int(l2["state"][0])
    seen.add((1, int(l2["state"][0])))

    # ---- 8. VALs
    v = _acks(L.DEFAULT, False, [("inv4", O.VAL, 4, (2, 4)), ("put_oog", O.VAL, 1, tsw)], keys)
    runner(L.BatchType.vals, v, mb3)
    _check("vals", v["opcode"], [R.VAL_SUCCESS] * 2)
    seen |= {(4, int(x)) for x in v["opcode"]}
    return seen


def required_outcomes(rmw: bool) -> set:
    """Every outcome code hermes_batch_ops_to_KVS can emit in this build (LAST_ACK_NO_BCAST is
    rewritten to ACK_SUCCESS before it leaves hermes_exec_ack, hermesKV.c:671-672)."""
    req = {(0, R.GET_COMPLETE), (0, R.GET_STALL), (0, R.PUT_SUCCESS), (0, R.PUT_STALL), (0, R.MISS),
           (0, R.REPLAY_SUCCESS), (1, R.PUT_COMPLETE_SEND_VALS), (1, B.REPLAY_COMPLETE_SEND_VALS),
           (2, R.INV_SUCCESS), (2, L.INV_OUT_OF_GROUP), ("node_suspected", 4), (3, R.ACK_SUCCESS),
           (3, R.LAST_ACK_SUCCESS), ("rw", R.PUT_COMPLETE), ("rw", B.NEW), (4, R.VAL_SUCCESS)}
    if rmw:
        req |= {(0, R.RMW_SUCCESS), (0, R.RMW_STALL), (0, R.RMW_ABORT), (0, B.EMPTY), (1, R.RMW_COMPLETE),
                (1, B.RMW_COMPLETE_SEND_VALS), (2, R.OP_INV_ABORT), ("rw", R.RMW_COMPLETE)}
    return {(a, int(b)) for a, b in req}


# ---------------------------------------------------------------- skew optimisations
SK = {"hot": 500, "rep": 507, "trunc": 514}


def _sk_ops(sizes, rows, keys):
    """rows: (key name, opcode, (ts_ver, ts_cid)); state NEW"""
    a = np.zeros(len(rows), dtype=L.op_dtype(sizes))
    for i, (name, oc, ts) in enumerate(rows):
        a[i]["key"] = keys[SK[name]]
        a[i]["opcode"] = int(oc)
        a[i]["state"] = int(B.NEW)
        a[i]["ts_ver"], a[i]["ts_cid"] = ts
        if oc == O.PUT:
            a[i]["value"][:] = ord("p") + i
            a[i]["val_len"] = sizes.st_value >> sizes.shift
    return a


def run_scripted_skew(runner, keys, sizes) -> set:
    """The reference's skew optimisations (skew_flags 3: ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS
    and ENABLE_WRITE_COALESCE_TO_THE_SAME_KEY_IN_SAME_NODE, config.h:79-80) on a 3-machine group,
    outcomes written out from hermesKV.c:196-356: a stalled GET records the key's timestamp when its
    own is (0, 0) and completes once the version is two above it; a stalled PUT records the key's
    version (16 bits) when its own version is 0 -- not in REPLAY -- and completes (PUT_COMPLETE) once
    that 16-bit version is two above its own. Returns (batch type, code) outcomes."""
    seen = set()
    mb = L.membership(3, 0)
    # ---- 1. local: the first PUT of `hot` writes (2, 0); the rest stall behind it
    l1 = _sk_ops(sizes, [("hot", O.PUT, (0, 0)), ("hot", O.GET, (0, 0)), ("hot", O.PUT, (0, 0)),
                         ("hot", O.PUT, (1, 0)), ("hot", O.GET, (0, 7)), ("trunc", O.PUT, (0, 0))], keys)
    runner(L.BatchType.local_ops, l1, mb)
    _check("skew local 1", l1["state"], [R.PUT_SUCCESS, R.GET_STALL, R.PUT_STALL, R.PUT_STALL, R.GET_COMPLETE,
                                         R.PUT_SUCCESS])
    _check("skew local 1 ts", l1["ts_ver"], [2, 2, 2, 1, 0, 2])
    _check("skew local 1 cid", l1["ts_cid"][:2], [0, 0])   # the GET recorded the key's (2, 0)
    seen |= {(0, int(x)) for x in l1["state"]}
    l1["state"][l1["state"] == R.PUT_SUCCESS] = B.IN_PROGRESS_PUT
    # ---- 2. INVs: peer 1 beats hot's write; rep is written by node 4 (not a member); trunc jumps
    #         past 2^16 (its version's low 16 bits are 4)
    inv = np.zeros(3, dtype=L.op_dtype(sizes))
    for i, (name, snd, ts) in enumerate([("hot", 1, (2, 1)), ("rep", 4, (2, 4)), ("trunc", 1, (0x10004, 1))]):
        inv[i]["key"] = keys[SK[name]]
        inv[i]["opcode"] = int(O.INV)
        inv[i]["state"] = snd
        inv[i]["ts_ver"], inv[i]["ts_cid"] = ts
        inv[i]["val_len"] = sizes.st_value >> sizes.shift
        inv[i]["value"][:] = ord("I") + i
    runner(L.BatchType.invs, inv, mb)
    _check("skew invs", inv["opcode"], [R.INV_SUCCESS] * 3)
    # ---- 3. ACKs of hot's write: completes (INVALID_WRITE -> INVALID)
    a = np.zeros(2, dtype=L.msg_dtype())
    a["key"] = keys[SK["hot"]]
    a["opcode"] = int(O.ACK)
    a["sender"] = [1, 2]
    a["ts_ver"], a["ts_cid"] = 2, 0
    runner(L.BatchType.acks, a, mb, rw=l1)
    _check("skew acks", a["opcode"], [R.ACK_SUCCESS] * 2)
    assert int(l1["state"][0]) == R.PUT_COMPLETE
    # ---- 4. retries and new ops: hot is INVALID (writer 1 alive) at (2, 1), rep INVALID (writer 4
    #         gone), trunc INVALID_WRITE at (0x10004, 1)
    l2 = _sk_ops(sizes, [("hot", O.GET, (2, 0)),      # INVALID, writer alive: stalls, 3 < 2 no
                         ("hot", O.PUT, (2, 0)),      # INVALID, no write in flight: writes (4, 0)
                         ("hot", O.PUT, (1, 0)),      # WRITE: 2 < 4 -> coalesced, PUT_COMPLETE
                         ("hot", O.GET, (2, 0)),      # WRITE: 3 < 4 -> GET_COMPLETE
                         ("hot", O.GET, (0, 0)),      # WRITE: records (4, 0)
                         ("hot", O.PUT, (0, 0)),      # WRITE: records 4
                         ("rep", O.GET, (0, 0)),      # write replay (REPLAY_SUCCESS, ts (2, 4))
                         ("rep", O.PUT, (0, 0)),      # REPLAY: no record, stays 0
                         ("rep", O.GET, (0, 0)),      # REPLAY: records (2, 4)
                         ("rep", O.PUT, (3, 0)),      # REPLAY: 4 < 2 no
                         ("trunc", O.PUT, (0, 0)),    # INVALID_WRITE: records 0x10004 & 0xFFFF = 4
                         ("trunc", O.PUT, (5, 0)),    # 6 < 4 (16 bits) no
                         ("trunc", O.PUT, (1, 0)),    # 2 < 4 -> PUT_COMPLETE
                         ("trunc", O.GET, (0, 0)),    # records (0x10004, 1)
                         ("trunc", O.GET, (5, 0))],   # reads compare 32 bits: 6 < 0x10004 -> complete
                 keys)
    runner(L.BatchType.local_ops, l2, mb)
    _check("skew local 2", l2["state"], [R.GET_STALL, R.PUT_SUCCESS, R.PUT_COMPLETE, R.GET_COMPLETE, R.GET_STALL,
                                         R.PUT_STALL, R.REPLAY_SUCCESS, R.PUT_STALL, R.GET_STALL, R.PUT_STALL,
                                         R.PUT_STALL, R.PUT_STALL, R.PUT_COMPLETE, R.GET_STALL, R.GET_COMPLETE])
    _check("skew local 2 ts", l2["ts_ver"], [2, 4, 1, 2, 4, 4, 2, 0, 2, 3, 4, 5, 1, 0x10004, 5])
    _check("skew local 2 cid", l2["ts_cid"][[4, 6, 8, 13]], [0, 4, 4, 1])
    seen |= {(0, int(x)) for x in l2["state"]}
    return seen
