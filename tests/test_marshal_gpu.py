"""The message-marshalling kernels (include/hermeskv_workload.h) one by one against numpy
restatements of the worker loop's wings callbacks (src/hermes/hermes_worker.c):

* ACKs   -- ack_skip_or_get_sender_id / ack_copy_and_modify_elem / ack_modify_elem_after_send
  (:69-118): an INV_SUCCESS INV answers with its 16-byte header as ST_OP_ACK from this machine, an
  OP_INV_ABORT with the whole element (when the ACK slot is op-sized); INV_SUCCESS, INV_ABORT and
  membership-change INVs become ST_EMPTY. (Other opcodes reach the reference's assert(0); the
  kernels send nothing for them.)
* VALs   -- val_skip_or_get_sender_id / val_copy_and_modify_elem / val_modify_elem_after_send
  (:122-157, assertions off as config.h:83 ships): every ACK element that is not ACK_SUCCESS, a
  membership change or empty sends its 16-byte header as ST_OP_VAL from this machine; all become
  ST_EMPTY.
* membership-change VALs -- memb_change_* (:162-203): ops in *_COMPLETE_SEND_VALS send a VAL and
  move to PUT_COMPLETE / RMW_COMPLETE / NEW (the key is the op's: the reference leaves the send
  slot's key as it was).
* packing and regrouping of the replica group's slabs (pure data movement).
Every flat, per-row and packed variant is compared byte for byte, inputs and outputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402

R = L.Resp
B = L.Bucket
OPC = {"INV_SUCCESS": int(R.INV_SUCCESS), "INV_ABORT": int(R.OP_INV_ABORT), "EMPTY": int(B.EMPTY),
       "MEMB": int(L.Op.MEMBERSHIP_CHANGE), "ACK_SUCCESS": int(R.ACK_SUCCESS),
       "LAST_ACK": int(R.LAST_ACK_SUCCESS), "OP_ACK": int(L.Op.ACK), "ACK": int(L.Op.ACK), "VAL": int(L.Op.VAL)}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _wl():
    from hermes_amd import replica_group  # noqa: F401  (argtypes of the group's kernels)
    from hermes_amd import workload as WL
    return WL


def _ack_ref(inv, ack_size, mid):
    """one INV element (bytes) -> (ACK bytes or None, INV after send)"""
    x = inv.copy()
    oc = int(x[8])
    y = None
    if oc == OPC["INV_SUCCESS"]:
        y = np.zeros(ack_size, np.uint8)
        y[:16] = x[:16]
        y[8], y[9] = OPC["ACK"], mid
    elif oc == OPC["INV_ABORT"] and ack_size >= len(x):
        y = x[:ack_size].copy()
        y[8], y[9] = OPC["INV_ABORT"], mid
    if oc in (OPC["INV_SUCCESS"], OPC["INV_ABORT"], OPC["MEMB"]):
        x[8] = OPC["EMPTY"]
    return y, x


def _val_ref(ack, mid):
    x = ack.copy()
    oc = int(x[8])
    y = None
    if oc not in (OPC["ACK_SUCCESS"], OPC["MEMB"], OPC["EMPTY"]):
        y = x[:16].copy()
        y[8], y[9] = OPC["VAL"], mid
    x[8] = OPC["EMPTY"]
    return y, x


def _random_elems(rng, n, esz, codes, p=None):
    a = rng.integers(0, 256, size=(n, esz), dtype=np.uint8)
    a[:, 8] = rng.choice(np.array(codes, np.uint8), size=n, p=p)
    return a


@pytest.mark.parametrize("op_size,ack_size", [(56, 16), (56, 56), (312, 312)])
def test_marshal_acks_flat_rows_aligned(op_size, ack_size):
    WL = _wl()
    _L = WL._L
    rng = np.random.default_rng(op_size + ack_size)
    mid = 5
    codes = [OPC["INV_SUCCESS"], OPC["INV_ABORT"], OPC["EMPTY"], OPC["MEMB"]]
    # flat: element i -> ACK slot i (ST_EMPTY where nothing is sent)
    n = 3000
    inv = _random_elems(rng, n, op_size, codes, [0.6, 0.15, 0.15, 0.1])
    d_inv, d_out = _dev(inv.reshape(-1)), torch.zeros(n * ack_size, dtype=torch.uint8, device="cuda")
    WL.check(_L.hkv_wl_marshal_acks(WL._ptr(d_inv), n, op_size, WL._ptr(d_out), ack_size, mid, None), "acks")
    torch.cuda.synchronize()
    got_out, got_inv = d_out.cpu().numpy().reshape(n, ack_size), d_inv.cpu().numpy().reshape(n, op_size)
    for i in range(n):
        y, x = _ack_ref(inv[i], ack_size, mid)
        assert np.array_equal(got_inv[i], x), i
        if y is None:
            assert got_out[i, 8] == OPC["EMPTY"], i
        else:
            assert np.array_equal(got_out[i, :len(y)], y), i
    # rows: [rows][C] with counts, ACKs compacted to the front of each row
    rows, C = 37, 64
    inv = _random_elems(rng, rows * C, op_size, codes, [0.6, 0.15, 0.15, 0.1])
    cnt = rng.integers(0, C + 1, size=rows).astype(np.int32)
    d_inv, d_cnt = _dev(inv.reshape(-1)), _dev(cnt)
    d_out = torch.zeros(rows * C * ack_size, dtype=torch.uint8, device="cuda")
    d_oc = torch.zeros(rows, dtype=torch.int32, device="cuda")
    WL.check(_L.hkv_wl_marshal_acks_rows(WL._ptr(d_inv), WL._ptr(d_cnt), rows, C, op_size, WL._ptr(d_out), ack_size,
                                         WL._ptr(d_oc), mid, None), "acks_rows")
    torch.cuda.synchronize()
    got_out = d_out.cpu().numpy().reshape(rows, C, ack_size)
    got_inv, got_oc = d_inv.cpu().numpy().reshape(rows, C, op_size), d_oc.cpu().numpy()
    inv = inv.reshape(rows, C, op_size)
    for r in range(rows):
        want = []
        for j in range(C):
            if j < cnt[r]:
                y, x = _ack_ref(inv[r, j], ack_size, mid)
                if y is not None:
                    want.append(y)
            else:
                x = inv[r, j]
            assert np.array_equal(got_inv[r, j], x), (r, j)
        assert got_oc[r] == len(want), r
        for k, y in enumerate(want):
            assert np.array_equal(got_out[r, k, :len(y)], y), (r, k)
    # aligned: [rows][width], ACK in the INV's position, ST_EMPTY past each row's count and where no ACK
    # goes, with ST_OP_MEMBERSHIP_CHANGE in byte 9 (hermes_skip_ack skips such a slot)
    d_inv = _dev(inv.reshape(-1))
    d_out = torch.zeros(rows * C * ack_size, dtype=torch.uint8, device="cuda")
    WL.check(_L.hkv_wl_marshal_acks_aligned(WL._ptr(d_inv), WL._ptr(d_cnt), rows, C, op_size, WL._ptr(d_out),
                                            ack_size, mid, None), "acks_aligned")
    torch.cuda.synchronize()
    got_out = d_out.cpu().numpy().reshape(rows, C, ack_size)
    for r in range(rows):
        for j in range(C):
            y = _ack_ref(inv[r, j], ack_size, mid)[0] if j < cnt[r] else None
            if y is None:
                assert got_out[r, j, 8] == OPC["EMPTY"] and got_out[r, j, 9] == OPC["MEMB"], (r, j)
            else:
                assert np.array_equal(got_out[r, j, :len(y)], y), (r, j)


@pytest.mark.parametrize("ack_size", [16, 56])
def test_vals_flat_rows_packed(ack_size):
    WL = _wl()
    _L = WL._L
    rng = np.random.default_rng(7 + ack_size)
    mid = 3
    codes = [OPC["LAST_ACK"], OPC["ACK_SUCCESS"], OPC["EMPTY"], OPC["MEMB"], OPC["OP_ACK"]]
    p = [0.3, 0.45, 0.1, 0.05, 0.1]
    n = 2500
    ack = _random_elems(rng, n, ack_size, codes, p)
    d_ack, d_out = _dev(ack.reshape(-1)), torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    WL.check(_L.hkv_wl_marshal_vals(WL._ptr(d_ack), n, ack_size, WL._ptr(d_out), mid, None), "vals")
    torch.cuda.synchronize()
    got_out, got_ack = d_out.cpu().numpy().reshape(n, 16), d_ack.cpu().numpy().reshape(n, ack_size)
    for i in range(n):
        y, x = _val_ref(ack[i], mid)
        assert np.array_equal(got_ack[i], x), i
        if y is None:
            assert got_out[i, 8] == OPC["EMPTY"], i
        else:
            assert np.array_equal(got_out[i], y), i
    # per-worker rows [W][stride] (counts), or packed (offsets): VALs compacted into [W][C]
    W, stride, C = 41, 90, 90
    cnt = rng.integers(0, stride + 1, size=W).astype(np.int32)
    ack = _random_elems(rng, W * stride, ack_size, codes, p).reshape(W, stride, ack_size)
    live = [ack[w, :cnt[w]] for w in range(W)]
    want = [[y for y in (_val_ref(e, mid)[0] for e in live[w]) if y is not None] for w in range(W)]
    for packed in (False, True):
        if packed:
            flat = np.concatenate(live).reshape(-1)
            off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
            d_ack, d_off = _dev(flat if flat.size else np.zeros(16, np.uint8)), _dev(off)
        else:
            d_ack, d_off = _dev(ack.reshape(-1)), None
        d_cnt = _dev(cnt)
        d_out = torch.zeros(W * C * 16, dtype=torch.uint8, device="cuda")
        d_vc = torch.zeros(W, dtype=torch.int32, device="cuda")
        WL.check(_L.hkv_wl_collect_vals(WL._ptr(d_ack), WL._ptr(d_cnt), W, stride, ack_size, WL._ptr(d_out), C,
                                        WL._ptr(d_vc), mid, None, WL._ptr(d_off) if packed else None, None),
                 "collect_vals")
        torch.cuda.synchronize()
        got_out, got_vc = d_out.cpu().numpy().reshape(W, C, 16), d_vc.cpu().numpy()
        for w in range(W):
            assert got_vc[w] == len(want[w]), (packed, w)
            for k, y in enumerate(want[w]):
                assert np.array_equal(got_out[w, k], y), (packed, w, k)
        got_ack = d_ack.cpu().numpy()
        if packed:
            assert (got_ack[: int(off[-1]) * ack_size].reshape(-1, ack_size)[:, 8] == OPC["EMPTY"]).all()
        else:
            g = got_ack.reshape(W, stride, ack_size)
            for w in range(W):
                assert (g[w, :cnt[w], 8] == OPC["EMPTY"]).all() and np.array_equal(g[w, cnt[w]:], ack[w, cnt[w]:])


def test_marshal_memb_vals():
    WL = _wl()
    _L = WL._L
    rng = np.random.default_rng(11)
    W, S, osz, C, mid = 23, 250, 56, 64, 2
    send = {int(R.PUT_COMPLETE_SEND_VALS): int(R.PUT_COMPLETE), int(B.RMW_COMPLETE_SEND_VALS): int(R.RMW_COMPLETE),
            int(B.REPLAY_COMPLETE_SEND_VALS): int(B.NEW)}
    states = np.array(list(send) + [int(B.IN_PROGRESS_PUT), int(R.GET_COMPLETE), int(B.NEW)], np.uint8)
    ops = rng.integers(0, 256, size=(W, S, osz), dtype=np.uint8)
    ops[:, :, 9] = rng.choice(states, size=(W, S), p=[0.06, 0.03, 0.03, 0.3, 0.38, 0.2])
    d_ops = _dev(ops.reshape(-1))
    d_out = torch.zeros(W * C * 16, dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(W, dtype=torch.int32, device="cuda")
    d_st = _dev(ops[:, :, 9].reshape(-1).copy())   # the state mirror follows the ops
    WL.check(_L.hkv_wl_marshal_memb_vals(WL._ptr(d_ops), W, S, osz, WL._ptr(d_out), C, WL._ptr(d_cnt), mid,
                                         WL._ptr(d_st), None), "memb_vals")
    torch.cuda.synchronize()
    got_ops = d_ops.cpu().numpy().reshape(W, S, osz)
    assert np.array_equal(d_st.cpu().numpy(), got_ops[:, :, 9].reshape(-1)), "state mirror differs"
    got_out, got_cnt = d_out.cpu().numpy().reshape(W, C, 16), d_cnt.cpu().numpy()
    for w in range(W):
        k = 0
        for j in range(S):
            x = ops[w, j].copy()
            st = int(x[9])
            if st in send:
                if k < C:
                    y = x[:16].copy()
                    y[8], y[9] = OPC["VAL"], mid
                    assert np.array_equal(got_out[w, k], y), (w, j)
                k += 1
                x[9] = send[st]
            assert np.array_equal(got_ops[w, j], x), (w, j)
        assert got_cnt[w] == min(k, C), w


def test_pack_and_regroup():
    """hkv_wl_pack_rows (rows -> one packed slab + offsets) and hkv_wl_regroup_aligned (peers'
    rows lined up with that slab -> per-worker batches, empty slots dropped, peer order)"""
    WL = _wl()
    _L = WL._L
    rng = np.random.default_rng(13)
    W, C, esz, P = 29, 40, 16, 3
    cnt = rng.integers(0, C + 1, size=W).astype(np.int32)
    rows = rng.integers(0, 256, size=(W, C, esz), dtype=np.uint8)
    d_rows, d_cnt = _dev(rows.reshape(-1)), _dev(cnt)
    d_pack = torch.zeros(W * C * esz, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(W + 1, dtype=torch.int32, device="cuda")
    WL.check(_L.hkv_wl_pack_rows(WL._ptr(d_rows), WL._ptr(d_cnt), W, C, esz, WL._ptr(d_pack), WL._ptr(d_off), None),
             "pack_rows")
    torch.cuda.synchronize()
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    assert np.array_equal(d_off.cpu().numpy(), off)
    want = np.concatenate([rows[w, :cnt[w]] for w in range(W)])
    assert np.array_equal(d_pack.cpu().numpy()[: off[-1] * esz].reshape(-1, esz), want)
    # the peers' answers, one row per peer lined up with the packed slab; some slots ST_EMPTY
    width = int(off[-1])
    ans = rng.integers(0, 256, size=(P, width, esz), dtype=np.uint8)
    ans[:, :, 8] = np.where(rng.random((P, width)) < 0.3, OPC["EMPTY"], OPC["ACK"])
    out_stride = P * C
    d_ans = _dev(ans.reshape(-1))
    d_out = torch.zeros(W * out_stride * esz, dtype=torch.uint8, device="cuda")
    d_oc = torch.zeros(W, dtype=torch.int32, device="cuda")
    WL.check(_L.hkv_wl_regroup_aligned(WL._ptr(d_ans), P, width, WL._ptr(d_off), WL._ptr(d_cnt), W, esz,
                                       WL._ptr(d_out), out_stride, WL._ptr(d_oc), None), "regroup_aligned")
    torch.cuda.synchronize()
    got, goc = d_out.cpu().numpy().reshape(W, out_stride, esz), d_oc.cpu().numpy()
    for w in range(W):
        keep = [ans[p, off[w] + j] for p in range(P) for j in range(cnt[w]) if ans[p, off[w] + j, 8] != OPC["EMPTY"]]
        assert goc[w] == len(keep), w
        for k, e in enumerate(keep):
            assert np.array_equal(got[w, k], e), (w, k)
