"""Shared test helpers: build op/message arrays and drive the known-answer scenario."""
from __future__ import annotations

import collections
import json
import os

import numpy as np
import pytest

from hermes_amd import layout as L

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def make_elems(spec: list, keys: np.ndarray, sizes: L.Sizes, msg: bool):
    dt = L.msg_dtype() if msg else L.op_dtype(sizes)
    a = np.zeros(len(spec), dtype=dt)
    for i, s in enumerate(spec):
        a[i]["key"] = keys[s["id"]]
        a[i]["opcode"] = int(getattr(L.Op, s["opcode"]))
        st = s.get("sender", int(L.Bucket.NEW))
        a[i]["sender" if msg else "state"] = st
        a[i]["ts_ver"] = s.get("ts_ver", 0)
        a[i]["ts_cid"] = s.get("ts_cid", 0)
        if not msg:
            if "value" in s:
                a[i]["value"][:] = ord(s["value"])
                a[i]["val_len"] = sizes.st_value >> sizes.shift
    return a


def check_fields(obj, expect: dict, what: str):
    for k, v in expect.items():
        if k in ("id", "index"):
            continue
        if k == "value":
            got = chr(int(obj["value"][0]))
            assert got == v, f"{what}: value {got!r} != {v!r}"
        elif k == "lwid":
            got = int(obj["rmw_lwid"]) >> 1
            assert got == v, f"{what}: lwid {got} != {v}"
        else:
            got = int(obj[k])
            assert got == v, f"{what}: {k} {got} != {v}"


def run_known_answers(engine, keys: np.ndarray):
    """engine: object with batch(btype, elems, membership, rw=None) and entry(key) -> entry record."""
    ka = load_golden("known_answers.json")
    cfg = ka["config"]
    mb = L.membership(cfg["machine_num"], cfg["machine_id"])
    step_elems = []
    for si, step in enumerate(ka["steps"]):
        btype = getattr(L.BatchType, step["batch"])
        msg = step["batch"] in ("acks", "vals")
        elems = make_elems(step["ops"], keys, L.DEFAULT, msg)
        rw = step_elems[step["rw_from_step"]] if "rw_from_step" in step else None
        engine.batch(btype, elems, mb, rw=rw)
        step_elems.append(elems)
        for j, exp in enumerate(step["expect_ops"]):
            check_fields(elems[j], exp, f"step {si} elem {j}")
        for exp in step.get("expect_rw", []):
            check_fields(rw[exp["index"]], exp, f"step {si} rw {exp['index']}")
        if "expect_key" in step:
            e = engine.entry(keys[step["expect_key"]["id"]])
            check_fields(e, step["expect_key"], f"step {si} key")
    miss = make_elems([{"id": i, "opcode": "GET"} for i in ka["always_miss_ids"]], keys, L.DEFAULT, False)
    engine.batch(L.BatchType.local_ops, miss, mb)
    assert (miss["state"] == int(L.Resp.MISS)).all()


def ack_callbacks(invs, ack_size, machine_id):
    """The worker's ACK callbacks (src/hermes/hermes_worker.c:69-118) on INV elements after their
    batch: (ACKs [n][ack_size], ST_EMPTY at byte 8 where none is sent; the INVs after send).
    INV_SUCCESS answers with its header as ST_OP_ACK from this machine, OP_INV_ABORT with the whole
    element when the ACK slot holds it; INV_SUCCESS, INV_ABORT and membership-change INVs become
    ST_EMPTY."""
    n, esz = invs.shape
    oc = invs[:, 8]
    acks = np.zeros((n, ack_size), np.uint8)
    acks[:, 8] = int(L.Bucket.EMPTY)
    ok = oc == int(L.Resp.INV_SUCCESS)
    acks[ok, :16] = invs[ok, :16]
    acks[ok, 8] = int(L.Op.ACK)
    if ack_size >= esz:
        ab = oc == int(L.Resp.OP_INV_ABORT)
        acks[ab, :esz] = invs[ab]
        acks[ab, 8] = int(L.Resp.OP_INV_ABORT)
        ok = ok | ab
    acks[ok, 9] = machine_id
    after = invs.copy()
    done = np.isin(oc, [int(L.Resp.INV_SUCCESS), int(L.Resp.OP_INV_ABORT), int(L.Op.MEMBERSHIP_CHANGE)])
    after[done, 8] = int(L.Bucket.EMPTY)
    return acks, after


def val_callbacks(acks: np.ndarray, live: np.ndarray, machine_id: int):
    """The worker's VAL callbacks (hermes_worker.c:122-157, assertions off as shipped) over ACK results
    in place: an element whose opcode is not ACK_SUCCESS, MEMBERSHIP_CHANGE or EMPTY is sent as a VAL
    (its first 16 bytes, opcode ST_OP_VAL, sender = this machine: val_copy_and_modify_elem); every
    non-empty element then leaves empty (val_skip_or_get_sender_id, val_modify_elem_after_send). Holes
    (live False) are no elements. Returns (VALs in the ACKs' positions, opcode ST_EMPTY where none;
    the ACKs after)."""
    oc = acks[:, 8]
    send = live & ~np.isin(oc, [int(L.Resp.ACK_SUCCESS), int(L.Op.MEMBERSHIP_CHANGE), int(L.Bucket.EMPTY)])
    vals = np.zeros((len(acks), 16), np.uint8)
    vals[:, 8] = int(L.Bucket.EMPTY)
    vals[send] = acks[send, :16]
    vals[send, 8] = int(L.Op.VAL)
    vals[send, 9] = machine_id
    after = acks.copy()
    after[live & (oc != int(L.Bucket.EMPTY)), 8] = int(L.Bucket.EMPTY)
    return vals, after


class Mirror:
    """Runs every batch launch of a device table on an oracle twin and compares."""

    def __init__(self, g, o, name):
        self.g, self.o, self.name = g, o, name
        self.launches = 0
        self.codes = collections.Counter()   # (batch type, "in8"/"out8"/"out9", code) over live elements
        self._orig = g.batch
        g.batch = self.batch

    def _count(self, btype, tag, col, arr, n_batches, stride, elem_size, counts):
        v = arr.reshape(n_batches, stride, elem_size)[:, :, col]
        if counts is not None:
            v = v[np.arange(stride)[None, :] < counts[:, None]]
        vals, cnt = np.unique(v, return_counts=True)
        for x, c in zip(vals.tolist(), cnt.tolist()):
            self.codes[(int(btype), tag, x)] += c

    def batch(self, btype, elems, n_batches, stride, elem_size, membership, counts=None, rw=None,
              rw_stride_bytes=0, node_suspected=None, stream=None, offsets=None, state_out=None, opcode_in=None,
              patch=None, rw_state=None, unique=False, rows=None, ack_out=None,
              ack_out_size=16, rw_opcodes=None):
        import torch
        if rw_opcodes is not None:   # the ACK launch's opcode mirror must be every read_write_ops slot's byte 8
            torch.cuda.synchronize()
            nrw = n_batches * (rw_stride_bytes // self.g.sizes.op)
            assert np.array_equal(rw_opcodes[:nrw].cpu().numpy(),
                                  rw[: nrw * self.g.sizes.op].cpu().numpy().reshape(nrw, self.g.sizes.op)[:, 8]), \
                "read_write_ops opcode mirror is stale"
        if rows is not None:
            return self._rows(btype, elems, n_batches, stride, elem_size, membership, offsets, stream, rw,
                              rw_stride_bytes, rw_state, rows, rw_opcodes, ack_out)
        if offsets is not None:
            return self._packed(btype, elems, n_batches, stride, elem_size, membership, offsets, stream, rw,
                                rw_stride_bytes, rw_state, unique, ack_out, ack_out_size, rw_opcodes)
        torch.cuda.synchronize()
        n = n_batches * stride * elem_size
        vt = np.dtype((np.void, elem_size))
        e_in = elems[:n].cpu().numpy().copy()
        if patch is not None:   # the pending refill the launch applies first (hkv_batch_desc.d_patch)
            from tests.test_workload_gpu import _apply_patches
            e_in = _apply_patches(e_in, patch[: n_batches * stride * 16].cpu().numpy(), elem_size,
                                  self.g.sizes.st_value)
        e_in = e_in.view(vt)
        e_orig = e_in.copy()
        c_in = counts[:n_batches].cpu().numpy().copy() if counts is not None else None
        if opcode_in is not None:   # the caller's opcode mirror must be every element's opcode byte
            assert np.array_equal(opcode_in[: n_batches * stride].cpu().numpy(),
                                  np.frombuffer(e_in.tobytes(), np.uint8).reshape(-1, elem_size)[:, 8])
        self._count(btype, "in8", 8, np.frombuffer(e_in.tobytes(), np.uint8), n_batches, stride, elem_size, c_in)
        rw_in = rw_op = None
        if rw is not None:
            rw_in = rw.cpu().numpy().copy().view(np.dtype((np.void, self.g.sizes.op)))
            st_before = rw_in.view(np.uint8).reshape(-1, self.g.sizes.op)[:, 9].copy()
        rws_in = rw_state.cpu().numpy().copy() if rw_state is not None else None
        self._orig(btype, elems, n_batches, stride, elem_size, membership, counts, rw, rw_stride_bytes,
                   node_suspected, stream, state_out=state_out, opcode_in=opcode_in, patch=patch, rw_state=rw_state,
                   unique=unique, rw_opcodes=rw_opcodes, ack_out=ack_out, ack_out_size=ack_out_size)
        torch.cuda.synchronize()
        self.o.batch_multi(int(btype), e_in, n_batches, stride, c_in, membership, rw_in,
                           rw_stride_bytes // self.g.sizes.op if rw is not None else 0)
        what = f"{self.name} launch {self.launches} type {int(btype)}"
        if ack_out is not None:   # the launch also ran the ACK callbacks on its applied INVs (d_ack_out)
            eo = e_in.view(np.uint8).reshape(-1, elem_size)
            j = np.arange(n_batches * stride) % stride
            live = j < np.repeat(c_in, stride) if c_in is not None else np.ones(n_batches * stride, bool)
            idx = np.nonzero(live)[0]
            want_acks, after = ack_callbacks(eo[idx].copy(), ack_out_size, self.g.machine_id)
            eo[idx] = after       # an answered INV leaves as after its send
            got_acks = ack_out[: n_batches * stride * ack_out_size].cpu().numpy().reshape(-1, ack_out_size)[idx]
            sent = want_acks[:, 8] != L.Bucket.EMPTY
            span = np.where(want_acks[:, 8] == int(L.Resp.OP_INV_ABORT), elem_size, 16)
            cmp = sent[:, None] & (np.arange(ack_out_size)[None, :] < span[:, None])
            if not ((got_acks == want_acks) | ~cmp).all() or not (got_acks[~sent, 8] == int(L.Bucket.EMPTY)).all():
                bad = np.nonzero(((got_acks != want_acks) & cmp).any(axis=1)
                                 | (~sent & (got_acks[:, 8] != int(L.Bucket.EMPTY))))[0]
                pytest.fail(f"{what}: fused ACKs differ at {len(bad)} elements, first {idx[bad[:8]]}")
        got = elems[:n].cpu().numpy()
        self._count(btype, "out8", 8, got, n_batches, stride, elem_size, c_in)
        self._count(btype, "out9", 9, got, n_batches, stride, elem_size, c_in)
        if not np.array_equal(got, e_in.view(np.uint8)):
            bad = np.nonzero(got != e_in.view(np.uint8))[0]
            rows = np.unique(bad // elem_size)[:4]
            show = "; ".join(f"elem {r}: in {e_orig.view(np.uint8).reshape(-1, elem_size)[r][:24].tolist()} "
                             f"dev {got.reshape(-1, elem_size)[r][:24].tolist()} "
                             f"oracle {e_in.view(np.uint8).reshape(-1, elem_size)[r][:24].tolist()}" for r in rows)
            # every element of the first bad element's key: index, opcode, state in / dev / oracle
            eo = e_orig.view(np.uint8).reshape(-1, elem_size)
            k0 = eo[rows[0], :8].tobytes()
            same = np.nonzero((eo[:, :8] == eo[rows[0], :8]).all(axis=1))[0][:24]
            gg, oo = got.reshape(-1, elem_size), e_in.view(np.uint8).reshape(-1, elem_size)
            show += f" || key {k0.hex()} elems " + " ".join(
                f"{j}:{eo[j, 8]}/{eo[j, 9]}->{gg[j, 9]}|{oo[j, 9]}" for j in same)
            pytest.fail(f"{what}: elements differ at {len(bad)} bytes, first elems {np.unique(bad // elem_size)[:8]}"
                        f" -- {show}")
        if rw is not None:
            rw_op = rw.cpu().numpy()
            assert np.array_equal(rw_op, rw_in.view(np.uint8)), f"{what}: read_write_ops differ"
            self._check_rw_state(rw_state, rws_in, st_before, rw_op.reshape(-1, self.g.sizes.op)[:, 9], what)
        self._check_log(what)
        assert np.array_equal(self.g.index_bytes(), self.o.index_bytes()), f"{what}: index differs"
        assert self.g.take_error_flags() == 0, f"{what}: device consistency flags"
        if state_out is not None:   # the local batch's state mirror: every element's state byte
            mirror = state_out[: n_batches * stride].cpu().numpy()
            assert np.array_equal(mirror, got.reshape(-1, elem_size)[:, 9]), f"{what}: state mirror differs"
        self.launches += 1

    def _check_log(self, what):
        """the whole log against the oracle's"""
        gl, ol = self.g.log_bytes(), self.o.log_bytes()[: self.g.cfg.log_cap]
        if not np.array_equal(gl, ol):
            bad = np.nonzero(gl != ol)[0]
            e = self.g.sizes.entry
            pytest.fail(f"{what}: log differs in entries {np.unique(bad // e)[:8]}, "
                        f"bytes-in-entry {np.unique(bad % e)[:16]}")

    def _check_rw_state(self, rw_state, rws_in, st_before, st_after, what):
        """d_rw_state: every completion the launch wrote into read_write_ops is in the mirror too, so a
        mirror that matched the ops' state bytes before the launch still matches them after it"""
        if rw_state is None:
            return
        n = min(len(st_before), len(rws_in))
        assert np.array_equal(rws_in[:n], st_before[:n]), f"{what}: the caller's state mirror was already stale"
        assert np.array_equal(rw_state.cpu().numpy()[:n], st_after[:n]), f"{what}: read_write_ops state mirror differs"

    def _rows(self, btype, elems, n_batches, total, elem_size, membership, offsets, stream, rw, rw_stride_bytes,
              rw_state, rows, rw_opcodes=None, ack_out=None):
        """An HKV_BATCH_ROWS launch: the oracle applies row after row (skip row excepted), each row's
        batches without their holes (opcode 0); the device's rows must equal them, holes untouched. ack_out
        (ACK launches): the VALs the launch made must be val_callbacks() of the oracle's results."""
        import torch
        torch.cuda.synchronize()
        n_rows, row_stride, skip = rows
        assert offsets is not None, "the tests' row launches are packed"
        off = offsets[: n_batches + 1].cpu().numpy().astype(np.int64)
        assert off[0] == 0 and off[-1] <= total
        bat = np.repeat(np.arange(n_batches), np.diff(off))
        nl = int(off[-1])   # elements past the last offset are in no batch (and must stay untouched)
        flat_all = elems.cpu().numpy().copy()
        rw_in = rw.cpu().numpy().copy().view(np.dtype((np.void, self.g.sizes.op))) if rw is not None else None
        st_before = rw_in.view(np.uint8).reshape(-1, self.g.sizes.op)[:, 9].copy() if rw is not None else None
        rws_in = rw_state.cpu().numpy().copy() if rw_state is not None else None
        ins = {}
        for r in range(n_rows):
            if r == skip:
                continue
            flat = flat_all[r * row_stride * elem_size:(r * row_stride + total) * elem_size].reshape(total, elem_size)
            ins[r] = flat.copy()
        self._orig(btype, elems, n_batches, total, elem_size, membership, rw=rw, rw_stride_bytes=rw_stride_bytes,
                   stream=stream, offsets=offsets, rw_state=rw_state, unique=True, rows=rows, rw_opcodes=rw_opcodes,
                   ack_out=ack_out)
        torch.cuda.synchronize()
        got_all = elems.cpu().numpy()
        vals_all = ack_out.cpu().numpy() if ack_out is not None else None
        what = f"{self.name} launch {self.launches} type {int(btype)} (rows)"
        for r, flat in ins.items():
            live = flat[:, 8] != 0
            live[nl:] = False
            cnt = np.bincount(bat[live[:nl]], minlength=n_batches).astype(np.int32)
            width = max(int(cnt.max()), 1) if n_batches else 1
            rws_ = np.zeros((n_batches, width, elem_size), np.uint8)
            pos = np.arange(width)[None, :] < cnt[:, None]
            rws_[pos] = flat[live]
            self._count(btype, "in8", 8, rws_.reshape(-1), n_batches, width, elem_size, cnt)
            e_in = rws_.reshape(-1).view(np.dtype((np.void, elem_size))).copy()
            self.o.batch_multi(int(btype), e_in, n_batches, width, cnt, membership, rw_in,
                               rw_stride_bytes // self.g.sizes.op if rw is not None else 0)
            want = flat.copy()
            want[live] = e_in.view(np.uint8).reshape(n_batches, width, elem_size)[pos]
            if vals_all is not None:   # the VAL callbacks over the row's results
                vwant, after = val_callbacks(want[:nl], live[:nl], self.g.machine_id)
                want[:nl] = after
                vgot = vals_all[r * row_stride * 16:(r * row_stride + nl) * 16].reshape(nl, 16)
                if not np.array_equal(vgot, vwant):
                    bad = np.nonzero((vgot != vwant).any(axis=1))[0]
                    pytest.fail(f"{what}: row {r} VALs differ at {len(bad)} positions, first {bad[:8]}: "
                                f"dev {vgot[bad[0]].tolist()} want {vwant[bad[0]].tolist()}")
                self.codes[(int(btype), "vals_sent", 0)] += int((vwant[:, 8] == int(L.Op.VAL)).sum())
            got = got_all[r * row_stride * elem_size:(r * row_stride + total) * elem_size].reshape(total, elem_size)
            grow = np.zeros_like(rws_)
            grow[pos] = got[live]
            self._count(btype, "out8", 8, grow.reshape(-1), n_batches, width, elem_size, cnt)
            self._count(btype, "out9", 9, grow.reshape(-1), n_batches, width, elem_size, cnt)
            if not np.array_equal(got, want):
                bad = np.nonzero((got != want).any(axis=1))[0]
                pytest.fail(f"{what}: row {r} elements differ at {len(bad)} elements, first {bad[:8]}")
        if rw is not None:
            rw_op = rw.cpu().numpy()
            assert np.array_equal(rw_op, rw_in.view(np.uint8)), f"{what}: read_write_ops differ"
            self._check_rw_state(rw_state, rws_in, st_before, rw_op.reshape(-1, self.g.sizes.op)[:, 9], what)
        self._check_log(what)
        assert np.array_equal(self.g.index_bytes(), self.o.index_bytes()), f"{what}: index differs"
        assert self.g.take_error_flags() == 0, f"{what}: device consistency flags"
        self.launches += 1

    def _packed(self, btype, elems, n_batches, total, elem_size, membership, offsets, stream, rw=None,
                rw_stride_bytes=0, rw_state=None, unique=False, ack_out=None, ack_out_size=16,
                rw_opcodes=None):
        """A packed (HKV_BATCH_PACKED) INV / ACK / VAL launch: the oracle applies the same batches
        laid out in rows; the device's packed output must equal the oracle's rows packed again."""
        import torch
        torch.cuda.synchronize()
        off = offsets[: n_batches + 1].cpu().numpy().astype(np.int64)
        cnt = np.diff(off).astype(np.int32)
        assert off[0] == 0 and off[-1] == total and (cnt >= 0).all()
        width = max(int(cnt.max()), 1) if n_batches else 1
        flat = elems[: total * elem_size].cpu().numpy().copy().reshape(total, elem_size)
        rows = np.zeros((n_batches, width, elem_size), np.uint8)
        pos = np.arange(width)[None, :] < cnt[:, None]
        rows[pos] = flat
        self._count(btype, "in8", 8, rows.reshape(-1), n_batches, width, elem_size, cnt)
        rw_in = rw.cpu().numpy().copy().view(np.dtype((np.void, self.g.sizes.op))) if rw is not None else None
        st_before = rw_in.view(np.uint8).reshape(-1, self.g.sizes.op)[:, 9].copy() if rw is not None else None
        rws_in = rw_state.cpu().numpy().copy() if rw_state is not None else None
        self._orig(btype, elems, n_batches, total, elem_size, membership, rw=rw, rw_stride_bytes=rw_stride_bytes,
                   stream=stream, offsets=offsets, rw_state=rw_state, unique=unique, ack_out=ack_out,
                   ack_out_size=ack_out_size, rw_opcodes=rw_opcodes)
        torch.cuda.synchronize()
        e_in = rows.reshape(-1).view(np.dtype((np.void, elem_size))).copy()
        self.o.batch_multi(int(btype), e_in, n_batches, width, cnt, membership, rw_in,
                           rw_stride_bytes // self.g.sizes.op if rw is not None else 0)
        want = e_in.view(np.uint8).reshape(n_batches, width, elem_size)[pos]
        got = elems[: total * elem_size].cpu().numpy().reshape(total, elem_size)
        what = f"{self.name} launch {self.launches} type {int(btype)} (packed)"
        grow = np.zeros_like(rows)
        grow[pos] = got
        if ack_out is not None:   # the launch also ran the ACK callbacks on its output (d_ack_out)
            grow[pos] = want
            want = want.copy()
            got_acks = ack_out[: total * ack_out_size].cpu().numpy().reshape(total, ack_out_size)
            want_acks, want = ack_callbacks(want, ack_out_size, self.g.machine_id)
            sent = want_acks[:, 8] != L.Bucket.EMPTY
            # the bytes an ACK carries: its 16-byte header, a whole INV-abort element (the callbacks
            # leave the rest of an op-sized ACK slot as it was)
            span = np.where(want_acks[:, 8] == int(L.Resp.OP_INV_ABORT), elem_size, 16)
            cmp = sent[:, None] & (np.arange(ack_out_size)[None, :] < span[:, None])
            if not ((got_acks == want_acks) | ~cmp).all() or not (got_acks[~sent, 8] == int(L.Bucket.EMPTY)).all():
                bad = np.nonzero(((got_acks != want_acks) & cmp).any(axis=1)
                                 | (~sent & (got_acks[:, 8] != int(L.Bucket.EMPTY))))[0]
                pytest.fail(f"{what}: fused ACKs differ at {len(bad)} elements, first {bad[:8]}")
        self._count(btype, "out8", 8, grow.reshape(-1), n_batches, width, elem_size, cnt)
        self._count(btype, "out9", 9, grow.reshape(-1), n_batches, width, elem_size, cnt)
        if not np.array_equal(got, want):
            bad = np.nonzero((got != want).any(axis=1))[0]
            pytest.fail(f"{what}: elements differ at {len(bad)} elements, first {bad[:8]}")
        if rw is not None:
            rw_op = rw.cpu().numpy()
            assert np.array_equal(rw_op, rw_in.view(np.uint8)), f"{what}: read_write_ops differ"
            self._check_rw_state(rw_state, rws_in, st_before, rw_op.reshape(-1, self.g.sizes.op)[:, 9], what)
        self._check_log(what)
        assert np.array_equal(self.g.index_bytes(), self.o.index_bytes()), f"{what}: index differs"
        assert self.g.take_error_flags() == 0, f"{what}: device consistency flags"
        self.launches += 1
