"""Host-side mirror of the reference's KVS interface, on top of libhermeskv.so.

Two ways in, matching the two halves of include/hermeskv.h:

* reference entry points -- `spacetime_init`, `spacetime_populate_fixed_len`,
  `hermes_batch_ops_to_KVS` -- same names, argument meaning and error behaviour as
  include/hermes/spacetime.h:211-230 (they call the exported C symbols: the drop-in path);
* `HermesKV`, one HBM-resident table per replica with the device fast path: many batches
  (one per virtual worker) concatenated into one launch on torch tensors, on torch's stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import layout as L
from .lib import ABI_VERSION, HkvBatchDesc, HkvConfig, Membership, check, raw

_L = raw()


def _membership_struct(mb: bytes) -> Membership:
    return Membership(int.from_bytes(bytes(mb[:8]).ljust(8, b"\0"), "little"))


# ---------------------------------------------------------------- reference entry points
def set_default_config(**kw) -> None:
    """hkv_set_default_config: must precede spacetime_init (e.g. machine_id, num_keys, rmw)."""
    cfg = make_config(**kw)
    check(_L.hkv_set_default_config(ctypes.byref(cfg)), "hkv_set_default_config")


def spacetime_init(instance_id: int) -> None:
    """spacetime.h:211 -- build and populate the default table in HBM."""
    _L.spacetime_init(int(instance_id))


def spacetime_populate_fixed_len(n: int, val_len: int) -> None:
    """spacetime.h:212."""
    _L.spacetime_populate_fixed_len(None, int(n), int(val_len))


def hermes_batch_ops_to_KVS(btype: int, op_array: np.ndarray, op_num: int, sizeof_op_elem: int,
                            curr_membership: bytes, node_suspected: list | None,
                            read_write_ops: np.ndarray | None, thread_id: int = 0) -> None:
    """spacetime.h:228-230 on host numpy arrays, mutated in place. `node_suspected` is a
    one-element list standing for the int* out-parameter (or None for NULL). As in the
    reference, read_write_ops must hold the table's rw_len (max_batch_size, 250) ops."""
    assert op_array.flags["C_CONTIGUOUS"]
    ns = ctypes.c_int(node_suspected[0] if node_suspected else -1)
    _L.hermes_batch_ops_to_KVS(int(btype), op_array.ctypes.data_as(ctypes.c_void_p), int(op_num),
                               int(sizeof_op_elem), _membership_struct(curr_membership),
                               ctypes.byref(ns) if node_suspected is not None else None,
                               read_write_ops.ctypes.data_as(ctypes.c_void_p) if read_write_ops is not None else None,
                               int(thread_id))
    if node_suspected is not None:
        node_suspected[0] = ns.value


# ---------------------------------------------------------------- tables
def make_config(num_keys: int = 1_000_000, num_bkts: int = 2 * 1024 * 1024, log_cap: int = 1 << 30,
                machine_id: int = 0, rmw: bool = False, big_objects: bool = False,
                extra_cache_lines: int = 0, device: int = 0, rw_len: int = 250, skew: int = 0) -> HkvConfig:
    """skew: hkv_config.skew_flags (SKEW_READ_COMPLETE | SKEW_WRITE_COALESCE, config.h:79-80)"""
    return HkvConfig(ABI_VERSION, machine_id, int(rmw), int(big_objects), int(extra_cache_lines), device, rw_len,
                     int(skew), num_keys, num_bkts, log_cap)


SKEW_READ_COMPLETE = 1    # ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS (include/hermeskv.h)
SKEW_WRITE_COALESCE = 2   # ENABLE_WRITE_COALESCE_TO_THE_SAME_KEY_IN_SAME_NODE


def sized_geometry(num_keys: int, sizes: L.Sizes = L.DEFAULT) -> tuple[int, int]:
    """Buckets and log capacity for `num_keys` (powers of two; about 2 keys per bucket as in
    the reference's 1M keys / 2^21 buckets, at most 2^27 buckets up to 2^28 keys and 2^29
    beyond (1B keys per replica: 32 GiB of index), and a log that never wraps)."""
    bkts = 1 << max(4, (2 * num_keys - 1).bit_length())
    need = num_keys * sizes.entry + sizes.kvs_value + 64
    cap = 1 << max(16, (need - 1).bit_length())
    return min(bkts, 1 << (27 if num_keys <= 1 << 28 else 29)), cap


BATCH_ENGINE = 1   # hkv_batch_desc.flags (include/hermeskv.h): the multi-kernel engine
BATCH_SMALL = 2    # the single-workgroup kernel (launches of at most 4096 elements)
BATCH_PACKED = 4   # INV / VAL batches back to back, d_counts = n_batches + 1 offsets
BATCH_UNIQUE = 8   # no key twice in the launch (INV batches: one pass)
BATCH_ROWS = 16    # with BATCH_UNIQUE: rows of one layout, element j of every row on one key


class HermesKV:
    """One HermesKV replica: a MICA-herd table in HBM plus the batch path on it."""

    default_flags = 0   # hkv_batch_desc.flags for every launch (tests pin one engine or the other)

    def __init__(self, num_keys: int | None = 1_000_000, num_bkts: int | None = None,
                 log_cap: int | None = None, machine_id: int = 0, rmw: bool = False,
                 big_objects: bool = False, extra_cache_lines: int = 0, device: int = 0,
                 rw_len: int = 250, populate: bool = True, skew: int = 0):
        self.sizes = L.Sizes(big_objects, extra_cache_lines if big_objects else 0)
        nk = num_keys or 0
        if num_bkts is None or log_cap is None:
            b, c = sized_geometry(max(nk, 1), self.sizes)
            num_bkts = num_bkts or b
            log_cap = log_cap or c
        self.cfg = make_config(nk, num_bkts, log_cap, machine_id, rmw, big_objects,
                               extra_cache_lines, device, rw_len, skew)
        self.skew = int(skew)
        self.device = device
        self.machine_id = machine_id
        self.rmw = rmw
        self.num_keys = nk
        h = ctypes.c_void_p()
        check(_L.hkv_table_create(ctypes.byref(self.cfg), ctypes.byref(h)), "hkv_table_create")
        self.h = h
        self._owned = True
        if populate and nk:
            self.populate(nk, self.sizes.kvs_value)

    @classmethod
    def default_table(cls) -> "HermesKV":
        """Non-owning view of the table the reference entry points use (spacetime_init)."""
        h = _L.hkv_default_table()
        if not h:
            raise RuntimeError("spacetime_init has not been called")
        self = cls.__new__(cls)
        self.h = ctypes.c_void_p(h)
        self._owned = False
        self.cfg = HkvConfig()
        check(_L.hkv_table_config(self.h, ctypes.byref(self.cfg)), "hkv_table_config")
        self.sizes = L.Sizes(bool(self.cfg.big_objects), self.cfg.extra_cache_lines if self.cfg.big_objects else 0)
        self.device, self.machine_id = self.cfg.device, self.cfg.machine_id
        self.rmw, self.num_keys = bool(self.cfg.rmw_enabled), self.cfg.num_keys
        self.skew = self.cfg.skew_flags
        return self

    def close(self) -> None:
        if getattr(self, "h", None) and getattr(self, "_owned", False):
            _L.hkv_table_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- setup
    def set_skew(self, skew: int) -> None:
        """hkv_table_set_skew: the table's skew optimisations from the next launch on"""
        check(_L.hkv_table_set_skew(self.h, int(skew)), "hkv_table_set_skew")
        self.cfg.skew_flags = int(skew)
        self.skew = int(skew)

    def populate(self, n: int, val_len: int) -> None:
        check(_L.hkv_table_populate(self.h, int(n), int(val_len)), "hkv_table_populate")

    @property
    def log_head(self) -> int:
        return _L.hkv_log_head(self.h)

    @property
    def evictions(self) -> int:
        return _L.hkv_num_index_evictions(self.h)

    # -- device fast path
    def batch(self, btype: int, elems: torch.Tensor, n_batches: int, stride: int, elem_size: int,
              membership: bytes, counts: torch.Tensor | None = None, rw: torch.Tensor | None = None,
              rw_stride_bytes: int = 0, node_suspected: torch.Tensor | None = None,
              stream: torch.cuda.Stream | None = None, offsets: torch.Tensor | None = None,
              state_out: torch.Tensor | None = None, opcode_in: torch.Tensor | None = None,
              patch: torch.Tensor | None = None, rw_state: torch.Tensor | None = None,
              unique: bool = False, rows: tuple[int, int, int] | None = None,
              ack_out: torch.Tensor | None = None, ack_out_size: int = 16,
              rw_opcodes: torch.Tensor | None = None) -> None:
        """Apply n_batches batches of one type, concatenated in `elems` (uint8, on the GPU),
        in concatenation order, asynchronously on `stream` (default: torch's current).
        offsets (INV / ACK / VAL batches): the batches stored back to back, batch b at elements
        [offsets[b], offsets[b+1]); `stride` is then the total (HKV_BATCH_PACKED). patch (local
        batches): 16 B per element of pending header writes (hkv_batch_desc.d_patch); rw_state (ACK
        batches): the read_write_ops' state-byte mirror, kept up to date by the completions. unique
        (INV batches): no key appears twice in the launch (HKV_BATCH_UNIQUE, one pass). rows (unique INV /
        ACK launches): (n_rows, row_stride, skip_row) -- n_rows launches of this layout, row r at element
        r * row_stride of elems, applied in row order in one pass (HKV_BATCH_ROWS; skip_row -1: none).
        ack_out (unique INV launches): every element's ACK as the worker's ACK callbacks make it,
        ack_out_size bytes each (hkv_batch_desc.d_ack_out); ACK rows launches: the VAL callbacks' output
        in the ACKs' positions. rw_opcodes (ACK batches): the
        read_write_ops' opcode mirror, one byte per slot (hkv_batch_desc.d_opcode_in): completions read the
        opcode there instead of the op."""
        assert elems.is_cuda and elems.dtype == torch.uint8
        total = stride if offsets is not None else n_batches * stride
        if rows is not None:
            assert unique and rows[0] >= 1 and (rows[0] == 1 or rows[1] >= total)
            assert elems.numel() >= ((rows[0] - 1) * rows[1] + total) * elem_size
        else:
            assert elems.numel() >= total * elem_size
        d = HkvBatchDesc()
        d.type = int(btype)
        d.n_batches = int(n_batches)
        d.stride = int(stride)
        d.elem_size = int(elem_size)
        d.flags = self.default_flags | (BATCH_UNIQUE if unique else 0)
        if rows is not None:
            d.flags |= BATCH_ROWS
            d.n_rows, d.row_stride, d.skip_row = int(rows[0]), int(rows[1]), int(rows[2])
        d.d_elems = elems.data_ptr()
        if state_out is not None:   # local batches: the mirror of each element's final state byte
            assert state_out.is_cuda and state_out.dtype == torch.uint8 and state_out.numel() >= n_batches * stride
            d.d_state_out = state_out.data_ptr()
        if opcode_in is not None:   # local batches: the caller's mirror of each element's opcode byte
            assert opcode_in.is_cuda and opcode_in.dtype == torch.uint8 and opcode_in.numel() >= n_batches * stride
            d.d_opcode_in = opcode_in.data_ptr()
        if rw_opcodes is not None:   # ACK batches: the read_write_ops' opcode mirror
            assert opcode_in is None and rw is not None and rw_opcodes.is_cuda and rw_opcodes.dtype == torch.uint8
            assert rw_opcodes.numel() >= n_batches * (rw_stride_bytes // self.sizes.op)
            d.d_opcode_in = rw_opcodes.data_ptr()
        if patch is not None:
            assert patch.is_cuda and patch.dtype == torch.uint8 and patch.numel() >= n_batches * stride * 16
            d.d_patch = patch.data_ptr()
        if rw_state is not None:
            assert rw_state.is_cuda and rw_state.dtype == torch.uint8
            d.d_rw_state = rw_state.data_ptr()
        if ack_out is not None:   # INV launches: the ACK callbacks; ACK rows launches: the VAL callbacks, per row
            span = total if rows is None else (rows[0] - 1) * rows[1] + total
            assert unique and ack_out.is_cuda and ack_out.dtype == torch.uint8 and ack_out.numel() >= span * ack_out_size
            d.d_ack_out = ack_out.data_ptr()
            d.ack_out_size = int(ack_out_size)
        if offsets is not None:
            assert counts is None and offsets.is_cuda and offsets.dtype == torch.int32
            assert offsets.numel() >= n_batches + 1
            d.flags |= BATCH_PACKED
            d.d_counts = offsets.data_ptr()
        if counts is not None:
            assert counts.is_cuda and counts.dtype == torch.int32 and counts.numel() >= n_batches
            d.d_counts = counts.data_ptr()
        if rw is not None:
            assert rw.is_cuda and rw.dtype == torch.uint8
            d.d_rw = rw.data_ptr()
            d.rw_stride_bytes = int(rw_stride_bytes)
        if node_suspected is not None:
            assert node_suspected.is_cuda and node_suspected.dtype == torch.int32
            d.d_node_suspected = node_suspected.data_ptr()
        for i, b in enumerate(membership[:8]):
            d.membership[i] = b
        s = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        check(_L.hkv_batch_async(self.h, ctypes.byref(d), ctypes.c_void_p(s)), "hkv_batch_async")

    def batch_host(self, btype: int, elems: np.ndarray, membership: bytes, rw: np.ndarray | None = None,
                   n_batches: int = 1, stride: int | None = None, counts: np.ndarray | None = None,
                   rw_stride_elems: int = 0, node_suspected: np.ndarray | None = None,
                   offsets: np.ndarray | None = None, unique: bool = False) -> None:
        """Round-trip numpy arrays through the device path (parity tests). offsets: packed INV /
        VAL batches (HKV_BATCH_PACKED), batch b = elems[offsets[b]:offsets[b+1]]."""
        dev = torch.device("cuda", self.device)
        if offsets is not None:
            t = torch.from_numpy(elems.view(np.uint8).reshape(-1).copy()).to(dev)
            to = torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int32)).to(dev)
            tn = torch.from_numpy(np.ascontiguousarray(node_suspected, dtype=np.int32)).to(dev) \
                if node_suspected is not None else None
            tr = torch.from_numpy(rw.view(np.uint8).reshape(-1).copy()).to(dev) if rw is not None else None
            self.batch(btype, t, n_batches, len(elems), elems.dtype.itemsize, membership, rw=tr,
                       rw_stride_bytes=rw_stride_elems * (rw.dtype.itemsize if rw is not None else 0),
                       node_suspected=tn, offsets=to, unique=unique)
            torch.cuda.synchronize(dev)
            elems.view(np.uint8).reshape(-1)[:] = t.cpu().numpy()
            if rw is not None:
                rw.view(np.uint8).reshape(-1)[:] = tr.cpu().numpy()
            if node_suspected is not None:
                node_suspected[:] = tn.cpu().numpy()
            return
        stride = len(elems) // n_batches if stride is None else stride
        esz = elems.dtype.itemsize
        t = torch.from_numpy(elems.view(np.uint8).reshape(-1).copy()).to(dev)
        # local launches also keep the state mirror (d_state_out), checked against the elements
        local = int(btype) in (int(L.BatchType.local_ops), int(L.BatchType.local_ops_after_membership_change))
        st = torch.full((n_batches * stride,), 0xEE, dtype=torch.uint8, device=dev) if local else None
        tc = torch.from_numpy(np.ascontiguousarray(counts, dtype=np.int32)).to(dev) if counts is not None else None
        tr = torch.from_numpy(rw.view(np.uint8).reshape(-1).copy()).to(dev) if rw is not None else None
        tn = torch.from_numpy(np.ascontiguousarray(node_suspected, dtype=np.int32)).to(dev) if node_suspected is not None else None
        self.batch(btype, t, n_batches, stride, esz, membership, tc, tr,
                   rw_stride_elems * (rw.dtype.itemsize if rw is not None else 0), tn, state_out=st, unique=unique)
        torch.cuda.synchronize(dev)
        elems.view(np.uint8).reshape(-1)[:] = t.cpu().numpy()
        if st is not None and not np.array_equal(st.cpu().numpy(),
                                                 elems.view(np.uint8).reshape(-1, esz)[: n_batches * stride, 9]):
            raise AssertionError("state mirror (d_state_out) differs from the elements' state bytes")
        if rw is not None:
            rw.view(np.uint8).reshape(-1)[:] = tr.cpu().numpy()
        if node_suspected is not None:
            node_suspected[:] = tn.cpu().numpy()

    def take_error_flags(self) -> int:
        """Internal-consistency flags raised by the device path since the last call (0 = none)."""
        v = ctypes.c_uint32(0)
        check(_L.hkv_take_error_flags(self.h, ctypes.byref(v)), "hkv_take_error_flags")
        return v.value

    def sync(self) -> None:
        check(_L.hkv_sync(self.h, None), "hkv_sync")

    # -- HBM image (reference byte layout)
    def index_bytes(self, offset: int = 0, nbytes: int | None = None) -> np.ndarray:
        nbytes = self.cfg.num_bkts * 64 - offset if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        check(_L.hkv_copy_index(self.h, out.ctypes.data_as(ctypes.c_void_p), offset, nbytes), "hkv_copy_index")
        return out

    def log_bytes(self, offset: int = 0, nbytes: int | None = None) -> np.ndarray:
        nbytes = self.cfg.log_cap - offset if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        check(_L.hkv_copy_log(self.h, out.ctypes.data_as(ctypes.c_void_p), offset, nbytes), "hkv_copy_log")
        return out

    def lookup_offset(self, key: int) -> int | None:
        """Log offset of a key's entry via the same 3-step lookup the batch path does."""
        key = int(key)
        bkt = (key & 0xFFFFFFFFFFFF) & (self.cfg.num_bkts - 1)
        slots = self.index_bytes(bkt * 64, 64).view("<u8")
        tag = key >> 48
        for s in slots:
            s = int(s)
            if (s & 1) and ((s >> 1) & 0x7FFFFF) == tag:
                off = s >> 24
                if self.log_head - off >= self.cfg.log_cap:
                    return None
                phys = off & (self.cfg.log_cap - 1)
                e = self.log_bytes(phys, 16).view("<u8")
                return phys if int(e[1]) == key else None
        return None

    def entry(self, key: int):
        off = self.lookup_offset(key)
        if off is None:
            return None
        return self.log_bytes(off, self.sizes.entry).view(L.entry_dtype(self.sizes))[0]

    def device_index(self) -> int:
        return _L.hkv_device_index(self.h)

    def device_log(self) -> int:
        return _L.hkv_device_log(self.h)


def hash_ids(ids: torch.Tensor, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """CityHash128(&id, 4).second for each uint32 id, on the GPU (mica_gen_keys)."""
    assert ids.is_cuda and ids.dtype == torch.int32
    out = torch.empty(ids.numel(), dtype=torch.int64, device=ids.device)
    s = (stream or torch.cuda.current_stream(ids.device)).cuda_stream
    check(_L.hkv_hash_ids(ctypes.c_void_p(ids.data_ptr()), ctypes.c_void_p(out.data_ptr()), ids.numel(),
                          ctypes.c_void_p(s)), "hkv_hash_ids")
    return out
