"""Device-resident protocol rounds for many virtual workers (one replica), built from the
batch path plus the worker loop's refill and marshalling (include/hermeskv_workload.h).

One `Round.step()` is one iteration of run_worker's loop (hermes_worker.c:438-546) for every
virtual worker at once: local batch -> INV broadcast -> incoming INV batch -> ACK batch ->
incoming VAL batch -> refill (which counts committed ops, inline-util.h:189-217).
Peers are either virtual (this module synthesises their ACKs and pre-generates their INVs
and VALs) or real GPUs exchanging slabs over RCCL (hermes_amd.replica_group).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import layout as L
from .kvs import HermesKV
from .lib import check, raw

_L = raw()
_P = ctypes.c_void_p


class HkvZipf(ctypes.Structure):
    _fields_ = [("theta", ctypes.c_double), ("zetan", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eta", ctypes.c_double), ("half_pow", ctypes.c_double), ("n", ctypes.c_uint64)]


_L.hkv_wl_gen_trace.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(HkvZipf),
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, _P]
_L.hkv_wl_refill.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                             _P, _P, _P, ctypes.c_int32, _P, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32, _P, _P,
                             _P, _P]
_L.hkv_wl_fold_counters.argtypes = [_P, _P]
_L.hkv_wl_refill_st.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                _P, _P, ctypes.c_int32, _P, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _P, _P]
_L.hkv_wl_refill_plan.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, _P, _P,
                                  ctypes.c_int32, _P, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _P, _P]
_L.hkv_wl_marshal_invs.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, _P, ctypes.c_uint32, _P]
_L.hkv_wl_marshal_invs_cap.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32, _P,
                                       ctypes.c_uint32, _P, _P, _P]
_L.hkv_wl_marshal_acks.argtypes = [_P, ctypes.c_int64, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32, _P]
_L.hkv_wl_marshal_memb_vals.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32, _P,
                                        ctypes.c_uint32, _P, _P]
_L.hkv_wl_max_to_host.argtypes = [_P, ctypes.c_int32, _P, _P]
_L.hkv_wl_marshal_vals.argtypes = [_P, ctypes.c_int64, ctypes.c_uint32, _P, ctypes.c_uint32, _P]
_L.hkv_wl_collect_vals.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32,
                                   _P, ctypes.c_uint32, _P, _P, _P]
_L.hkv_wl_peer_acks_pm.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_uint32,
                                   ctypes.c_int32, _P, _P, ctypes.c_int32, _P, ctypes.c_uint32, _P, _P]
_L.hkv_wl_collect_vals_blocks.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32,
                                          _P, ctypes.c_uint32, _P, _P, ctypes.c_int32, _P]
_L.hkv_wl_peer_acks.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_uint32,
                                ctypes.c_int32, _P, _P, ctypes.c_int32, _P, ctypes.c_uint32, _P, _P]
_L.hkv_wl_peer_round_scratch.restype = ctypes.c_size_t
_L.hkv_wl_peer_round_scratch.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
_L.hkv_wl_gen_peer_round.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(HkvZipf),
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, _P, _P]
_L.hkv_wl_peer_ts.argtypes = [_P, _P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P,
                              ctypes.c_uint32, _P]
_L.hkv_wl_marshal_invs_credits.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_int32,
                                           _P, ctypes.c_uint32, _P, _P, ctypes.c_int32, _P]
_L.hkv_wl_peer_acks_queue.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, ctypes.c_uint32,
                                      ctypes.c_int32, _P, _P, _P, _P, ctypes.c_int32, _P, ctypes.c_uint32, _P]
_L.hkv_wl_vals_credit.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, _P, ctypes.c_int32,
                                  _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, _P]
_L.hkv_wl_ack_offsets.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P]
_L.hkv_wl_pack_rows.argtypes = [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _P, _P, _P]
_L.hkv_wl_peer_locate.argtypes = [_P, _P, ctypes.c_int64, ctypes.c_uint32, _P, _P]
_L.hkv_wl_peer_ts_at.argtypes = [_P, _P, _P, _P, ctypes.c_int64, ctypes.c_uint32, _P, ctypes.c_uint32, _P]
_L.hkv_wl_refill_plan_peer_ts.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, _P, _P,
                                          ctypes.c_int32, _P, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _P, _P, _P, _P,
                                          _P, ctypes.c_int64, ctypes.c_uint32, _P, ctypes.c_uint32, _P]
_L.hkv_wl_peer_ts_words.restype = ctypes.c_uint64
_L.hkv_wl_peer_ts_words.argtypes = [_P]


REFILL_ALL = 1      # hkv_wl_refill flags (include/hermeskv_workload.h)
READ_TS_RESET = 2
COALESCE_HOT = 4
HOT_KEYS = 100      # COALESCE_N_HOTTEST_KEYS, config.h:78


def refill_flags(kvs: HermesKV, retry: bool, coalesce_hot: bool = False) -> int:
    """hkv_wl_refill flags for a policy: refill_ops' retry (the reference) or a fresh batch per
    round; GET timestamps reset when the table completes stalled reads (the reference ties both to
    ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS); hot-request coalescing on request."""
    f = 0 if retry else REFILL_ALL
    if kvs.skew & 1:   # SKEW_READ_COMPLETE
        f |= READ_TS_RESET
    if coalesce_hot:
        f |= COALESCE_HOT
    return f


def slots_per_worker(write_permille: int, rmw_permille: int = 0, batch: int = 250) -> int:
    """INV slots per worker and round (the send credits): the mean number of writes in a
    250-op batch plus 8 standard deviations, rounded up to 8, at most the batch. Writes beyond
    it stay in PUT_SUCCESS and go out in a later round (counted in `held`)."""
    p = min(1.0, write_permille / 1000.0)
    mean = batch * p
    sd = math.sqrt(batch * p * (1 - p))
    c = int(math.ceil((mean + 8 * sd + 1) / 8.0) * 8)
    return max(8, min(batch, c))


def zipf_params(n: int, theta: float) -> HkvZipf:
    """Constants of the Gray et al. / YCSB Zipfian generator over ids [0, n)."""
    if theta <= 0:
        return HkvZipf(0.0, 0.0, 0.0, 0.0, 0.0, n)
    zetan = 0.0
    chunk = 10_000_000
    for lo in range(1, n + 1, chunk):
        i = np.arange(lo, min(n, lo + chunk - 1) + 1, dtype=np.float64)
        zetan += float(np.sum(i ** -theta))
    zeta2 = 1.0 + 2.0 ** -theta
    alpha = 1.0 / (1.0 - theta)
    eta = (1.0 - (2.0 / n) ** (1.0 - theta)) / (1.0 - zeta2 / zetan)
    return HkvZipf(theta, zetan, alpha, eta, 1.0 + 0.5 ** theta, n)


def _ptr(t: torch.Tensor | None):
    return _P(t.data_ptr()) if t is not None else None


def init_mirrors(ops: torch.Tensor, op_size: int, states: torch.Tensor):
    """The state mirror of freshly written ops; from then on the round's kernels keep it (local launch,
    marshals, ACK launches, refill plan)."""
    states.copy_(ops.view(-1, op_size)[:, 9])


class CommitAudit:
    """How the ops a round commits completed (diagnostics: run only in untimed steps).

    refill_ops counts GET_COMPLETE, PUT_COMPLETE and RMW_COMPLETE alike (inline-util.h:189-217),
    but under the opt-in skew optimisations (config.h:79-80) two of them can complete without
    doing what the name says:
    * hermes_complete_hot_read_optimization (hermesKV.c:224-238) completes a stalled GET without
      copying a value. Its val_len stays 0 (refill_ops zeroes a GET's, inline-util.h:276), where
      hermes_read_actions (:240-246) sets the entry's;
    * hermes_complete_coalesced_write (:209-221) completes a stalled PUT in the local batch,
      without a write of its own, against the 16-bit version in its ts. That version was either
      recorded by this PUT at its first stall (its slot's ts.version was 0 when refill_ops put it
      there) or inherited from the slot's previous op, since refill_ops never resets a PUT's
      timestamp (:260-276).
    A PUT's own write completes in the ACK batch (or the after-membership-change batch), never in
    the local batch. Provenance is known only for PUTs refilled while the audit runs: PUT_COMPLETEs
    of older PUTs are counted under `put_coalesced_unknown`."""

    FIELDS = ("get_value", "get_no_value", "put_own", "put_coalesced_recorded", "put_coalesced_inherited",
              "put_coalesced_unknown", "rmw", "other")

    def __init__(self, rnd):
        self.r = rnd
        n = rnd.ops.numel() // rnd.op
        dev = rnd.ops.device
        self.prov = torch.full((n,), 3, dtype=torch.uint8, device=dev)   # 3 unknown, 1 recorded, 2 inherited
        self.after_local = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.acc = torch.zeros(len(self.FIELDS), dtype=torch.int64, device=dev)
        self.counting = False          # False: provenance tracking only (the first audited round)
        self.rounds = 0

    def _view(self):
        return self.r.ops.view(-1, self.r.op)

    def pre_local(self):
        """before the local launch: the provenance of every slot refilled for this round"""
        ops = self._view()
        patch = getattr(self.r, "patch", None)
        if getattr(self.r, "fused", False) and patch is not None:
            p = patch.view(-1, 16)
            fresh, oc = p[:, 14] == 1, p[:, 8]
        else:
            fresh, oc = ops[:, 9] == int(L.Bucket.NEW), ops[:, 8]
        tsv = ops[:, 12:16].contiguous().view(torch.int32).view(-1)
        put = fresh & (oc == int(L.Op.PUT))
        self.prov = torch.where(put, torch.where(tsv != 0, 2, 1).to(torch.uint8),
                                torch.where(fresh, torch.zeros_like(self.prov), self.prov))

    def post_local(self):
        ops = self._view()
        st, oc, vl = ops[:, 9], ops[:, 8], ops[:, 10]
        self.after_local.copy_(st)
        if not self.counting:
            return
        get_c = (oc == int(L.Op.GET)) & (st == int(L.Resp.GET_COMPLETE))
        put_c = st == int(L.Resp.PUT_COMPLETE)
        self.acc[0] += (get_c & (vl != 0)).sum()
        self.acc[1] += (get_c & (vl == 0)).sum()
        self.acc[3] += (put_c & (self.prov == 1)).sum()
        self.acc[4] += (put_c & (self.prov == 2)).sum()
        self.acc[5] += (put_c & (self.prov >= 3)).sum()

    def end(self):
        """after the round, before the refill counts it"""
        if not self.counting:
            self.counting = True
            return
        st = self._view()[:, 9]
        put_c = st == int(L.Resp.PUT_COMPLETE)
        self.acc[2] += (put_c & (self.after_local != int(L.Resp.PUT_COMPLETE))).sum()
        self.acc[6] += (st == int(L.Resp.RMW_COMPLETE)).sum()
        self.acc[7] += (st == int(L.Op.MEMBERSHIP_COMPLETE)).sum()
        self.rounds += 1

    def result(self, committed: int | None = None) -> dict:
        """per-round means; `committed`: the refill's commit count over the same rounds (the sum
        of the breakdown must equal it)"""
        v = self.acc.cpu().tolist()
        d = dict(zip(self.FIELDS, v))
        total = sum(v)
        strict = d["get_value"] + d["put_own"] + d["put_coalesced_recorded"] + d["rmw"] + d["other"]
        n = max(self.rounds, 1)
        out = {"rounds": self.rounds, "per_round": {k: x / n for k, x in d.items()},
               "committed_per_round": total / n, "committed_strict_per_round": strict / n,
               "strict_fraction": strict / total if total else None}
        if committed is not None:
            out["refill_committed_per_round"] = committed / n
            out["consistent"] = committed == total
        return out


def _s(stream=None):
    return _P((stream or torch.cuda.current_stream()).cuda_stream)


def patchable(sizes: L.Sizes) -> bool:
    """Whether a local launch takes refill patches (hkv_batch_desc.d_patch) without a pass of its own over the
    ops: ops of at most 64 B (k_local_pre / k_local_fused) or, for bigger ones, values of at most 320 B with the
    op's pad after its value inside its last 8-byte word (k_lookup + k_resolve0_direct, patch_in_resolve)"""
    pad = sizes.op - L.OP_VALUE_OFF - sizes.st_value
    return sizes.op <= 64 or (sizes.st_value <= 320 and sizes.op % 8 == 0 and 0 <= pad <= 8)


class Round:
    """Buffers and kernels of one replica's protocol round over `n_workers` virtual workers."""

    LOCAL = 250                      # MAX_BATCH_KVS_OPS_SIZE, config.h:42

    def __init__(self, kvs: HermesKV, n_workers: int, membership: bytes, peer_ids: list[int],
                 zipf: HkvZipf, write_permille: int = 200, rmw_permille: int = 0,
                 remote_per_peer: int = 50, trace_len: int = 8192, seed: int = 0x5EED,
                 virtual_peers: bool = True, max_steps: int = 64, retry_stalled: bool = False,
                 fit_ack_stride: bool = True, val_credits: int | None = None, pack_remote: bool = True,
                 hades: bool = False, coalesce_hot: bool = False, fused_refill: bool | None = None):
        self.kvs = kvs
        self.W = n_workers
        self.mb = membership
        self.peers = list(peer_ids)
        self.zipf = zipf
        self.sizes = kvs.sizes
        self.op = kvs.sizes.op
        self.ack_size = self.op if kvs.rmw else L.OP_META_SIZE
        self.rpp = remote_per_peer
        self.R = len(self.peers)
        self.virtual = virtual_peers
        self.retry = retry_stalled     # True: refill_ops semantics (stalled ops keep their slot)
        self.coalesce_hot = coalesce_hot   # ENABLE_COALESCE_OF_HOT_REQS (refill_ops, inline-util.h:237-257)
        self.rflags = refill_flags(kvs, retry_stalled, coalesce_hot)
        # fused_refill: the refill is planned from the state mirror (hkv_wl_refill_plan) and applied by
        # the next local launch as patches, so the op slab is read and written once per round. Not with
        # hot-request coalescing (a sequential walk over the ops) or VAL credits (their marshal keeps no
        # mirror). Big ops (configs[2]'s 312 B) take the patches in the launch's in-place resolve, which
        # needs values of at most 320 B with the op's pad after the value inside its last 8-byte word
        # (hkv_batch.hip, patch_in_resolve); that pays where most slots are refilled each round (fresh
        # batches: 0.655-0.659 -> 0.704-0.716 G ops/s), while under retry, with few slots refilled, the
        # patch reads of every element cost more than the in-place refill saves (61.1-61.5 against
        # 63.0-63.6 M, gpurun_out/r06q), so big ops plan only under fresh batches. Default: wherever it pays.
        can_fuse = not coalesce_hot and val_credits is None and patchable(kvs.sizes)
        pays = kvs.sizes.op <= 64 or not retry_stalled
        self.fused = (can_fuse and pays) if fused_refill is None else (fused_refill and can_fuse)
        # otherwise 312-B ops are refilled in place, but from the same state mirror (hkv_wl_refill_st), so a
        # slot the refill keeps is not read
        self.st_refill = not self.fused and not coalesce_hot and val_credits is None and self.op > 64
        self.machine_id = kvs.machine_id
        dev = torch.device("cuda", kvs.device)
        W, S = n_workers, self.LOCAL
        u8 = dict(dtype=torch.uint8, device=dev)
        self.ops = torch.zeros(W * S * self.op, **u8)
        self.states = torch.zeros(W * S, **u8)   # the local batch's mirror of every op's state byte
        self.opcodes = torch.zeros(W * S, **u8)  # the refill's mirror of every op's opcode byte
        self.patch = torch.zeros(W * S * 16, **u8) if self.fused else None   # planned refills (d_patch)
        self.C = slots_per_worker(write_permille, rmw_permille)   # INV send credits per worker
        self.inv_out = torch.zeros(W * self.C * self.op, **u8)
        self.inv_count = torch.zeros(W, dtype=torch.int32, device=dev)
        self.held = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ack_stride = self.C * max(self.R, 1)   # capacity; the round uses self.ack_width
        self.ack_width = self.ack_stride
        # fit_ack_stride: each round's ACK batch is packed (HKV_BATCH_PACKED, about 20 ACKs per
        # worker instead of R x C slots); its offsets, total and the largest INV count are computed
        # on the GPU and read back while the remote INV batch runs
        self.fit = fit_ack_stride and virtual_peers and self.R > 0 and val_credits is None
        # val_credits: VAL messages each worker may send per round (the VAL channel's credits, which
        # the virtual peers return every round). Then a worker's ACKs queue up in its row of `acks`
        # (aq_n of them) and are polled only while it has no VALs outstanding (hermes_worker.c:479);
        # VALs beyond the credits are carried (vq) and sent first next round; INVs whose ACKs wait
        # in the queue keep their INV credits. None: every round applies every ACK and sends every
        # VAL (credits that never bind).
        self.V = val_credits
        if val_credits is not None:
            assert virtual_peers and val_credits >= 0
            self.aq_n = torch.zeros(W, dtype=torch.int32, device=dev)
            self.vq = torch.zeros(W * self.C * L.OP_META_SIZE, **u8)
            self.vq_n = torch.zeros(W, dtype=torch.int32, device=dev)
            self.val_overflow = torch.zeros(1, dtype=torch.int64, device=dev)
            self.val_totals = torch.zeros(2, dtype=torch.int64, device=dev)  # VALs sent, gated worker-rounds
        self.maxc_h = torch.zeros(4, dtype=torch.int32, pin_memory=True) if self.fit else None
        # the host spins on the flag word the kernel writes after the total (no event, no gap)
        self._ack_seq = 0
        self._ack_flag = ctypes.c_int32.from_address(self.maxc_h.data_ptr() + 8) if self.fit else None
        self.ack_off = torch.zeros(W + 1, dtype=torch.int32, device=dev) if self.fit else None
        self.ack_total = 0
        # peer-major ACKs (fit path): each virtual peer's answers to the round's INVs as one block,
        # applied as a launch of its own with HKV_BATCH_UNIQUE (one ACK per key and peer: a key has at
        # most one local write in flight); ack_off then holds the INV offsets and inv_round the INV total
        self.ack_pm = self.fit
        # ... and all peers' blocks in one launch (HKV_BATCH_ROWS: each key looked up once, its ACKs applied
        # in peer order; 64-B entries, 16-B ACKs; otherwise one launch per peer)
        self.ack_rows = self.sizes.entry == 64 and self.ack_size <= 64
        # ... which also makes the VALs of the writes it completes (the VAL callbacks, hermes_worker.c:122-157,
        # into val_out in the ACKs' positions: hkv_batch_desc.d_ack_out on an ACK launch) instead of a
        # collection pass over the ACK slab (otherwise: k_collect_vals, compacted per worker)
        self.fused_vals = self.ack_pm and self.ack_rows and self.ack_size == 16 and val_credits is None
        self._vals_made = False
        self.inv_round = 0
        self.ack_m = self.C
        self.acks = torch.zeros(W * self.ack_stride * self.ack_size, **u8)
        self.ack_count = torch.zeros(W, dtype=torch.int32, device=dev)
        self.val_out = torch.zeros(W * self.ack_stride * L.OP_META_SIZE, **u8)
        self.val_count = torch.zeros(W, dtype=torch.int32, device=dev)
        self.rstride = self.rpp * max(self.R, 1)
        self.ack_out = torch.zeros(W * self.rstride * self.ack_size, **u8)
        self.cursor = torch.zeros(W, dtype=torch.int32, device=dev)
        self.counters = torch.zeros(4096, dtype=torch.int64, device=dev)  # HKV_WL_COUNTER_WORDS
        self.inv_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.elem_totals = torch.zeros(3, dtype=torch.int64, device=dev)  # INV, ACK, VAL elements applied
        self.count_elems = True        # keep inv_total / elem_totals (small torch ops per step)
        self.peer_t = torch.tensor(self.peers or [0], dtype=torch.uint8, device=dev)
        self.trace_len = trace_len
        self.seed = seed
        self.trace_key = torch.empty(W * trace_len, dtype=torch.int64, device=dev)
        self.trace_op = torch.empty(W * trace_len, dtype=torch.uint8, device=dev)
        # hot-request coalescing reads the trace's key ids and keeps its pointers per worker
        self.trace_id = torch.empty(W * trace_len, dtype=torch.int32, device=dev) if coalesce_hot else None
        self.hot = torch.full((W * 2 * HOT_KEYS,), 0xFF, dtype=torch.uint8, device=dev) if coalesce_hot else None
        check(_L.hkv_wl_gen_trace(_ptr(self.trace_key), _ptr(self.trace_op), _ptr(self.trace_id), W, trace_len,
                                  ctypes.byref(zipf), write_permille, rmw_permille,
                                  ctypes.c_uint64(seed ^ (self.machine_id << 48)), _s()), "gen_trace")
        self.clock = 0
        self.max_steps = max_steps
        self.rmw_pm = rmw_permille
        self.remote_inv = []
        self.remote_val = []
        self.remote_counts = []        # per round index: [n live peers] -> per-worker counts
        # RMW builds: each virtual peer's write of the round per [entry][peer], for its INV-aborts
        self.peer_ts = None
        if virtual_peers and self.R and kvs.rmw:
            self.peer_ts = torch.zeros(int(_L.hkv_wl_peer_ts_words(kvs.h)), dtype=torch.int64, device=dev)
        self.pack_remote = virtual_peers and self.R > 0 and pack_remote
        self.remote_packed = []        # per round index: (INVs, VALs, batch offsets, total, entry offsets)
        # our ACKs to each peer's INVs written by that peer's INV launch itself (hkv_batch_desc.d_ack_out)
        # instead of a marshal pass over the applied INVs
        self.fused_acks = (self.pack_remote and ((kvs.sizes.entry == 64 and self.op <= 64) or
                                                 (kvs.sizes.entry == 320 and self.op <= 320)))
        self.drops = []                # peers dropped from the membership (membership_change)
        self.alive = self.R            # live peers: the first `alive` slots of the remote slabs
        self._counts = {}
        self.hades = None
        if hades:
            self._hades_start()
        self._gen_remote()
        self.audit: CommitAudit | None = None   # audit_rounds(): per-outcome commit breakdown (untimed)
        self._pts_done = None          # (clock, live peers) whose virtual-peer timestamps the last refill took
        self.refill(first=True)

    def _gen_remote(self):
        """INV + VAL slabs [W][R * rpp] of the virtual peers, one per round index: each peer's
        first write of a key in the round, compacted per worker in peer order
        (hkv_wl_gen_peer_round); the timestamps are taken at the start of each round"""
        if not (self.virtual and self.R):
            return
        W, R, dev = self.W, self.R, torch.device("cuda", self.kvs.device)
        u8 = dict(dtype=torch.uint8, device=dev)
        scratch = torch.empty(int(_L.hkv_wl_peer_round_scratch(W, self.rpp, R)), **u8)
        pc = torch.empty(W * R, dtype=torch.int32, device=dev)
        for k in range(self.max_steps):
            ri = torch.zeros(W * self.rstride * self.op, **u8)
            rv = torch.zeros(W * self.rstride * L.OP_META_SIZE, **u8)
            check(_L.hkv_wl_gen_peer_round(_ptr(ri), _ptr(rv), _ptr(pc), W, self.rpp, _ptr(self.peer_t), R, self.op,
                                           self.sizes.st_value, self.sizes.shift, ctypes.byref(self.zipf),
                                           self.rmw_pm, k, ctypes.c_uint64(self.seed * 7919 + self.machine_id),
                                           _ptr(scratch), _s()), "gen_peer_round")
            cum = torch.cumsum(pc.view(W, R), dim=1, dtype=torch.int32)
            self.remote_counts.append([None] + [cum[:, n - 1].contiguous() for n in range(1, R + 1)])
            self.remote_inv.append(ri)
            self.remote_val.append(rv)
            if self.pack_remote:
                # the same elements back to back (HKV_BATCH_PACKED), peer-major: rounds where every peer
                # is live launch over the live INVs / VALs only, not the slabs' empty slots, and each
                # peer's INVs -- at most one per key, as a coordinator has one write per key in flight --
                # go in a launch of their own with HKV_BATCH_UNIQUE (one pass). Batch r * W + w holds
                # peer r's elements of worker w's row. (Drawn once per round index, outside timed steps.)
                pcw = pc.view(W, R).long()
                start = torch.cumsum(pcw, dim=1) - pcw                 # where peer r starts in row w
                cnt = pcw.t().reshape(-1)                              # batch (r, w), peer-major
                off = torch.zeros(R * W + 1, dtype=torch.int64, device=dev)
                torch.cumsum(cnt, 0, out=off[1:])
                total = int(off[-1].item())
                b = torch.repeat_interleave(torch.arange(R * W, device=dev), cnt)
                j = torch.arange(total, device=dev) - off[b]
                r_, w_ = b // W, b % W
                src = w_ * self.rstride + start.t().reshape(-1)[b] + j   # element of the row layout
                pi = ri.view(-1, self.op)[src].reshape(-1) if total else torch.empty(self.op, **u8)
                pv = rv.view(-1, L.OP_META_SIZE)[src].reshape(-1) if total else torch.empty(L.OP_META_SIZE, **u8)
                off32 = off.to(torch.int32)
                base = [int(off[r * W].item()) for r in range(R + 1)]
                per_peer = [(base[r], base[r + 1] - base[r], (off[r * W:(r + 1) * W + 1] - base[r]).to(torch.int32))
                            for r in range(R)]
                phys = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
                check(_L.hkv_wl_peer_locate(self.kvs.h, _ptr(pi), total, self.op, _ptr(phys), _s()), "peer_locate")
                self.remote_packed.append((pi, pv, off32, total, phys, per_peer))
        del scratch

    # -- pieces of one round
    def refill(self, first: bool = False, next_round: bool = False):
        """refill_ops for the next round. next_round (the end of Round.step, clock already advanced): the
        plan and the next round's virtual-peer timestamps in one launch (hkv_wl_refill_plan_peer_ts), which
        the next step then does not repeat."""
        if self.fused and not first and next_round and self.pack_remote and self.R and self.alive:
            k = self.clock % max(len(self.remote_inv), 1)
            pi, pv, _, _, phys, _ = self.remote_packed[k]
            total = self._packed_total(k, self.alive)
            check(_L.hkv_wl_refill_plan_peer_ts(_ptr(self.states), self.W, self.LOCAL, self.sizes.st_value,
                                                self.sizes.shift, _ptr(self.trace_key), _ptr(self.trace_op),
                                                self.trace_len, _ptr(self.cursor), self.machine_id, self.rflags,
                                                _ptr(self.counters), _ptr(self.opcodes), _ptr(self.patch), self.kvs.h,
                                                _ptr(pi), _ptr(pv), _ptr(phys), total, self.op, _ptr(self.peer_ts),
                                                self.clock, _s()), "refill_plan_peer_ts")
            self._pts_done = (self.clock, self.alive)
            return
        if self.fused and not first:   # a plan the next local launch applies (the ops stay as they are)
            check(_L.hkv_wl_refill_plan(_ptr(self.states), self.W, self.LOCAL, self.sizes.st_value, self.sizes.shift,
                                        _ptr(self.trace_key), _ptr(self.trace_op), self.trace_len, _ptr(self.cursor),
                                        self.machine_id, self.rflags, _ptr(self.counters), _ptr(self.opcodes),
                                        _ptr(self.patch), _s()), "refill_plan")
            return
        if self.st_refill and not first:
            check(_L.hkv_wl_refill_st(_ptr(self.ops), self.W, self.LOCAL, self.op, self.sizes.st_value, self.sizes.shift,
                                      _ptr(self.trace_key), _ptr(self.trace_op), self.trace_len, _ptr(self.cursor),
                                      self.machine_id, self.rflags, _ptr(self.counters), _ptr(self.opcodes),
                                      _ptr(self.states), _s()), "refill_st")
            return
        check(_L.hkv_wl_refill(_ptr(self.ops), self.W, self.LOCAL, self.op, self.sizes.st_value, self.sizes.shift,
                               _ptr(self.trace_key), _ptr(self.trace_op), _ptr(self.trace_id), self.trace_len,
                               _ptr(self.cursor), self.machine_id, int(first), self.rflags, _ptr(self.counters),
                               _ptr(self.opcodes), _ptr(self.hot), _s()),
              "refill")
        if first:
            init_mirrors(self.ops, self.op, self.states)

    def local_batch(self):
        self.kvs.batch(L.BatchType.local_ops, self.ops, self.W, self.LOCAL, self.op, self.mb, state_out=self.states,
                       opcode_in=self.opcodes, patch=self.patch)

    def close(self):
        """Nothing is left pending between rounds (kept for callers that close a round)."""

    def marshal_invs(self):
        if self.V is not None:
            check(_L.hkv_wl_marshal_invs_credits(_ptr(self.ops), self.W, self.LOCAL, self.op, _ptr(self.inv_out),
                                                 self.C, _ptr(self.inv_count), self.machine_id, _ptr(self.held),
                                                 _ptr(self.aq_n), max(self.alive, 1), _s()), "marshal_invs")
            return
        check(_L.hkv_wl_marshal_invs_cap(_ptr(self.ops), self.W, self.LOCAL, self.op, _ptr(self.inv_out), self.C,
                                         _ptr(self.inv_count), self.machine_id, _ptr(self.held), _ptr(self.states),
                                         _s()), "marshal_invs")

    def virtual_peer_acks(self, n_peers: int | None = None):
        """ACKs (INV-aborts for RMWs a peer's own write beats) of the first n_peers virtual peers
        (default all) to this round's INVs"""
        if self.ack_pm:
            check(_L.hkv_wl_peer_acks_pm(self.kvs.h, _ptr(self.inv_out), _ptr(self.inv_count), self.W, self.C,
                                         self.op, _ptr(self.acks), self.ack_size, self.ack_m,
                                         _ptr(self.ack_count), _ptr(self.peer_t), self.R if n_peers is None else n_peers,
                                         _ptr(self.peer_ts), self.clock, _ptr(self.ack_off), _s()), "peer_acks_pm")
            return
        check(_L.hkv_wl_peer_acks(self.kvs.h, _ptr(self.inv_out), _ptr(self.inv_count), self.W, self.C, self.op,
                                  _ptr(self.acks), self.ack_size, self.ack_width, _ptr(self.ack_count),
                                  _ptr(self.peer_t), self.R if n_peers is None else n_peers, _ptr(self.peer_ts),
                                  self.clock, _ptr(self.ack_off) if self.fit else None, _s()), "peer_acks")

    def peer_timestamps(self, k: int, n_peers: int):
        """Round start: the live peers' INVs and VALs of round index k take their timestamps"""
        check(_L.hkv_wl_peer_ts(self.kvs.h, _ptr(self.remote_inv[k]), _ptr(self.remote_val[k]),
                                _ptr(self.remote_counts[k][n_peers]), self.W, self.rstride, self.op,
                                _ptr(self.peer_ts), self.clock, _s()), "peer_ts")

    def _packed_total(self, k: int, n_peers: int) -> int:
        """elements of the first n_peers peers in round index k's packed slabs"""
        return sum(n for _, n, _ in self.remote_packed[k][5][:n_peers])

    def peer_timestamps_packed(self, k: int, n_peers: int | None = None):
        """the same for the packed slabs, whose INVs' entries were located when they were drawn (the first
        n_peers peers' elements; default all)"""
        pi, pv, _, total, phys, _ = self.remote_packed[k]
        if n_peers is not None:
            total = self._packed_total(k, n_peers)
        check(_L.hkv_wl_peer_ts_at(self.kvs.h, _ptr(pi), _ptr(pv), _ptr(phys), total, self.op, _ptr(self.peer_ts),
                                   self.clock, _s()), "peer_ts_at")

    def inv_batch(self, invs: torch.Tensor, n_batches: int, stride: int, counts: torch.Tensor | None = None,
                  offsets: torch.Tensor | None = None, unique: bool = False):
        self.kvs.batch(L.BatchType.invs, invs, n_batches, stride, self.op, self.mb, counts=counts, offsets=offsets,
                       unique=unique)

    def inv_batches_per_peer(self, k: int, n_peers: int | None = None):
        """Every peer's INVs of round index k as a launch of its own (HKV_BATCH_UNIQUE), in peer order.
        n_peers: the first n_peers peers only (default all)"""
        pi, _, _, _, _, per_peer = self.remote_packed[k]
        for base, n, off in per_peer[:n_peers]:
            if n:
                if self.fused_acks:
                    self.kvs.batch(L.BatchType.invs, pi[base * self.op:], self.W, n, self.op, self.mb, offsets=off,
                                   unique=True, ack_out=self.ack_out[base * self.ack_size:], ack_out_size=self.ack_size)
                else:
                    self.kvs.batch(L.BatchType.invs, pi[base * self.op:], self.W, n, self.op, self.mb, offsets=off,
                                   unique=True)

    def marshal_acks(self, invs: torch.Tensor, n: int, out: torch.Tensor):
        check(_L.hkv_wl_marshal_acks(_ptr(invs), n, self.op, _ptr(out), self.ack_size, self.machine_id, _s()),
              "marshal_acks")

    def _rws(self):
        """the state mirror the ACK batch keeps current (only the fused refill plans from it; the
        VAL-credits marshal does not maintain it)"""
        return self.states if self.fused or self.st_refill else None

    def _rwo(self):
        """the opcode mirror the ACK batch completes from (the refill keeps it; the local launch checks it
        against every op)"""
        return self.opcodes

    def ack_batch(self, acks: torch.Tensor | None = None, n_batches: int | None = None, stride: int | None = None,
                  counts: torch.Tensor | None = None):
        acks = self.acks if acks is None else acks
        if self.fit and stride is None and self.ack_pm:   # one launch per peer, in peer order
            T = self.inv_round
            n_rows = self.ack_total // max(T, 1) if T else 0
            if self.ack_rows and n_rows:
                self.kvs.batch(L.BatchType.acks, acks, self.W, T, self.ack_size, self.mb, rw=self.ops,
                               rw_stride_bytes=self.LOCAL * self.op, offsets=self.ack_off, rw_state=self._rws(),
                               unique=True, rows=(n_rows, T, -1), rw_opcodes=self._rwo(),
                               ack_out=self.val_out if self.fused_vals else None)
                self._vals_made = self.fused_vals
                return
            for r in range(n_rows):
                self.kvs.batch(L.BatchType.acks, acks[r * T * self.ack_size:], self.W, T, self.ack_size, self.mb,
                               rw=self.ops, rw_stride_bytes=self.LOCAL * self.op, offsets=self.ack_off,
                               rw_state=self._rws(), unique=True, rw_opcodes=self._rwo())
            return
        if self.fit and stride is None:   # this round's packed ACKs
            self.kvs.batch(L.BatchType.acks, acks, self.W, self.ack_total, self.ack_size, self.mb,
                           rw=self.ops, rw_stride_bytes=self.LOCAL * self.op, offsets=self.ack_off,
                           rw_state=self._rws(), rw_opcodes=self._rwo())
            return
        self.kvs.batch(L.BatchType.acks, acks, n_batches or self.W, stride or self.ack_width, self.ack_size,
                       self.mb, counts=self.ack_count if counts is None else counts, rw=self.ops,
                       rw_stride_bytes=self.LOCAL * self.op, rw_state=self._rws(), rw_opcodes=self._rwo())

    def marshal_vals(self, acks: torch.Tensor, n: int, out: torch.Tensor):
        check(_L.hkv_wl_marshal_vals(_ptr(acks), n, self.ack_size, _ptr(out), self.machine_id, _s()),
              "marshal_vals")

    def collect_vals(self):
        """VALs of the writes this round's ACK batch completed, compacted per worker (val_out
        [W][ack_stride], val_count): only the ACK slab's live elements are read. Nothing to do when the
        ACK rows launch made them itself (fused_vals: val_out then holds them in the ACKs' positions)."""
        if self._vals_made:
            self._vals_made = False
            return
        if self.ack_pm:
            check(_L.hkv_wl_collect_vals_blocks(_ptr(self.acks), _ptr(self.ack_count), self.W, self.ack_width,
                                                self.ack_size, _ptr(self.val_out), self.C, _ptr(self.val_count),
                                                self.machine_id, None, _ptr(self.ack_off),
                                                self.ack_total // max(self.inv_round, 1) if self.inv_round else 1,
                                                _s()), "collect_vals")
            return
        check(_L.hkv_wl_collect_vals(_ptr(self.acks), _ptr(self.ack_count), self.W, self.ack_width, self.ack_size,
                                     _ptr(self.val_out), self.C, _ptr(self.val_count), self.machine_id,
                                     None, _ptr(self.ack_off) if self.fit else None, _s()), "collect_vals")

    def peer_acks_queued(self, n_peers: int):
        """The first n_peers virtual peers' ACKs to this round's INVs appended to each worker's ACK
        queue; ack_count = the queue for workers without outstanding VALs, 0 for the others"""
        if self.count_elems:
            self.val_totals[1] += (self.vq_n > 0).sum()
        check(_L.hkv_wl_peer_acks_queue(self.kvs.h, _ptr(self.inv_out), _ptr(self.inv_count), self.W, self.C, self.op,
                                        _ptr(self.acks), self.ack_size, self.ack_stride, _ptr(self.aq_n),
                                        _ptr(self.vq_n), _ptr(self.ack_count), _ptr(self.peer_t), n_peers,
                                        _ptr(self.peer_ts), self.clock, _s()), "peer_acks_queue")

    def vals_under_credits(self):
        """Carried VALs first, then those of the writes this round's ACK batch completed, at most
        val_credits per worker (val_out / val_count); the rest carried to the next round"""
        check(_L.hkv_wl_vals_credit(_ptr(self.acks), _ptr(self.aq_n), _ptr(self.ack_count), self.W, self.ack_stride,
                                    self.ack_size, _ptr(self.vq), _ptr(self.vq_n), self.C, _ptr(self.val_out),
                                    _ptr(self.val_count), self.ack_stride, self.V, self.machine_id,
                                    _ptr(self.val_overflow), _s()), "vals_credit")
        if self.count_elems:
            self.val_totals[0] += self.val_count.sum()

    def val_batch(self, vals: torch.Tensor, n_batches: int, stride: int, counts: torch.Tensor | None = None,
                  offsets: torch.Tensor | None = None):
        self.kvs.batch(L.BatchType.vals, vals, n_batches, stride, L.OP_META_SIZE, self.mb, counts=counts,
                       offsets=offsets)

    # -- a whole round with virtual peers
    def step(self, events: dict | None = None, timed_batches=("local", "invs", "acks", "vals"),
             drop: int | None = None):
        """One round of every virtual worker. `drop`: the last virtual peer fails in this round
        after sending its INVs (no ACKs, no VALs from it); the round ends with membership_change. `events` (name -> list) collects (start, end)
        torch.cuda.Event pairs for the batches named in `timed_batches` (each event record costs
        a few microseconds of GPU time, so a timed region records only what it reports)."""
        def timed(name, fn):
            if events is None or name not in timed_batches:
                fn()
                return
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            events.setdefault(name, []).append((a, b))

        k = self.clock % max(len(self.remote_inv), 1)
        if drop is not None:
            assert self.virtual and self.alive and drop == self.peers[self.alive - 1], "drop the last live peer"
        sent = self.alive                          # peers whose INVs this round applies
        alive = self.alive - (drop is not None)    # peers that answer them (ACKs) and send VALs
        # the packed slabs (same elements, same order): the live peers are their first `alive` peers (a
        # failed peer is always the last live one), so after a failure the rounds apply a prefix of them
        packed = self.pack_remote
        pts_done, self._pts_done = self._pts_done == (self.clock, sent), None
        if self.R and sent and not pts_done:   # (the last refill may have taken them already)
            if packed:
                self.peer_timestamps_packed(k, sent)
            else:
                self.peer_timestamps(k, sent)
        if self.audit is not None:
            self.audit.pre_local()
        timed("local", self.local_batch)
        if self.audit is not None:
            self.audit.post_local()
        self.marshal_invs()
        if self.count_elems:
            self.inv_total += self.inv_count.sum()
        if self.fit and alive:
            self._ack_seq = self._ack_seq % 0x7FFFFFFF + 1
            check(_L.hkv_wl_ack_offsets(_ptr(self.inv_count), self.W, 1 if self.ack_pm else alive,
                                        _ptr(self.ack_off), _ptr(self.maxc_h), self._ack_seq, _s()), "ack_offsets")
        if self.R:
            ri, rv = self.remote_inv[k], self.remote_val[k]
            ic = self._slot_counts(k, sent)
            if packed:
                pi, pv, off, total, _, _ = self.remote_packed[k]
                timed("invs", lambda: self.inv_batches_per_peer(k, sent))
                if not self.fused_acks:   # (else the INV launches wrote them)
                    self.marshal_acks(pi, self._packed_total(k, sent), self.ack_out)
            else:
                timed("invs", lambda: self.inv_batch(ri, self.W, self.rstride, counts=ic))
                self.marshal_acks(ri, self.W * self.rstride, self.ack_out)
            m = self.C
            if self.fit and alive:   # the GPU is still on the INV batch: this wait leaves no gap
                spins = 0
                while self._ack_flag.value != self._ack_seq:
                    spins += 1
                    if spins % 65536 == 0:   # a lost flag fails loudly instead of spinning on
                        torch.cuda.synchronize()
                        if self._ack_flag.value != self._ack_seq:
                            raise RuntimeError("ACK layout flag never arrived")
                self.ack_total = int(self.maxc_h[0])
                if self.ack_pm:   # the offsets counted INVs: one block of them per answering peer
                    self.inv_round = self.ack_total
                    self.ack_total *= alive
                m = min(int(self.maxc_h[1]), self.C)
            if alive and self.V is not None:
                self.peer_acks_queued(alive)
                timed("acks", lambda: self.ack_batch(stride=self.ack_stride))
                if self.count_elems:
                    self.elem_totals[1] += self.ack_count.sum()
                self.vals_under_credits()
            elif alive:
                self.ack_m = max(1, m)
                self.ack_width = self.ack_m * alive
                self.virtual_peer_acks(alive)
                timed("acks", self.ack_batch)
                if self.count_elems:
                    self.elem_totals[1] += self.ack_count.sum()
                self.collect_vals()
            # a dropped peer sent its INVs but fails before its VALs
            vc = self._slot_counts(k, alive)
            if packed:
                timed("vals", lambda: self.val_batch(pv, alive * self.W, self._packed_total(k, alive), offsets=off))
            else:
                timed("vals", lambda: self.val_batch(rv, self.W, self.rstride, counts=vc))
            if self.count_elems:
                self.elem_totals[0] += ic.sum()
                if alive:
                    self.elem_totals[2] += vc.sum()
        if self.hades is not None:
            if drop is not None:         # the peer is gone; the membership follows the agreement
                self._peer_gone(drop)
            self._hades_period()
        elif drop is not None:
            self.membership_change(drop)
        if self.audit is not None:
            self.audit.end()
        self.clock += 1
        self.refill(next_round=True)

    def _slot_counts(self, k: int, n_peers: int):
        """Per-worker counts applying the first n_peers peers' elements of round index k's
        remote slabs (peer order within each worker's row)"""
        if n_peers == 0:
            if 0 not in self._counts:
                self._counts[0] = torch.zeros(self.W, dtype=torch.int32, device=self.inv_count.device)
            return self._counts[0]
        return self.remote_counts[k][n_peers]

    def membership_change(self, peer: int):
        """The group drops `peer` (group_membership_update, inline-util.h:26-43) and every worker
        runs the after-membership-change batch on its ops (hermes_worker.c:526-542): writes and
        replays that waited only for the dropped peer's ACK complete, and their VALs go out
        (hkv_wl_marshal_memb_vals). From now on the peer's slot of the remote slabs is not applied;
        reads of keys it left INVALID replay the write (early value propagation)."""
        g = self.mb[1] & ~(1 << peer) & 0xFF
        self._after_membership_change(L.membership(0, self.machine_id, alive=g))
        self._peer_gone(peer)

    def _peer_gone(self, peer: int):
        self.drops.append(peer)
        self.alive -= 1
        self.fit = self.fit and self.alive > 0

    def _after_membership_change(self, mb: bytes):
        self.mb = mb
        self.kvs.batch(L.BatchType.local_ops_after_membership_change, self.ops, self.W, self.LOCAL, self.op, self.mb,
                       state_out=self.states)
        check(_L.hkv_wl_marshal_memb_vals(_ptr(self.ops), self.W, self.LOCAL, self.op, _ptr(self.val_out),
                                          self.ack_stride, _ptr(self.val_count), self.machine_id, _ptr(self.states),
                                          _s()), "marshal_memb_vals")

    # -- Hades: this replica and every virtual peer run the agreement
    def _hades_start(self):
        from .hades import Hades, exchange_views
        ids = [self.machine_id] + self.peers
        self.hades_n = max(ids) + 1
        self.hades = {i: Hades(self.hades_n, i) for i in ids}
        self.hades_changes = []         # (round, agreed g_membership) of this replica's changes
        self._exchange = exchange_views
        full = sum(1 << i for i in ids)
        for _ in range(16):             # spin_until_all_nodes_are_in_membership
            for h in self.hades.values():
                h.update()
            self._exchange([self.hades.get(i) for i in range(self.hades_n)])
            if all(h.state()[0] == full for h in self.hades.values()):
                return
        raise RuntimeError("Hades bootstrap did not reach the full membership")

    def _hades_period(self):
        """update_view_and_issue_hbs + group_membership_update + poll_for_remote_views
        (hermes_worker.c:262-291) for this replica and its live virtual peers; a failed peer no
        longer heartbeats. When this replica's agreed membership changes, every worker runs the
        after-membership-change batch under it."""
        from .hades import MajorityLost
        live = {i: h for i, h in self.hades.items() if i not in self.drops}
        res = {i: h.update() for i, h in live.items()}
        self._exchange([live.get(i) for i in range(self.hades_n)])
        changed, mb, _ = res[self.machine_id]
        if changed:
            if bin(mb[1]).count("1") < self.hades_n // 2:   # inline-util.h:39-42
                raise MajorityLost(f"membership {mb[1]:#04x} of {self.hades_n}")
            self.hades_changes.append((self.clock, mb[1]))
            self._after_membership_change(bytes(mb[:3]) + bytes(5))

    def fold_counters(self) -> torch.Tensor:
        """counters[0..4] brought up to date (refill leaves per-worker-group partial sums)"""
        check(_L.hkv_wl_fold_counters(_ptr(self.counters), _s()), "fold_counters")
        return self.counters

    def audit_rounds(self, n: int) -> dict:
        """One round that only tracks provenance, then n rounds whose commits are broken down by
        outcome (CommitAudit); checked against the refill's own commit count over the same rounds."""
        self.audit = CommitAudit(self)
        self.step()
        c0 = int(self.fold_counters()[0].item())
        for _ in range(n):
            self.step()
        c1 = int(self.fold_counters()[0].item())
        out = self.audit.result(c1 - c0)
        self.audit = None
        return out

    def committed(self) -> int:
        return int(self.fold_counters()[0].item())

    def stats(self) -> dict:
        c = self.fold_counters()[:5].cpu().tolist()
        d = {"committed": c[0], "misses": c[1], "writes_completed": c[2], "dropped": c[3], "rmw_aborts": c[4],
             "invs_held": int(self.held.item())}
        if self.V is not None:
            v = self.val_totals.cpu().tolist()
            d.update(vals_sent=v[0], gated_worker_rounds=v[1], vals_carried=int(self.vq_n.sum().item()),
                     acks_queued=int(self.aq_n.sum().item()), val_overflow=int(self.val_overflow.item()))
        return d
