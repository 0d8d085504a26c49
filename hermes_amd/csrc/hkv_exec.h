// hkv_exec.h -- per-entry state machine of the HermesKV protocol, device side.
//
// Each function applies ONE element to a register copy of its key's object meta (Meta), the
// way the reference's exec function applies it to the entry. The batch engine (hkv_batch.hip)
// decides which meta an element sees: elements that cannot change the meta (would_mutate
// false) run in parallel against one snapshot, and a key's mutating elements run one per
// round, each on its own shadow image of the entry, in element order. Within one exec call
// no other thread touches the key's meta, so the reference's per-key seqlock
// (concur_ctrl.h:144-224) has no work to do; only its NET effect on the version survives a
// batch boundary, so the lock/unlock pair is folded into the version arithmetic:
//   lock+unlock_dec -> +0, lock+unlock_inc -> +2, lock+unlock_inc_by_three -> +4,
//   lock+unlock_custom(v) -> v, and "locked version - 1" reads are the plain version.
// tests/test_oracle.py pins these net effects against the reference's own cctrl_* functions.
// Each function cites the reference function whose observable behaviour it reproduces.
#pragma once
#include <hip/hip_runtime.h>
#include "hkv_codes.h"

namespace hkv {

struct Meta {        // spacetime_object_meta (spacetime.h:138-148) + log val_len
    uint32_t w4;     // entry bytes 16..19: opcode, val_len, state, ack_bv
    uint32_t w5;     // 20..23: RMW_flag|last_writer_id, op_buffer_index, lock, ts.cid
    uint32_t ver;    // 24..27: ts.version
    uint32_t llw_ver;
    uint8_t llw_cid;
};

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) { return *reinterpret_cast<const uint64_t *>(p); }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) { *reinterpret_cast<uint32_t *>(p) = v; }

// field accessors on the register copy
__device__ __forceinline__ uint8_t m_val_len(const Meta &m) { return (uint8_t)(m.w4 >> 8); }
__device__ __forceinline__ void m_set_val_len(Meta &m, uint8_t v) { m.w4 = (m.w4 & 0xFFFF00FFu) | ((uint32_t)v << 8); }
__device__ __forceinline__ uint8_t m_state(const Meta &m) { return (uint8_t)(m.w4 >> 16); }
__device__ __forceinline__ void m_set_state(Meta &m, uint8_t v) { m.w4 = (m.w4 & 0xFF00FFFFu) | ((uint32_t)v << 16); }
__device__ __forceinline__ uint8_t m_ack_bv(const Meta &m) { return (uint8_t)(m.w4 >> 24); }
__device__ __forceinline__ void m_set_ack_bv(Meta &m, uint8_t v) { m.w4 = (m.w4 & 0x00FFFFFFu) | ((uint32_t)v << 24); }
__device__ __forceinline__ uint8_t m_rmw(const Meta &m) { return (uint8_t)(m.w5 & 1u); }
__device__ __forceinline__ void m_set_rmw(Meta &m, uint8_t f) { m.w5 = (m.w5 & ~1u) | (f & 1u); }
__device__ __forceinline__ uint8_t m_lwid(const Meta &m) { return (uint8_t)((m.w5 >> 1) & 0x7Fu); }
__device__ __forceinline__ void m_set_lwid(Meta &m, uint8_t w) { m.w5 = (m.w5 & ~0xFEu) | ((uint32_t)(w & 0x7Fu) << 1); }
__device__ __forceinline__ uint8_t m_obi(const Meta &m) { return (uint8_t)(m.w5 >> 8); }
__device__ __forceinline__ void m_set_obi(Meta &m, uint8_t v) { m.w5 = (m.w5 & 0xFFFF00FFu) | ((uint32_t)v << 8); }
__device__ __forceinline__ uint8_t m_cid(const Meta &m) { return (uint8_t)(m.w5 >> 24); }
__device__ __forceinline__ void m_set_cid(Meta &m, uint8_t v) { m.w5 = (m.w5 & 0x00FFFFFFu) | ((uint32_t)v << 24); }

// Entries and shadows are 8-byte aligned: the meta moves as two 8-byte words (bytes 16..31) and
// byte 32, three memory instructions instead of five.
__device__ __forceinline__ void meta_load(const uint8_t *e, Meta &m)
{
    const uint64_t a = *reinterpret_cast<const uint64_t *>(e + 16);
    const uint64_t b = *reinterpret_cast<const uint64_t *>(e + 24);
    m.w4 = (uint32_t)a;
    m.w5 = (uint32_t)(a >> 32);
    m.ver = (uint32_t)b;
    m.llw_cid = (uint8_t)(b >> 32);
    m.llw_ver = (uint32_t)(b >> 40) | ((uint32_t)e[32] << 24);
}

__device__ __forceinline__ void meta_store(uint8_t *e, const Meta &m)
{
    // the seqlock byte is free at batch boundaries
    *reinterpret_cast<uint64_t *>(e + 16) = (uint64_t)m.w4 | ((uint64_t)(m.w5 & 0xFF00FFFFu) << 32);
    *reinterpret_cast<uint64_t *>(e + 24) = (uint64_t)m.ver | ((uint64_t)m.llw_cid << 32) | ((uint64_t)m.llw_ver << 40);
    e[32] = (uint8_t)(m.llw_ver >> 24);
}

// Lamport order on (version, cid): concur_ctrl.h:63-75
__device__ __forceinline__ uint64_t pack_ts(uint32_t ver, uint8_t cid) { return ((uint64_t)ver << 8) | cid; }

// element header (spacetime_op_meta_t, spacetime.h:151-166)
__device__ __forceinline__ uint8_t e_opcode(const uint8_t *x) { return x[8]; }
__device__ __forceinline__ uint8_t e_state(const uint8_t *x) { return x[9]; }
__device__ __forceinline__ uint64_t e_ts(const uint8_t *x) { return pack_ts(ld32(x + 12), x[11]); }
__device__ __forceinline__ void e_set_ts(uint8_t *x, uint32_t ver, uint8_t cid) { x[11] = cid; st32(x + 12, ver); }
__device__ __forceinline__ uint8_t e_rmw(const uint8_t *x) { return x[16] & 1u; }
__device__ __forceinline__ void e_set_rmw(uint8_t *x, uint8_t f) { x[16] = (uint8_t)((x[16] & 0xFEu) | (f & 1u)); }

// Byte-exact copy between the op value (offset 18) and the log value (offset 33): the two
// never share an alignment, so the middle moves as aligned dwords built with v_alignbyte from
// the aligned source dwords that overlap the range (both objects are 8-byte aligned and a
// multiple of 8 long, so no dword outside the source object is touched), and only the < 4
// head/tail bytes move one by one.
__device__ __forceinline__ void copy_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint32_t n)
{
    uint32_t head = (4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u;
    if (head > n) head = n;
    for (uint32_t k = 0; k < head; ++k) dst[k] = src[k];
    const uint8_t *s = src + head;
    const uint32_t sh = (uint32_t)(uintptr_t)s & 3u;
    // aligned down by pointer arithmetic, not through an integer, so an LDS or global source
    // keeps its address space (an int-to-pointer cast would make every access a flat one)
    const uint32_t *sa = reinterpret_cast<const uint32_t *>(s - sh);
    uint32_t *da = reinterpret_cast<uint32_t *>(dst + head);
    const uint32_t nw = (n - head) >> 2;
    if (sh == 0) {
        for (uint32_t j = 0; j < nw; ++j) da[j] = sa[j];
    } else {
        uint32_t lo = nw ? sa[0] : 0u;
        for (uint32_t j = 0; j < nw; ++j) {
            uint32_t hi = sa[j + 1];
            da[j] = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
        }
    }
    for (uint32_t k = head + 4 * nw; k < n; ++k) dst[k] = src[k];
}

template <int SV>
__device__ __forceinline__ void copy_value(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint32_t n)
{
    copy_bytes(dst, src, SV > 0 ? (uint32_t)SV : n);
}

// A value copy an exec function leaves to its caller (Ctx::vc): big values (287 B) copied by one
// lane touch a few cache lines per dword, 64 lines per wave instruction; the caller copies them
// afterwards a whole wave per value (wave_value_copies)
struct VCopy {
    uint8_t *dst;
    const uint8_t *src;
    uint32_t fill = 0;   // 0x100 | b: the source is n bytes b, nothing is loaded (a refill patch's value)
};

struct Ctx {           // per-launch constants
    Geometry g;
    uint8_t g_membership;
    uint8_t w_ack_init;
    uint8_t *rw;       // this element's batch read_write_ops (ACKs)
    uint8_t *rws;      // its state-byte mirror (hkv_batch_desc.d_rw_state), or null
    const uint8_t *rwo = nullptr;   // its opcode mirror (hkv_batch_desc.d_opcode_in of an ACK launch), or null
    int *rw_done;      // non-null: exec_ack leaves the read_write_ops completion to the caller
    VCopy *vc;         // non-null: big-value copies are recorded here instead of made (at most one per dispatch)
};

template <int SV>
__device__ __forceinline__ void copy_value_c(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint32_t n,
                                             const Ctx &c)
{
    if (SV != 31 && c.vc) {
        c.vc->dst = dst;
        c.vc->src = src;
        return;
    }
    copy_value<SV>(dst, src, n);
}

__device__ __forceinline__ bool is_last_ack(uint8_t bv, const Ctx &c)  // spacetime.h:253-259
{
    return (uint8_t)(bv & c.g_membership) == c.g_membership;
}

// hermes_local_state_to_op, hermesKV.c:143-153
template <int SV>
__device__ __forceinline__ void local_state_to_op(uint8_t *op, const Meta &m, const uint8_t *entry, const Ctx &c)
{
    e_set_rmw(op, m_rmw(m));
    op[9] = kReplaySuccess;
    e_set_ts(op, m.ver, m_cid(m));
    op[10] = (uint8_t)(c.g.st_value >> c.g.shift);
    copy_value_c<SV>(op + kOpValueOff, entry + kEntryValueOff, c.g.st_value, c);
}

// hermes_write_replay_actions, hermesKV.c:155-175
template <int SV>
__device__ __forceinline__ void write_replay(uint8_t *op, uint8_t idx, Meta &m, const uint8_t *entry, const Ctx &c)
{
    m_set_state(m, kReplay);
    m_set_obi(m, idx);
    m.llw_ver = m.ver;
    m.llw_cid = m_cid(m);
    m_set_ack_bv(m, c.w_ack_init);
    local_state_to_op<SV>(op, m, entry, c);
}

// hermes_check_membership_n_write_replay_actions, hermesKV.c:179-194
template <int SV>
__device__ __forceinline__ void membership_replay(uint8_t *op, uint8_t idx, Meta &m, const uint8_t *entry, const Ctx &c)
{
    uint8_t node = m_lwid(m);
    if (node < 8 && ((c.g_membership >> node) & 1u)) op[9] = kGetStall;
    else if (m_obi(m) == kObiEmpty) write_replay<SV>(op, idx, m, entry, c);
}

// hermes_update_actions_n_unlock, hermesKV.c:100-141 (net of lock + unlock_inc[_by_three])
template <int SV>
__device__ __forceinline__ void update_actions(uint8_t *op, uint8_t *entry, uint8_t idx, Meta &m, const Ctx &c, uint8_t rmw_flag)
{
    copy_value_c<SV>(entry + kEntryValueOff, op + kOpValueOff, c.g.st_value, c);
    m_set_val_len(m, (uint8_t)((op[10] >> c.g.shift) + kOpMetaSize));
    m_set_rmw(m, rmw_flag);
    m_set_state(m, kWrite);
    m_set_obi(m, idx);
    uint32_t step = (!c.g.rmw_enabled || rmw_flag == 1) ? 2u : 4u;
    uint8_t node = (uint8_t)c.g.machine_id;
    m.llw_ver = m.ver + step;
    m.llw_cid = node;
    m_set_ack_bv(m, c.w_ack_init);
    m.ver += step;
    m_set_cid(m, node);
    e_set_ts(op, m.ver, node);
    e_set_rmw(op, rmw_flag);
    op[9] = rmw_flag ? kRmwSuccess : kPutSuccess;
}

// hermes_complete_hot_read_optimization, hermesKV.c:224-238 (HKV_SKEW_READ_COMPLETE): a stalled
// GET records the key's timestamp when its own is (0, 0), and completes -- without a value, as
// shipped ("TODO we also need to get the value here") -- once the key's version is two above it.
// cur: the timestamp exec_read saw (the meta's; a write replay leaves it unchanged).
__device__ __forceinline__ void hot_read_complete(uint8_t *op, uint32_t cur_ver, uint8_t cur_cid)
{
    if (op[9] != kGetStall) return;
    const uint32_t over = ld32(op + 12);
    if (over == 0 && op[11] == 0) e_set_ts(op, cur_ver, cur_cid);
    else if (over + 1u < cur_ver) op[9] = kGetComplete;
}

// hermes_exec_read, hermesKV.c:251-311
template <int SV>
__device__ __forceinline__ void exec_read(uint8_t *op, uint8_t *entry, uint8_t idx, Meta &m, const Ctx &c)
{
    uint8_t st = m_state(m);
    if (st == kValid) {
        copy_value_c<SV>(op + kOpValueOff, entry + kEntryValueOff, c.g.st_value, c);
        op[9] = kGetComplete;
        op[10] = (uint8_t)((m_val_len(m) >> c.g.shift) - kOpMetaSize);
    } else if (st == kInvalidWrite || st == kWrite || st == kReplay) {
        op[9] = kGetStall;
    } else {
        op[9] = kEmpty;
        if (st == kInvalid) membership_replay<SV>(op, idx, m, entry, c);
    }
    if (c.g.skew & kSkewReadComplete) hot_read_complete(op, m.ver, m_cid(m));
}

// hermes_exec_write, hermesKV.c:314-356, with hermes_marshal_write_coalesce_optimization and
// hermes_complete_coalesced_write (:196-221) under HKV_SKEW_WRITE_COALESCE: a PUT that stalls in
// VALID/INVALID (op buffer index set), WRITE or INVALID_WRITE -- not REPLAY -- records the key's
// version as 16 bits when its own ts.version is 0; any stalled PUT completes once its
// ts.version + 1 is below that 16-bit version. (The ts of a refilled PUT is whatever its slot
// held: refill_ops resets only GETs', inline-util.h:268-272.)
template <int SV>
__device__ __forceinline__ void exec_write(uint8_t *op, uint8_t *entry, uint8_t idx, Meta &m, const Ctx &c)
{
    uint8_t st = m_state(m);
    if ((st == kValid || st == kInvalid) && m_obi(m) == kObiEmpty) {
        update_actions<SV>(op, entry, idx, m, c, 0);
        return;
    }
    op[9] = kPutStall;
    if (c.g.skew & kSkewWriteCoalesce) {
        const uint32_t cv = m.ver & 0xFFFFu;   // (uint16_t)(version - 1) under the lock
        uint32_t over = ld32(op + 12);
        if (st != kReplay && over == 0) {
            st32(op + 12, cv);
            over = cv;
        }
        if (over > 0 && over + 1u < cv) op[9] = kPutComplete;
    }
}

// hermes_exec_rmw, hermesKV.c:358-428
template <int SV>
__device__ __forceinline__ void exec_rmw(uint8_t *op, uint8_t *entry, uint8_t idx, Meta &m, const Ctx &c)
{
    if (op[9] == kInProgressRmw) {
        uint64_t ots = e_ts(op);
        if (ots < pack_ts(m.ver, m_cid(m))) {
            op[9] = kRmwAbort;
            if (ots == pack_ts(m.llw_ver, m.llw_cid)) m_set_obi(m, kObiEmpty);
        }
        return;
    }
    op[9] = kEmpty;
    uint8_t st = m_state(m);
    if (st == kValid) {
        if (m_obi(m) == kObiEmpty) update_actions<SV>(op, entry, idx, m, c, 1);
    } else if (st == kInvalid) {
        membership_replay<SV>(op, idx, m, entry, c);
    }
    if (op[9] != kRmwSuccess && op[9] != kReplaySuccess) op[9] = kRmwStall;
}

// hermes_exec_check_update_completion, hermesKV.c:430-484
__device__ __forceinline__ void exec_update_completion(uint8_t *op, Meta &m, const Ctx &c)
{
    if (!is_last_ack(m_ack_bv(m), c)) return;
    m_set_obi(m, kObiEmpty);
    uint8_t st = m_state(m);
    if (st == kInvalidWrite || st == kValid || st == kInvalid) {
        if (st == kInvalidWrite) m_set_state(m, kInvalid);
        op[9] = op[8] == kOpPut ? kPutComplete : kRmwComplete;
    } else if (st == kWrite || st == kReplay) {
        e_set_ts(op, m.ver, m_cid(m));
        if (st == kWrite) op[9] = op[8] == kOpPut ? kPutCompleteSendVals : kRmwCompleteSendVals;
        else op[9] = kReplayCompleteSendVals;
        m_set_state(m, kValid);
    }
}

// hermes_exec_inv, hermesKV.c:489-588
template <int SV>
__device__ __forceinline__ void exec_inv(uint8_t *inv, uint8_t *entry, Meta &m, const Ctx &c)
{
    const bool rmw_on = c.g.rmw_enabled != 0;
    const uint64_t its = e_ts(inv);
    const uint64_t cur = pack_ts(m.ver, m_cid(m));
    const uint8_t inv_rmw = e_rmw(inv);
    if (its >= cur || (rmw_on && inv_rmw)) {
        if (cur < its) {
            uint8_t st = m_state(m);
            if (st == kValid) m_set_state(m, kInvalid);
            else if (st == kWrite || st == kReplay) m_set_state(m, (rmw_on && m_rmw(m)) ? kInvalid : kInvalidWrite);
            m_set_val_len(m, (uint8_t)c.g.kvs_value);
            m_set_rmw(m, inv_rmw);
            m_set_lwid(m, inv[9]);
            copy_value_c<SV>(entry + kEntryValueOff, inv + kOpValueOff, c.g.st_value, c);
            m.ver = (uint32_t)(its >> 8);
            m_set_cid(m, (uint8_t)its);
        } else if (cur == its) {
            if (m_state(m) == kWrite) inv[8] = kInvOutOfGroup;
            m_set_lwid(m, inv[9]);
        } else {  // smaller, RMW INV: answer with an INV-abort carrying the local state
            uint8_t sender = inv[9];
            local_state_to_op<SV>(inv, m, entry, c);
            inv[9] = sender;
            inv[8] = kOpInvAbort;
        }
    }
    if (inv[8] != kOpInvAbort && inv[8] != kInvOutOfGroup) inv[8] = kInvSuccess;
}

// exec_ack's read_write_ops completion of slot `done` (hermesKV.c:660-668): GET -> NEW, PUT ->
// PUT_COMPLETE, RMW -> RMW_COMPLETE; a slot of any other opcode keeps its state, so it is not written.
// The opcode comes from the caller's opcode mirror when the launch has one (c.rwo), else from the op.
__device__ __forceinline__ void complete_rw_slot(const Ctx &c, int done)
{
    uint8_t *w = c.rw + (size_t)done * c.g.op_size;
    const uint8_t oc = c.rwo ? c.rwo[done] : w[8];
    if (oc != kOpGet && oc != kOpPut && oc != kOpRmw) return;
    const uint8_t ns = oc == kOpGet ? kNew : oc == kOpPut ? kPutComplete : kRmwComplete;
    w[9] = ns;
    if (c.rws) c.rws[done] = ns;
}

// hermes_exec_ack, hermesKV.c:591-674
__device__ __forceinline__ void exec_ack(uint8_t *ack, Meta &m, const Ctx &c)
{
    int done = kObiEmpty;
    uint64_t ats = e_ts(ack);
    if (ats == pack_ts(m.llw_ver, m.llw_cid) && m_obi(m) != kObiEmpty) {
        uint8_t sender = ack[9];
        if (sender < 8) m_set_ack_bv(m, (uint8_t)(m_ack_bv(m) | (1u << sender)));
        if (is_last_ack(m_ack_bv(m), c)) {
            done = m_obi(m);
            uint8_t st = m_state(m);
            if (st == kValid || st == kInvalid || st == kInvalidWrite) {
                if (st == kInvalidWrite) m_set_state(m, kInvalid);
                ack[8] = kLastAckNoBcast;
                m_set_obi(m, kObiEmpty);
            } else if (st == kWrite || st == kReplay) {
                m_set_state(m, kValid);
                ack[8] = kLastAckSuccess;
                m_set_obi(m, kObiEmpty);
            }
        }
    }
    if ((ack[8] == kLastAckSuccess || ack[8] == kLastAckNoBcast) && done != kObiEmpty && c.rw_done) {
        *c.rw_done = done;   // the caller completes the slot (complete_rw_slot)
    } else if ((ack[8] == kLastAckSuccess || ack[8] == kLastAckNoBcast) && done != kObiEmpty && c.rw != nullptr) {
        // every completer of this slot writes the same byte (it depends only on the slot's
        // own opcode), so concurrent segments completing one slot are benign
        complete_rw_slot(c, done);
    }
    if (ack[8] != kLastAckSuccess) ack[8] = kAckSuccess;
}


// hermes_exec_val, hermesKV.c:676-703
__device__ __forceinline__ void exec_val(uint8_t *val, Meta &m)
{
    if (e_ts(val) == pack_ts(m.ver, m_cid(m))) m_set_state(m, kValid);
    val[8] = kValSuccess;
}

// hermes_exec_dispatcher, hermesKV.c:847-897
template <int SV>
__device__ __forceinline__ void dispatch(int type, uint8_t *x, uint8_t *entry, uint8_t idx, Meta &m, const Ctx &c)
{
    switch (type) {
    case kLocal: {
        uint8_t oc = x[8];
        if (oc == kOpGet) exec_read<SV>(x, entry, idx, m, c);
        else if (oc == kOpPut) exec_write<SV>(x, entry, idx, m, c);
        else if (c.g.rmw_enabled && oc == kOpRmw) exec_rmw<SV>(x, entry, idx, m, c);
        break;
    }
    case kLocalAfterMemb:
        if (x[8] == kOpPut || x[8] == kOpRmw || x[9] == kInProgressReplay) exec_update_completion(x, m, c);
        break;
    case kInvs: exec_inv<SV>(x, entry, m, c); break;
    case kAcks:
        if (!c.g.rmw_enabled || x[8] == kOpAck) exec_ack(x, m, c);
        else if (x[8] == kOpInvAbort) {
            exec_inv<SV>(x, entry, m, c);
            x[8] = kAckSuccess;
        }
        break;
    case kVals: exec_val(x, m); break;
    default: break;
    }
}

// Sound over-approximation of "executing element x on an entry whose meta is m would change
// m". When it returns false, dispatch() provably leaves m untouched (it may still write the
// element and, for GET/INV-abort, read the entry value). The long-segment engine relies on
// exactly this: non-candidates are resolved in parallel against one snapshot of the meta,
// candidates are applied one at a time in element order.
__device__ __forceinline__ bool would_mutate(int type, const uint8_t *x, const Meta &m, const Ctx &c)
{
    const uint8_t st = m_state(m);
    const bool obi_empty = m_obi(m) == kObiEmpty;
    const uint8_t lw = m_lwid(m);
    const bool lw_alive = lw < 8 && ((c.g_membership >> lw) & 1u);
    const uint64_t cur = pack_ts(m.ver, m_cid(m));
    switch (type) {
    case kLocal: {
        const uint8_t oc = x[8];
        if (oc == kOpGet) return st == kInvalid && !lw_alive && obi_empty;              // replay
        if (oc == kOpPut) return (st == kValid || st == kInvalid) && obi_empty;         // write
        if (oc == kOpRmw && c.g.rmw_enabled) {
            if (x[9] == kInProgressRmw) {                                               // abort + obi clear
                uint64_t ots = e_ts(x);
                return ots < cur && ots == pack_ts(m.llw_ver, m.llw_cid);
            }
            return obi_empty && (st == kValid || (st == kInvalid && !lw_alive));
        }
        return false;
    }
    case kLocalAfterMemb: {
        bool eligible = x[8] == kOpPut || x[8] == kOpRmw || x[9] == kInProgressReplay;
        return eligible && is_last_ack(m_ack_bv(m), c) &&
               (!obi_empty || st == kInvalidWrite || st == kWrite || st == kReplay);
    }
    case kAcks:
        if (!c.g.rmw_enabled || x[8] == kOpAck) {
            if (e_ts(x) != pack_ts(m.llw_ver, m.llw_cid) || obi_empty) return false;
            uint8_t s = x[9];
            uint8_t nb = (uint8_t)(m_ack_bv(m) | (s < 8 ? (1u << s) : 0u));
            return nb != m_ack_bv(m) || is_last_ack(nb, c);
        }
        if (x[8] != kOpInvAbort) return false;
        // an INV-abort element runs hermes_exec_inv: fall through
        [[fallthrough]];
    case kInvs: {
        uint64_t its = e_ts(x);
        return its > cur || (its == cur && lw != (x[9] & 0x7Fu));
    }
    case kVals: return e_ts(x) == cur && st != kValid;
    default: return true;
    }
}

__device__ __forceinline__ bool meta_equal(const Meta &a, const Meta &b)
{
    return a.w4 == b.w4 && (a.w5 & 0xFF00FFFFu) == (b.w5 & 0xFF00FFFFu) && a.ver == b.ver &&
           a.llw_ver == b.llw_ver && a.llw_cid == b.llw_cid;
}

// hermes_skip_dispatcher, hermesKV.c:709-769 (the INV membership-change side effect is
// handled by the lookup kernel, which records the last such element per batch)
__device__ __forceinline__ bool skip_elem_os(int type, uint8_t oc, uint8_t st)
{
    switch (type) {
    case kLocal:
        return st == kPutSuccess || st == kRmwSuccess || st == kReplaySuccess || st == kInProgressPut ||
               st == kInProgressReplay || st == kOpMembChange || st == kPutCompleteSendVals;
    case kLocalAfterMemb:
        return !(st == kInProgressPut || st == kInProgressRmw || st == kInProgressReplay);
    case kInvs: return oc == kOpMembChange;
    case kAcks: return st == kOpMembChange;
    default: return false;
    }
}

__device__ __forceinline__ bool skip_elem(int type, const uint8_t *x) { return skip_elem_os(type, x[8], x[9]); }

}  // namespace hkv
