/*
 * hkv_oracle.c -- TEST INFRASTRUCTURE ONLY. See hkv_oracle.h for scope, pinning and layouts.
 *
 * A straight sequential restatement of the reference batch path. Every function cites the
 * reference function (file:line) whose behaviour it restates. The product (libhermeskv.so)
 * is written independently (element-order rounds with per-key first-candidate words and
 * shadow images, hkv_batch.hip); this file is the single-threaded definition of "what the
 * reference would have produced".
 *
 * The reference seqlock (include/utils/concur_ctrl.h:144-224) is modelled exactly: lock sets
 * the lock byte and bumps the version by one, and each unlock variant applies its own version
 * rule, so every intermediate value the reference computes from a locked version is
 * reproduced. Lock-free snapshot loops (hermesKV.c:81-96) run once: there is one thread and
 * versions are even at batch boundaries (an odd version would make the reference spin forever).
 */
#include "hkv_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- codes (spacetime.h:42-113) */
enum { S_VALID = 1, S_INVALID, S_INVALID_WRITE, S_WRITE, S_REPLAY };
enum {
    OP_GET = 111, OP_PUT, OP_RMW, OP_INV, OP_ACK, OP_VAL, OP_CRD, OP_MEMB_CHANGE, OP_MEMB_COMPLETE
};
enum {
    R_GET_COMPLETE = 121, R_PUT_SUCCESS, R_REPLAY_SUCCESS, R_INV_SUCCESS, R_ACK_SUCCESS,
    R_LAST_ACK_SUCCESS, R_LAST_ACK_NO_BCAST, R_PUT_COMPLETE, R_VAL_SUCCESS, R_MISS,
    R_GET_STALL, R_PUT_STALL, R_PUT_COMPLETE_SEND_VALS, R_SEND_CRD,
    R_RMW_SUCCESS, R_RMW_STALL, R_RMW_COMPLETE, R_RMW_ABORT, R_OP_INV_ABORT
};
enum {
    B_EMPTY = 140, B_NEW, B_COMPLETE, B_IN_PROGRESS_PUT, B_IN_PROGRESS_REPLAY, B_REPLAY_COMPLETE,
    B_IN_PROGRESS_GET, B_REPLAY_COMPLETE_SEND_VALS, B_IN_PROGRESS_RMW, B_RMW_COMPLETE_SEND_VALS
};
enum { F_INV_OUT_OF_GROUP = 153 };
enum { T_LOCAL = 0, T_LOCAL_AFTER_MEMB, T_INVS, T_ACKS, T_VALS };

#define OBI_EMPTY 255       /* ST_OP_BUFFER_INDEX_EMPTY spacetime.h:35 */
#define LWID_EMPTY 127      /* LAST_WRITER_ID_EMPTY spacetime.h:34 */
#define CID_EMPTY 255       /* TIE_BREAKER_ID_EMPTY concur_ctrl.h:14 */
#define OP_META_SIZE 16     /* sizeof(spacetime_op_meta_t) */
#define OBJ_META_SIZE 15    /* sizeof(spacetime_object_meta) */
#define ENTRY_META_OFF 18   /* sizeof(mica_key) + opcode + val_len */

struct hko_kvs {
    hko_config cfg;
    uint32_t st_value;      /* ST_VALUE_SIZE */
    uint32_t kvs_value;     /* KVS_VALUE_SIZE */
    uint32_t entry;         /* sizeof(struct mica_op) */
    uint32_t shift;         /* SHIFT_BITS */
    uint8_t *index;
    uint8_t *log;
    uint64_t bkt_mask, log_mask, log_head;
    int64_t num_insert_op, num_index_evictions;
};

/* ---------------------------------------------------------------- little-endian helpers */
static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

/* op / message fields (spacetime.h:151-185) */
#define O_OPCODE(o) ((o)[8])
#define O_STATE(o) ((o)[9]) /* state for ops, sender for inv/ack/val */
#define O_VALLEN(o) ((o)[10])
#define O_TSCID(o) ((o)[11])
#define O_TSVER(o) ld32((o) + 12)
#define O_SET_TSVER(o, v) st32((o) + 12, (v))
#define O_RMW(o) ((o)[16] & 1u)
#define O_SET_RMW(o, f) ((o)[16] = (uint8_t)(((o)[16] & 0xFEu) | ((f) & 1u)))
#define O_VALUE(o) ((o) + 18)

/* object meta fields (spacetime.h:138-148), m = entry + 18 */
#define M_STATE(m) ((m)[0])
#define M_ACKBV(m) ((m)[1])
#define M_RMW(m) ((m)[2] & 1u)
#define M_SET_RMW(m, f) ((m)[2] = (uint8_t)(((m)[2] & 0xFEu) | ((f) & 1u)))
#define M_LWID(m) ((uint8_t)((m)[2] >> 1))
#define M_SET_LWID(m, w) ((m)[2] = (uint8_t)(((m)[2] & 1u) | (((w) & 0x7Fu) << 1)))
#define M_OBI(m) ((m)[3])
#define M_LOCK(m) ((m)[4])
#define M_TSCID(m) ((m)[5])
#define M_TSVER(m) ld32((m) + 6)
#define M_SET_TSVER(m, v) st32((m) + 6, (v))
#define M_LLWCID(m) ((m)[10])
#define M_LLWVER(m) ld32((m) + 11)
#define M_SET_LLWVER(m, v) st32((m) + 11, (v))

/* ---------------------------------------------------------------- sizes (hrd.h:36-47, mica.h:21-23) */
uint32_t hko_kvs_value_size(const hko_config *c)
{
    return c->big_objects ? c->extra_cache_lines * 64u + 46u : 46u;
}
uint32_t hko_st_value_size(const hko_config *c) { return hko_kvs_value_size(c) - OBJ_META_SIZE; }
uint32_t hko_entry_size(const hko_config *c) { return (ENTRY_META_OFF + hko_kvs_value_size(c) + 7u) & ~7u; }
uint32_t hko_op_size(const hko_config *c) { return (OP_META_SIZE + 2u + hko_st_value_size(c) + 7u) & ~7u; }

/* ---------------------------------------------------------------- CityHash128 (city.c:85-400) */
static const uint64_t CK0 = 0xc3a5c85c97cb3127ULL;
static const uint64_t CK1 = 0xb492b66fbe98f273ULL;
static const uint64_t CK2 = 0x9ae16a3b2f90404fULL;
static const uint64_t CK3 = 0xc949d7c7509e6557ULL;

static uint64_t ch_mix16(uint64_t u, uint64_t v) /* HashLen16 -> Hash128to64, city.c:101-136 */
{
    const uint64_t mul = 0x9ddfea08eb382d69ULL;
    uint64_t a = (u ^ v) * mul;
    a ^= a >> 47;
    uint64_t b = (v ^ a) * mul;
    b ^= b >> 47;
    return b * mul;
}
static uint64_t ch_shiftmix(uint64_t v) { return v ^ (v >> 47); }
static uint64_t ch_rot(uint64_t v, int s) { return s == 0 ? v : (v >> s) | (v << (64 - s)); }

static uint64_t ch_len0to16(const uint8_t *s, size_t len) /* city.c:138-157 */
{
    if (len > 8) {
        uint64_t a = ld64(s), b = ld64(s + len - 8);
        return ch_mix16(a, ch_rot(b + len, (int)len)) ^ b;
    }
    if (len >= 4) {
        uint64_t a = ld32(s);
        return ch_mix16(len + (a << 3), ld32(s + len - 4));
    }
    if (len > 0) {
        uint32_t y = (uint32_t)s[0] + ((uint32_t)s[len >> 1] << 8);
        uint32_t z = (uint32_t)len + ((uint32_t)s[len - 1] << 2);
        return ch_shiftmix(y * CK2 ^ z * CK3) * CK2;
    }
    return CK2;
}

/* CityMurmur for len <= 16 (city.c:276-308); longer inputs are not on the path */
static void ch_murmur_short(const uint8_t *s, size_t len, uint64_t a, uint64_t b,
                            uint64_t *first, uint64_t *second)
{
    uint64_t c, d;
    a = ch_shiftmix(a * CK1) * CK1;
    c = b * CK1 + ch_len0to16(s, len);
    d = ch_shiftmix(a + (len >= 8 ? ld64(s) : c));
    a = ch_mix16(a, c);
    b = ch_mix16(d, b);
    *first = a ^ b;
    *second = ch_mix16(b, a);
}

void hko_cityhash128(const void *sv, size_t len, uint64_t *first, uint64_t *second)
{
    const uint8_t *s = (const uint8_t *)sv;
    if (len >= 16) { /* not used by the path; callers keep len < 16 */
        *first = *second = 0;
        return;
    }
    if (len >= 8) /* city.c:388-394: seeded, empty remaining string */
        ch_murmur_short(NULL, 0, ld64(s) ^ (len * CK0), ld64(s + len - 8) ^ CK1, first, second);
    else          /* city.c:395-398 */
        ch_murmur_short(s, len, CK0, CK1, first, second);
}

void hko_gen_keys(uint64_t *out_second, int64_t n) /* mica.c:149-165 (only .second is a key) */
{
    for (int64_t i = 0; i < n; i++) {
        int32_t id = (int32_t)i;
        uint64_t f, s;
        hko_cityhash128(&id, 4, &f, &s);
        out_second[i] = s;
    }
}

/* ---------------------------------------------------------------- seqlock (concur_ctrl.h:144-213)
 * With the reference's CAS and ordering, so that worker threads can share one table as the
 * reference's workers do (main.c:193-210; the multi-core CPU baseline, hkv_oracle_bench.c). One
 * thread runs exactly the sequential semantics: the CAS always succeeds and every lock-free
 * snapshot validates on its first pass. The version word sits at entry byte 24 (4-aligned). */
static inline void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}
static inline uint32_t ver_load(const uint8_t *m) { return __atomic_load_n((const uint32_t *)(m + 6), __ATOMIC_ACQUIRE); }
static inline void ver_store(uint8_t *m, uint32_t v) { __atomic_store_n((uint32_t *)(m + 6), v, __ATOMIC_RELEASE); }
static inline void lock_release(uint8_t *m) { __atomic_store_n(m + 4, (uint8_t)0, __ATOMIC_RELEASE); }

static void cc_lock(uint8_t *m)
{
    for (;;) {
        while (__atomic_load_n(m + 4, __ATOMIC_RELAXED) == 1) cpu_relax();
        uint8_t expect = 0;
        if (__atomic_compare_exchange_n(m + 4, &expect, (uint8_t)1, 0, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) break;
    }
    ver_store(m, M_TSVER(m) + 1);   /* odd while locked: lock-free readers retry */
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
}
static void cc_unlock_dec(uint8_t *m)
{
    ver_store(m, M_TSVER(m) - 1);
    lock_release(m);
}
static void cc_unlock_custom(uint8_t *m, uint8_t cid, uint32_t version)
{
    __atomic_store_n(m + 5, cid, __ATOMIC_RELAXED);
    ver_store(m, version);
    lock_release(m);
}
static uint32_t cc_unlock_inc(uint8_t *m, uint8_t cid, uint32_t by)
{
    __atomic_store_n(m + 5, cid, __ATOMIC_RELAXED);
    const uint32_t v = M_TSVER(m) + by;
    ver_store(m, v);
    lock_release(m);
    return v;
}

/* byte copy of bytes another thread may be writing (validated by the version afterwards) */
static inline void racy_copy(uint8_t *dst, const uint8_t *src, size_t n)
{
    const volatile uint8_t *s = src;
    for (size_t i = 0; i < n; i++) dst[i] = s[i];
}

/* cctrl_timestamp_is_same_and_valid (concur_ctrl.h:217-224) of a snapshot against the live meta */
static inline int snap_valid(const uint8_t *snap, const uint8_t *m)
{
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint32_t v = M_TSVER(snap);
    return (v & 1u) == 0 && v == ver_load(m) && snap[5] == __atomic_load_n(m + 5, __ATOMIC_RELAXED);
}

/* hermes_lock_free_read_obj_meta, hermesKV.c:81-96 */
static void snapshot(uint8_t *snap, const uint8_t *m)
{
    for (;;) {
        racy_copy(snap, m, OBJ_META_SIZE);
        if (snap_valid(snap, m)) return;
        cpu_relax();
    }
}

static int ts_less(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) /* concur_ctrl.h:70-75 */
{
    return v1 < v2 || (v1 == v2 && c1 < c2);
}
static int ts_equal(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) { return v1 == v2 && c1 == c2; }

/* membership helpers (spacetime.h:253-259, inline-util.h:20-24); membership bytes:
 * [0] num_of_alive_remotes, [1] g_membership, [2] w_ack_init, [3..7] seqlock */
static int memb_is_last_ack(uint8_t ack_bv, const uint8_t *mb) { return (ack_bv & mb[1]) == mb[1]; }
static int memb_has_node(const uint8_t *mb, uint8_t node)
{
    return node < 8 && ((mb[1] >> node) & 1u); /* bv_bit_get asserts node < 8 */
}

/* ---------------------------------------------------------------- exec helpers */
static uint8_t get_val_len(const hko_kvs *kv, const uint8_t *entry) /* spacetime.h:263-267 */
{
    return (uint8_t)((entry[17] >> kv->shift) - OP_META_SIZE);
}

/* hermes_update_actions_n_unlock, hermesKV.c:100-141 (virtual node ids off) */
static void update_and_unlock(hko_kvs *kv, uint8_t *op, uint8_t *entry, uint8_t idx,
                              const uint8_t *mb, uint8_t rmw_flag)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    memcpy(m + OBJ_META_SIZE, O_VALUE(op), kv->st_value);
    entry[17] = (uint8_t)((O_VALLEN(op) >> kv->shift) + OP_META_SIZE);
    M_SET_RMW(m, rmw_flag);
    M_STATE(m) = S_WRITE;
    M_OBI(m) = idx;
    int small_step = !kv->cfg.rmw_enabled || rmw_flag == 1;
    M_SET_LLWVER(m, M_TSVER(m) + (small_step ? 1u : 3u));
    M_ACKBV(m) = mb[2];
    uint8_t node = (uint8_t)kv->cfg.machine_id;
    M_LLWCID(m) = node;
    O_SET_TSVER(op, cc_unlock_inc(m, node, small_step ? 1u : 3u));
    O_SET_RMW(op, rmw_flag);
    O_STATE(op) = rmw_flag == 1 ? R_RMW_SUCCESS : R_PUT_SUCCESS;
    O_TSCID(op) = node;
}

/* hermes_local_state_to_op, hermesKV.c:143-153 (called with the key locked) */
static void local_state_to_op(hko_kvs *kv, uint8_t *op, uint8_t *m)
{
    O_SET_RMW(op, M_RMW(m));
    O_STATE(op) = R_REPLAY_SUCCESS;
    O_SET_TSVER(op, M_TSVER(m) - 1);
    O_TSCID(op) = M_TSCID(m);
    O_VALLEN(op) = (uint8_t)(kv->st_value >> kv->shift);
    memcpy(O_VALUE(op), m + OBJ_META_SIZE, kv->st_value);
}

/* hermes_write_replay_actions, hermesKV.c:155-175 */
static void write_replay(hko_kvs *kv, uint8_t *op, uint8_t idx, uint8_t *m, const uint8_t *mb)
{
    M_STATE(m) = S_REPLAY;
    M_OBI(m) = idx;
    M_SET_LLWVER(m, M_TSVER(m) - 1);
    M_LLWCID(m) = M_TSCID(m);
    M_ACKBV(m) = mb[2];
    local_state_to_op(kv, op, m);
}

/* hermes_check_membership_n_write_replay_actions, hermesKV.c:179-194 */
static void membership_check_replay(hko_kvs *kv, uint8_t *op, uint8_t idx, uint8_t *m, const uint8_t *mb)
{
    if (memb_has_node(mb, M_LWID(m)))
        O_STATE(op) = R_GET_STALL;
    else if (M_OBI(m) == OBI_EMPTY)
        write_replay(kv, op, idx, m, mb);
}

/* hermes_read_actions, hermesKV.c:240-246 */
static void read_into_op(hko_kvs *kv, uint8_t *op, uint8_t *entry)
{
    racy_copy(O_VALUE(op), entry + ENTRY_META_OFF + OBJ_META_SIZE, kv->st_value);
    O_STATE(op) = R_GET_COMPLETE;
    O_VALLEN(op) = get_val_len(kv, entry);
}

/* ---------------------------------------------------------------- skew optimisations (config.h:77-80) */
#define SKEW_READ_COMPLETE 1u
#define SKEW_WRITE_COALESCE 2u

/* hermes_complete_hot_read_optimization, hermesKV.c:224-238 */
static void hot_read_complete(uint8_t *op, uint32_t ts_ver, uint8_t ts_cid)
{
    if (O_STATE(op) != R_GET_STALL) return;
    if (O_TSVER(op) == 0 && O_TSCID(op) == 0) {   /* first stall: remember the timestamp */
        O_SET_TSVER(op, ts_ver);
        O_TSCID(op) = ts_cid;
    } else if (O_TSVER(op) + 1u < ts_ver) {      /* two versions later: complete (no value copied) */
        O_STATE(op) = R_GET_COMPLETE;
    }
}

/* hermes_marshal_write_coalesce_optimization, hermesKV.c:196-206 (the IN_PROGRESS_PUT it sets is
 * overwritten with PUT_STALL by its caller) */
static void write_coalesce_mark(hko_kvs *kv, uint8_t *op, uint16_t curr_version)
{
    if ((kv->cfg.skew_flags & SKEW_WRITE_COALESCE) && O_TSVER(op) == 0) {
        O_SET_TSVER(op, curr_version);
        O_STATE(op) = B_IN_PROGRESS_PUT;
    }
}

/* hermes_complete_coalesced_write, hermesKV.c:208-221 */
static void write_coalesce_complete(hko_kvs *kv, uint8_t *op, uint16_t curr_ts)
{
    if ((kv->cfg.skew_flags & SKEW_WRITE_COALESCE) && O_STATE(op) == R_PUT_STALL)
        if (O_TSVER(op) > 0 && O_TSVER(op) + 1u < (uint32_t)curr_ts) O_STATE(op) = R_PUT_COMPLETE;
}

/* ---------------------------------------------------------------- exec functions */
/* hermes_exec_read, hermesKV.c:251-311: a lock-free pass (copy the meta, act on the live state,
 * validate the copy's timestamp afterwards), or a locked one for INVALID keys */
static void ex_read(hko_kvs *kv, uint8_t *op, uint8_t *entry, uint8_t idx, const uint8_t *mb)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    uint8_t prev[OBJ_META_SIZE];
    int locked = 0;
    uint32_t cur_ver;
    uint8_t cur_cid;
    O_STATE(op) = B_EMPTY;
    do {
        racy_copy(prev, m, OBJ_META_SIZE);
        cur_ver = M_TSVER(prev);
        cur_cid = M_TSCID(prev);
        switch (__atomic_load_n(m, __ATOMIC_ACQUIRE)) {
        case S_VALID: read_into_op(kv, op, entry); break;
        case S_INVALID_WRITE: case S_WRITE: case S_REPLAY: O_STATE(op) = R_GET_STALL; break;
        default:
            locked = 1;
            cc_lock(m);
            cur_ver = M_TSVER(m) - 1;   /* "when locking we do version++" */
            cur_cid = M_TSCID(m);
            switch (M_STATE(m)) {
            case S_VALID: read_into_op(kv, op, entry); break;
            case S_INVALID_WRITE: case S_WRITE: case S_REPLAY: O_STATE(op) = R_GET_STALL; break;
            case S_INVALID: membership_check_replay(kv, op, idx, m, mb); break;
            default: break;
            }
            cc_unlock_dec(m);
            break;
        }
    } while (!snap_valid(prev, m) && !locked);
    if (kv->cfg.skew_flags & SKEW_READ_COMPLETE) hot_read_complete(op, cur_ver, cur_cid);
}

/* hermes_exec_write, hermesKV.c:314-356 */
static void ex_write(hko_kvs *kv, uint8_t *op, uint8_t *entry, uint8_t idx, const uint8_t *mb)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    O_STATE(op) = B_EMPTY;
    cc_lock(m);
    const uint16_t curr_version = (uint16_t)(M_TSVER(m) - 1);
    switch (M_STATE(m)) {
    case S_VALID: case S_INVALID:
        if (M_OBI(m) != OBI_EMPTY) {
            cc_unlock_dec(m);
            write_coalesce_mark(kv, op, curr_version);
        } else {
            update_and_unlock(kv, op, entry, idx, mb, 0);
        }
        break;
    case S_INVALID_WRITE: case S_WRITE:
        write_coalesce_mark(kv, op, curr_version);
        cc_unlock_dec(m);
        break;
    case S_REPLAY:
        cc_unlock_dec(m);
        break;
    default: break;
    }
    if (O_STATE(op) != R_PUT_SUCCESS) O_STATE(op) = R_PUT_STALL;
    write_coalesce_complete(kv, op, curr_version);
}

/* hermes_exec_rmw, hermesKV.c:358-428 */
static void ex_rmw(hko_kvs *kv, uint8_t *op, uint8_t *entry, uint8_t idx, const uint8_t *mb)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    if (O_STATE(op) == B_IN_PROGRESS_RMW) {
        uint8_t snap[OBJ_META_SIZE];
        snapshot(snap, m);
        if (ts_less(O_TSVER(op), O_TSCID(op), M_TSVER(snap), M_TSCID(snap))) {
            O_STATE(op) = R_RMW_ABORT;
            cc_lock(m);
            if (ts_equal(O_TSVER(op), O_TSCID(op), M_LLWVER(snap), M_LLWCID(snap)))
                M_OBI(m) = OBI_EMPTY;
            cc_unlock_dec(m);
        }
        return;
    }
    O_STATE(op) = B_EMPTY;
    cc_lock(m);
    switch (M_STATE(m)) {
    case S_VALID:
        if (M_OBI(m) != OBI_EMPTY) cc_unlock_dec(m);
        else update_and_unlock(kv, op, entry, idx, mb, 1);
        break;
    case S_INVALID:
        membership_check_replay(kv, op, idx, m, mb);
        /* fall through */
    case S_INVALID_WRITE: case S_WRITE: case S_REPLAY:
        cc_unlock_dec(m);
        break;
    default: break;
    }
    if (O_STATE(op) != R_RMW_SUCCESS && O_STATE(op) != R_REPLAY_SUCCESS) O_STATE(op) = R_RMW_STALL;
}

/* hermes_exec_check_update_completion, hermesKV.c:430-484 */
static void ex_update_completion(hko_kvs *kv, uint8_t *op, uint8_t *entry, const uint8_t *mb)
{
    (void)kv;
    uint8_t *m = entry + ENTRY_META_OFF;
    uint8_t snap[OBJ_META_SIZE];
    snapshot(snap, m);
    if (!memb_is_last_ack(M_ACKBV(snap), mb)) return;
    cc_lock(m);
    if (memb_is_last_ack(M_ACKBV(m), mb)) {
        M_OBI(m) = OBI_EMPTY;
        switch (M_STATE(m)) {
        case S_INVALID_WRITE:
            M_STATE(m) = S_INVALID;
            /* fall through */
        case S_VALID: case S_INVALID:
            O_STATE(op) = O_OPCODE(op) == OP_PUT ? R_PUT_COMPLETE : R_RMW_COMPLETE;
            break;
        case S_WRITE: case S_REPLAY:
            O_SET_TSVER(op, M_TSVER(m) - 1);
            O_TSCID(op) = M_TSCID(m);
            if (M_STATE(m) == S_WRITE)
                O_STATE(op) = O_OPCODE(op) == OP_PUT ? R_PUT_COMPLETE_SEND_VALS : B_RMW_COMPLETE_SEND_VALS;
            else
                O_STATE(op) = B_REPLAY_COMPLETE_SEND_VALS;
            M_STATE(m) = S_VALID;
            break;
        default: break;
        }
    }
    cc_unlock_dec(m);
}

/* hermes_exec_inv, hermesKV.c:489-588 */
static void ex_inv(hko_kvs *kv, uint8_t *inv, uint8_t *entry)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    const int rmw_on = kv->cfg.rmw_enabled != 0;
    uint32_t iv = O_TSVER(inv);
    uint8_t ic = O_TSCID(inv);
    uint8_t snap[OBJ_META_SIZE];
    snapshot(snap, m);
    if (!ts_less(iv, ic, M_TSVER(snap), M_TSCID(snap)) || (rmw_on && O_RMW(inv) == 1)) {
        cc_lock(m);
        if (ts_less(M_TSVER(m) - 1, M_TSCID(m), iv, ic)) {
            switch (M_STATE(m)) {
            case S_VALID: M_STATE(m) = S_INVALID; break;
            case S_WRITE: case S_REPLAY:
                M_STATE(m) = (rmw_on && M_RMW(m) == 1) ? S_INVALID : S_INVALID_WRITE;
                break;
            default: break;
            }
            entry[17] = (uint8_t)kv->kvs_value;
            M_SET_RMW(m, O_RMW(inv));
            M_SET_LWID(m, O_STATE(inv));
            memcpy(m + OBJ_META_SIZE, O_VALUE(inv), kv->st_value);
            cc_unlock_custom(m, ic, iv);
        } else if (ts_equal(M_TSVER(m) - 1, M_TSCID(m), iv, ic)) {
            if (M_STATE(m) == S_WRITE) O_OPCODE(inv) = F_INV_OUT_OF_GROUP;
            M_SET_LWID(m, O_STATE(inv));
            cc_unlock_custom(m, ic, iv);
        } else {
            if (rmw_on && O_RMW(inv) == 1) {
                uint8_t sender = O_STATE(inv);
                local_state_to_op(kv, inv, m);
                O_STATE(inv) = sender;
                O_OPCODE(inv) = R_OP_INV_ABORT;
            }
            cc_unlock_dec(m);
        }
    }
    if (O_OPCODE(inv) != R_OP_INV_ABORT && O_OPCODE(inv) != F_INV_OUT_OF_GROUP)
        O_OPCODE(inv) = R_INV_SUCCESS;
}

/* hermes_exec_ack, hermesKV.c:591-674 */
static void ex_ack(hko_kvs *kv, uint8_t *ack, uint8_t *entry, const uint8_t *mb, uint8_t *rw, uint32_t op_size)
{
    (void)kv;
    uint8_t *m = entry + ENTRY_META_OFF;
    int done_idx = OBI_EMPTY;
    uint32_t av = O_TSVER(ack);
    uint8_t ac = O_TSCID(ack);
    uint8_t snap[OBJ_META_SIZE];
    snapshot(snap, m);
    if (ts_equal(av, ac, M_LLWVER(snap), M_LLWCID(snap))) {
        cc_lock(m);
        if (M_OBI(m) != OBI_EMPTY && ts_equal(av, ac, M_LLWVER(m), M_LLWCID(m))) {
            uint8_t sender = O_STATE(ack);
            if (sender < 8) M_ACKBV(m) = (uint8_t)(M_ACKBV(m) | (1u << sender));
            if (memb_is_last_ack(M_ACKBV(m), mb)) {
                done_idx = M_OBI(m);
                switch (M_STATE(m)) {
                case S_VALID: case S_INVALID:
                    O_OPCODE(ack) = R_LAST_ACK_NO_BCAST;
                    M_OBI(m) = OBI_EMPTY;
                    break;
                case S_INVALID_WRITE:
                    M_STATE(m) = S_INVALID;
                    O_OPCODE(ack) = R_LAST_ACK_NO_BCAST;
                    M_OBI(m) = OBI_EMPTY;
                    break;
                case S_WRITE: case S_REPLAY:
                    M_STATE(m) = S_VALID;
                    O_OPCODE(ack) = R_LAST_ACK_SUCCESS;
                    M_OBI(m) = OBI_EMPTY;
                    break;
                default: break;
                }
            }
        }
        cc_unlock_dec(m);
    }
    if ((O_OPCODE(ack) == R_LAST_ACK_SUCCESS || O_OPCODE(ack) == R_LAST_ACK_NO_BCAST) &&
        done_idx != OBI_EMPTY && rw != NULL) {
        uint8_t *w = rw + (size_t)done_idx * op_size;
        switch (O_OPCODE(w)) {
        case OP_GET: O_STATE(w) = B_NEW; break;
        case OP_PUT: O_STATE(w) = R_PUT_COMPLETE; break;
        case OP_RMW: O_STATE(w) = R_RMW_COMPLETE; break;
        default: break;
        }
    }
    if (O_OPCODE(ack) != R_LAST_ACK_SUCCESS) O_OPCODE(ack) = R_ACK_SUCCESS;
}

/* hermes_exec_val, hermesKV.c:676-703 */
static void ex_val(uint8_t *val, uint8_t *entry)
{
    uint8_t *m = entry + ENTRY_META_OFF;
    uint8_t snap[OBJ_META_SIZE];
    snapshot(snap, m);
    if (ts_equal(M_TSVER(snap), M_TSCID(snap), O_TSVER(val), O_TSCID(val))) {
        cc_lock(m);
        if (ts_equal(M_TSVER(m) - 1, M_TSCID(m), O_TSVER(val), O_TSCID(val))) M_STATE(m) = S_VALID;
        cc_unlock_dec(m);
    }
    O_OPCODE(val) = R_VAL_SUCCESS;
}

/* ---------------------------------------------------------------- skip + dispatch (hermesKV.c:709-897) */
static int skip_elem(int type, uint8_t *e, int *node_suspected)
{
    uint8_t st = O_STATE(e);
    switch (type) {
    case T_LOCAL:
        return st == R_PUT_SUCCESS || st == R_RMW_SUCCESS || st == R_REPLAY_SUCCESS ||
               st == B_IN_PROGRESS_PUT || st == B_IN_PROGRESS_REPLAY || st == OP_MEMB_CHANGE ||
               st == R_PUT_COMPLETE_SEND_VALS;
    case T_LOCAL_AFTER_MEMB:
        return !(st == B_IN_PROGRESS_PUT || st == B_IN_PROGRESS_RMW || st == B_IN_PROGRESS_REPLAY);
    case T_INVS:
        if (O_OPCODE(e) == OP_MEMB_CHANGE) {
            if (node_suspected) *node_suspected = O_VALUE(e)[0];
            return 1;
        }
        return 0;
    case T_ACKS: return st == OP_MEMB_CHANGE;
    default: return 0;
    }
}

static void dispatch(hko_kvs *kv, int type, uint8_t *e, uint8_t *entry, const uint8_t *mb,
                     uint8_t idx, uint8_t *rw)
{
    uint32_t op_size = hko_op_size(&kv->cfg);
    switch (type) {
    case T_LOCAL:
        if (O_OPCODE(e) == OP_GET) ex_read(kv, e, entry, idx, mb);
        else if (O_OPCODE(e) == OP_PUT) ex_write(kv, e, entry, idx, mb);
        else if (kv->cfg.rmw_enabled && O_OPCODE(e) == OP_RMW) ex_rmw(kv, e, entry, idx, mb);
        break;
    case T_LOCAL_AFTER_MEMB:
        if (O_OPCODE(e) == OP_PUT || O_OPCODE(e) == OP_RMW || O_STATE(e) == B_IN_PROGRESS_REPLAY)
            ex_update_completion(kv, e, entry, mb);
        break;
    case T_INVS: ex_inv(kv, e, entry); break;
    case T_ACKS:
        if (!kv->cfg.rmw_enabled || O_OPCODE(e) == OP_ACK) ex_ack(kv, e, entry, mb, rw, op_size);
        else if (O_OPCODE(e) == R_OP_INV_ABORT) {
            ex_inv(kv, e, entry);
            O_OPCODE(e) = R_ACK_SUCCESS;
        }
        break;
    case T_VALS: ex_val(e, entry); break;
    default: break;
    }
}

uint8_t *hko_lookup(hko_kvs *kv, uint64_t key)
{
    const uint8_t *bkt = kv->index + (key & 0xFFFFFFFFFFFFULL & kv->bkt_mask) * 64u;
    uint32_t tag = (uint32_t)(key >> 48);
    for (int j = 0; j < 8; j++) {
        uint64_t slot = ld64(bkt + 8 * j);
        if ((slot & 1u) && ((slot >> 1) & 0x7FFFFFu) == tag) {
            uint64_t off = slot >> 24;
            uint8_t *entry = kv->log + (off & kv->log_mask);
            if (kv->log_head - off >= kv->cfg.log_cap) entry = NULL;
            if (entry && ld64(entry + 8) == key) return entry;
            return NULL;
        }
    }
    return NULL;
}

/* hermes_batch_ops_to_KVS, hermesKV.c:905-996: pass 1 skip + bucket, pass 2 slot probe,
 * pass 3 key compare + exec in array order, else ST_MISS into byte 9 */
void hko_batch(hko_kvs *kv, int type, uint8_t *ops, int op_num, uint16_t esz,
               const uint8_t membership[8], int *node_suspected, uint8_t *rw)
{
    if (op_num <= 0) return;
    uint8_t **entry = (uint8_t **)calloc((size_t)op_num, sizeof(uint8_t *));
    /* passes 1+2: the index is immutable during a batch, so the lookup can be done up front */
    for (int i = 0; i < op_num; i++) {
        uint8_t *e = ops + (size_t)esz * i;
        if (skip_elem(type, e, node_suspected)) continue;
        uint64_t key = ld64(e);
        const uint8_t *bkt = kv->index + (key & 0xFFFFFFFFFFFFULL & kv->bkt_mask) * 64u;
        uint32_t tag = (uint32_t)(key >> 48);
        for (int j = 0; j < 8; j++) {
            uint64_t slot = ld64(bkt + 8 * j);
            if ((slot & 1u) && ((slot >> 1) & 0x7FFFFFu) == tag) {
                uint64_t off = slot >> 24;
                entry[i] = kv->log + (off & kv->log_mask);
                if (kv->log_head - off >= kv->cfg.log_cap) entry[i] = NULL;
                break;
            }
        }
    }
    for (int i = 0; i < op_num; i++) {
        uint8_t *e = ops + (size_t)esz * i;
        if (skip_elem(type, e, node_suspected)) continue;
        if (entry[i] != NULL && ld64(entry[i] + 8) == ld64(e))
            dispatch(kv, type, e, entry[i], membership, (uint8_t)i, rw);
        else
            O_STATE(e) = R_MISS;
    }
    free(entry);
}

void hko_batch_multi(hko_kvs *kv, int type, uint8_t *ops, int n_batches, int stride,
                     const int32_t *counts, uint16_t esz, const uint8_t membership[8],
                     int32_t *node_suspected, uint8_t *rw, int64_t rw_stride)
{
    for (int b = 0; b < n_batches; b++) {
        int ns = node_suspected ? node_suspected[b] : -1;
        hko_batch(kv, type, ops + (size_t)b * stride * esz, counts ? counts[b] : stride, esz,
                  membership, &ns, rw ? rw + (size_t)b * rw_stride : NULL);
        if (node_suspected) node_suspected[b] = ns;
    }
}

/* ---------------------------------------------------------------- init + populate */
hko_kvs *hko_create(const hko_config *c) /* mica_init, mica.c:17-76 */
{
    hko_kvs *kv = (hko_kvs *)calloc(1, sizeof(hko_kvs));
    kv->cfg = *c;
    kv->kvs_value = hko_kvs_value_size(c);
    kv->st_value = hko_st_value_size(c);
    kv->entry = hko_entry_size(c);
    kv->shift = c->big_objects ? 3u : 0u;
    kv->bkt_mask = c->num_bkts - 1;
    kv->log_mask = c->log_cap - 1;
    kv->log_head = 0;
    kv->index = (uint8_t *)calloc(c->num_bkts, 64);
    /* slack so an entry that straddles the physical end stays in bounds */
    kv->log = (uint8_t *)calloc(c->log_cap + kv->entry, 1);
    return kv;
}

void hko_destroy(hko_kvs *kv)
{
    if (!kv) return;
    free(kv->index);
    free(kv->log);
    free(kv);
}

void hko_set_machine_id(hko_kvs *kv, uint32_t machine_id) { kv->cfg.machine_id = machine_id; }

/* mica_insert_one, mica.c:78-146 */
static void mica_insert(hko_kvs *kv, const uint8_t *img)
{
    uint64_t key = ld64(img + 8);
    uint8_t *bkt = kv->index + ((key & 0xFFFFFFFFu) & kv->bkt_mask) * 64u;
    uint32_t tag = (uint32_t)(key >> 48);
    kv->num_insert_op++;
    int use = -1;
    for (int i = 0; i < 8; i++) {
        uint64_t slot = ld64(bkt + 8 * i);
        if (((slot >> 1) & 0x7FFFFFu) == tag || (slot & 1u) == 0) use = i;
    }
    if (use == -1) {
        use = (int)(tag & 7u);
        kv->num_index_evictions++;
    }
    st64(bkt + 8 * use, 1u | ((uint64_t)tag << 1) | (kv->log_head << 24));
    memcpy(kv->log + (kv->log_head & kv->log_mask), img, kv->entry);
    kv->log_head += kv->entry;
    kv->log_head = (kv->log_head + 7) & ~7ULL;
    if (kv->cfg.log_cap - kv->log_head <= (uint64_t)kv->kvs_value + 32)
        kv->log_head = (kv->log_head + kv->cfg.log_cap) & ~kv->log_mask;
}

/* spacetime_populate_fixed_len, spacetime.c:32-68 (+ spacetime_object_meta_init :17-23).
 * The reference leaves ack_bv, RMW_flag and last_local_write_ts as stack garbage; both this
 * oracle and the product define them as zero. */
void hko_populate(hko_kvs *kv, int64_t n, int val_len)
{
    uint8_t *img = (uint8_t *)calloc(1, kv->entry);
    uint8_t *m = img + ENTRY_META_OFF;
    img[16] = OP_PUT;
    img[17] = (uint8_t)(val_len >> kv->shift);
    M_STATE(m) = S_VALID;
    M_SET_LWID(m, LWID_EMPTY);
    M_OBI(m) = OBI_EMPTY;
    M_LOCK(m) = 0;
    M_TSCID(m) = CID_EMPTY;
    M_SET_TSVER(m, 0);
    for (int64_t i = n - 1; i >= 0; i--) {
        int32_t id = (int32_t)i;
        uint64_t f, s;
        hko_cityhash128(&id, 4, &f, &s);
        st64(img, f);
        st64(img + 8, s);
        memset(m + OBJ_META_SIZE, (int)(uint8_t)('a' + (i % 20)), kv->st_value);
        mica_insert(kv, img);
    }
    free(img);
}

uint8_t *hko_index(hko_kvs *kv) { return kv->index; }
uint8_t *hko_log(hko_kvs *kv) { return kv->log; }
uint64_t hko_log_head(hko_kvs *kv) { return kv->log_head; }
int64_t hko_num_index_evictions(hko_kvs *kv) { return kv->num_index_evictions; }

/* lets the CPU baseline start from a table image copied out of HBM */
void hko_set_log_head(hko_kvs *kv, uint64_t head) { kv->log_head = head; }

/* ---------------------------------------------------------------- test hooks
 * The seqlock / timestamp / ack-quorum restatements above, exported so tests/test_oracle.py can
 * compare them with the reference's own concur_ctrl.h / bit_vector.h (oracle/ref_prims.c).
 * cc: 6 bytes {lock, tie_breaker_id, version} as conc_ctrl_t; variant 0 dec, 1 inc,
 * 2 inc_by_three, 3 custom. Returns the version an inc variant reports, else 0. */
uint32_t hko_test_cctrl_lock_unlock(uint8_t *cc, int variant, uint8_t cid, uint32_t version)
{
    uint8_t buf[32] __attribute__((aligned(8)));
    uint8_t *m = buf + 2;   /* the version word 4-aligned, as at entry byte 24 */
    uint32_t resp = 0;
    memset(buf, 0, sizeof buf);
    memcpy(m + 4, cc, 6);
    cc_lock(m);
    switch (variant) {
    case 0: cc_unlock_dec(m); break;
    case 1: resp = cc_unlock_inc(m, cid, 1u); break;
    case 2: resp = cc_unlock_inc(m, cid, 3u); break;
    default: cc_unlock_custom(m, cid, version); break;
    }
    memcpy(cc, m + 4, 6);
    return resp;
}

int hko_test_ts_less(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) { return ts_less(v1, c1, v2, c2); }
int hko_test_ts_equal(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) { return ts_equal(v1, c1, v2, c2); }

int hko_test_is_last_ack(uint8_t ack_bv, const uint8_t membership[8]) { return memb_is_last_ack(ack_bv, membership); }
int hko_test_has_node(const uint8_t membership[8], uint8_t node) { return memb_has_node(membership, node); }

/* the key's current version through a lock-free read (the CPU baseline's virtual peers) */
uint32_t hko_key_version(hko_kvs *kv, uint64_t key)
{
    uint8_t *e = hko_lookup(kv, key);
    if (!e) return 0;
    uint8_t snap[OBJ_META_SIZE];
    snapshot(snap, e + ENTRY_META_OFF);
    return M_TSVER(snap);
}
