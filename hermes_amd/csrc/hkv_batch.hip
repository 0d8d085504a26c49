// hkv_batch.hip -- the HermesKV batch path on gfx950 (hermes_batch_ops_to_KVS, hermesKV.c:905-996).
//
// One launch applies n_batches batches of one type. Its result is defined as the reference
// applying them element by element in concatenation order. Nothing is sorted: elements stay in
// element order, and the elements of each key are resolved in rounds.
//
//   k_lookup    one element per 4 lanes, in element order: skip test (hermesKV.c:709-769),
//               bucket probe over the 64-B bucket (hermesKV.c:952-975), wrap test, 8-B key
//               compare (hermesKV.c:977-993; a miss writes ST_MISS into byte 9). A hit reads
//               the key's object meta S_0 from the same log line and offers itself as round
//               0's first candidate if would_mutate(elem, S_0) (hkv_exec.h).
//   round r     every key keeps F_r, the smallest element index among its candidates (one
//               atomicMin on the F word of the key's log line). Then
//                 k_resolve: an element before F_r (or of a key without a candidate) sees S_r in
//                   the sequential order and S_r does not change under it: it runs the
//                   reference's exec function on a private copy of S_r against the live entry,
//                   in parallel with everything else. F_r itself runs the exec function on a
//                   shadow image of the entry (S_r -> S_{r+1}), so the entry still holds S_r for
//                   every concurrent reader; later elements stay pending.
//                 k_cand (r+1): every pending element tests would_mutate against S_{r+1}, read
//                   from the shadow of round r's first candidate; k_commit copies each key's
//                   last shadow into its entry once, after the last round.
//   fallback    elements still pending after the last round (keys mutated in every round) are
//               gathered per key into workgroup-owned lists (key -> workgroup by its last first
//               candidate), sorted by element index in LDS, and finished in element order: runs
//               of up to 32 by one thread, longer runs by the whole workgroup with block-wide
//               first-candidate passes over chunks (k_fb_exec).
//
// Exactness rests on one property: would_mutate() is sound (false => the exec function leaves
// the meta unchanged). Every resolved element checks it: a private copy that did change raises
// bit 0 of *error_flags, which every parity test asserts is zero.
//
// Slots and F words are tagged with the launch (key word) and the round (F word), so no scratch
// is cleared between launches: a slot whose tag is older reads as empty, and a newer round's F
// value is numerically smaller than every older one, so atomicMin replaces stale words.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "hkv_exec.h"
#include "hkv_internal.h"

namespace hkv {

constexpr uint32_t kNone = 0xFFFFFFFFu;
// per-element stage between passes; kStCommit: the element's shadow holds its key's latest state
// (committed to the entry by k_commit unless a later round's first candidate supersedes it)
enum : uint8_t { kStDone = 0, kStCommit = 1, kStPend = 2 };
enum { kCtrFbM = 1, kCtrFbL = 2 };  // fallback: mem cursor, list length

struct BatchArgs {
    uint8_t *elems;
    const int32_t *counts;
    const int32_t *offsets;      // packed INV/VAL launches (counts NULL, stride = n): batch offsets
    const uint8_t *index;
    uint8_t *log;
    uint8_t *rw;
    int32_t *ns_idx;
    unsigned long long *fw;      // [log_cap / 64] F word per 64-B log line (table-wide), see fw_index
    unsigned long long *fx, *fy; // [log_cap / 64] INV words X, Y (INV direct path; zero between launches)
    unsigned long long *ft;      // [log_cap / 64][8] ACK words T (ACK direct path; epoch << 32 | ~i)
    uint32_t fw_mask;
    uint32_t *ent;               // [n] entry id of every element (kNone: skipped or missing)
    uint8_t *st;                 // [n] stage (kSt*)
    uint32_t *pf;                // [n] pending element: its key's first candidate of the last round
    uint8_t *shadow;             // [cap][entry_size] entry image a round's first candidate produced
    unsigned long long *mem;     // [2 cap] fallback (F_R, element) pairs of workgroups with more than kFbLds
    uint32_t *fbl;               // [cap] fallback list: elements still pending after the last round
    uint32_t *ctr;               // kCtr*
    unsigned int *error_flags;
    Geometry g;
    int64_t n;
    int64_t rw_stride;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint32_t rtag0;              // round 0's tag; round r uses rtag0 + r
    uint8_t ltag;                // launch tag (1..255) in the seqlock byte of keys with a round-0 candidate
    int32_t rounds;              // rounds after round 0 before the fallback
    int32_t inv_direct;          // INV launch on the direct path (k_inv_resolve)
    int32_t ack_direct;          // ACK launch on the direct path (k_ack_resolve)
    uint8_t g_membership;
    uint8_t w_ack_init;
    int32_t *node_suspected;     // small launches write it themselves
    int32_t n_batches;
    const uint8_t *host_src;     // small launches staged in host memory (BatchLaunch)
    uint8_t *host_dst;
    uint8_t *dev_region;
    uint64_t region_bytes;
    uint32_t *done_flag;
    uint32_t done_value;
    unsigned long long *prof;    // HKV_SMALL_PROF: phase timestamps of k_small (debug)
    const SmallBatch *hdr;       // mixed small launches: the batch headers (in dev_region)
    uint8_t *state_out;          // local launches: each element's final state byte (may be NULL)
    const uint8_t *opc;          // local launches: the caller's opcode mirror (may be NULL, see k_local_pre)
    const uint8_t *patch;        // local direct path: pending header writes (hkv_batch_desc.d_patch), or NULL
    uint16_t *fk;                // local launches with RMWs: [n] each round-0 candidate's kind of mutation (fk_kind,
                                 // k_lookup), so k_resolve0_direct can resolve the elements after an absorbing F
    uint64_t *hx;                // big local launches with patches (patch_in_resolve): [2 n] each patched element's
                                 // header word (bytes 8..15) as patched and its op's last 8-byte word, from
                                 // k_lookup for k_resolve0_direct; NULL otherwise
    uint8_t *rws;                // ACK launches: read_write_ops state mirror (hkv_batch_desc.d_rw_state), or NULL
    const uint8_t *rwo;          // ACK launches: read_write_ops opcode mirror (hkv_batch_desc.d_opcode_in), or NULL
    int32_t n_rows, skip_row;    // HKV_BATCH_ROWS: rows applied in order (k_unique_rows), one skipped (-1: none)
    int64_t row_stride;          // elements between rows
    int32_t dbg;                 // HKV_DBG: timing experiments that skip work (results invalid); always 0
                                 // unless the library is built with -DHKV_DEBUG_MODES (HKV_DBG_ON)
    int32_t check_unique;        // HKV_CHECK_UNIQUE: HKV_BATCH_UNIQUE launches verify their keys are unique
    uint8_t *ack_out;            // INV launches: each element's ACK (hkv_batch_desc.d_ack_out), or NULL
    uint32_t ack_out_size;
};

// Rounds after round 0 per batch type: how often a hot key usually mutates in one launch beyond
// the first time. An ACK batch sets an ack bit and then completes; INVs carry at most a few
// distinct timestamps per key and launch. Keys that mutate more go to the fallback.
// None for VAL batches and for local batches without RMWs: their first mutation leaves the key in
// an absorbing state (absorbing_state), so k_resolve0 finishes every key.
__host__ __device__ constexpr int rounds_for(int type, bool rmw)
{
    return type == kVals || (type == kLocal && !rmw) ? 0 : 2;
}

// The state a key is in after any mutation by an element of this batch type, when that state
// makes every later element of the launch a non-mutating one whose result depends on the state
// alone (rounds_for == 0):
//   local, RMWs off: a mutation is a PUT (update_actions -> WRITE, hermesKV.c:100-141) or a GET
//     replay (-> REPLAY, :155-175); under either, GETs stall (:279-282) and PUTs stall (:352-354).
//   VALs: hermes_exec_val only ever sets VALID (:676-703) and its opcode is VAL_SUCCESS whatever
//     the state; under VALID no VAL mutates.
template <int TYPE>
__device__ __forceinline__ uint8_t absorbing_state()
{
    return TYPE == kVals ? kValid : kWrite;
}

// The meta every element after F (its key's only mutation in the launch) runs against, from S_0.
// Without the skew optimisations only the absorbing state matters. With them, a stalled GET or
// PUT also reads the timestamp and tells WRITE from REPLAY (hermesKV.c:196-238), so the meta is
// S_1 itself: after a PUT, update_actions' WRITE with version + 2 and this machine's cid
// (hermesKV.c:100-141, RMWs off); after a GET replay, REPLAY with the timestamp unchanged
// (:155-175). f_is_put: F is known to be a PUT (else its opcode is read).
template <int TYPE>
__device__ __forceinline__ Meta after_first(const BatchArgs &a, const Meta &m0, uint32_t f, int f_is_put)
{
    Meta m1 = m0;
    m_set_state(m1, absorbing_state<TYPE>());
    if (TYPE != kLocal || a.g.skew == 0) return m1;
    uint8_t foc = f_is_put ? (uint8_t)kOpPut : a.elems[(int64_t)f * a.esz + 8];
    if (a.hx && !f_is_put) {   // patch_in_resolve: F's op may not be patched yet (its patch is valid at byte 14)
        const uint64_t pb = *reinterpret_cast<const uint64_t *>(a.patch + (int64_t)f * 16 + 8);
        if ((pb >> 48) & 0xFFu) foc = (uint8_t)pb;
    }
    if (foc != kOpGet) {
        m1.ver += 2;
        m_set_cid(m1, (uint8_t)a.g.machine_id);
    } else {
        m_set_state(m1, kReplay);
    }
    return m1;
}

// INV direct path (INV launches without RMWs, fewer than 2^23 elements). Without RMWs,
// hermes_exec_inv (hermesKV.c:489-588) on one key, element by element from S_0, comes to this:
// let M be the largest INV timestamp of the key's elements.
//   M > ts_0:  the first element with ts M (A) installs its value, RMW flag and M; the state moves
//              once (VALID -> INVALID, WRITE/REPLAY -> INVALID_WRITE, others stay), val_len :=
//              KVS_VALUE_SIZE; last_writer_id := sender of the last element with ts M (B).
//   M = ts_0:  last_writer_id := sender of the last element with ts ts_0 (B); nothing else.
//   M < ts_0:  nothing.
// Every element's opcode is INV_SUCCESS (an INV_ABORT / OUT_OF_GROUP input stays), except
// OUT_OF_GROUP for an element with ts = ts_0 in state WRITE, which holds until the first element
// with a larger ts (P). Per key (log line) three words:
//   X = max over raising elements of (ts << 24 | ~i) -> M and A (k_lookup);
//   F = round 0's word: P, offered by raising elements of keys in state WRITE (k_lookup);
//   Y = 1 + B when B != A (k_inv_resolve), or for keys without a raise.
// k_lookup finishes the elements below ts_0; k_inv_resolve writes the other opcodes, A keeps X in
// its own scratch slot (mem[A]) and the other elements with ts M flag A's slot pf[A] ("B is not
// A") and raise Y; in k_inv_commit A (or, without a raise, B) applies the key's meta and clears X
// and Y. Most keys of a launch have one element: it is A and B, never touches Y, and commits from
// its own slots without reading X again.
enum : uint8_t { kIvRaise = 1, kIvEq = 2, kIvWrite = 4, kIvCand = 8, kIvApply = 16 };
constexpr int64_t kInvDirectMax = 1 << 23;

// ACK direct path (ACK launches without RMWs). Without RMWs, hermes_exec_ack (hermesKV.c:591-674)
// changes a key only through ACKs that match its pending write (ts = last local write's ts, op
// buffer index set): each ORs its sender's bit into ack_bv, and the first one after which ack_bv
// covers the group membership G completes the write (op buffer index := EMPTY, INVALID_WRITE ->
// INVALID, WRITE/REPLAY -> VALID, the read_write_op slot completes; LAST_ACK_SUCCESS from WRITE or
// REPLAY). The ACKs never change the timestamp they match against, so with T[s] = the first
// matching element of sender s (s < 8) and N = G minus the bits already set, that element is
//   j* = max over s in N of T[s] (none if some T[s] is missing), or the first matching element
//        of any sender when N is empty (min of the T[s] and F, the first match from a sender >= 8).
// Without a completion the applier is the first match of a sender < 8 (only those set bits).
// ack_bv ends as ack_bv | the bits of the senders whose T[s] <= j* (every T[s] without a
// completion). Opcodes: ACK_SUCCESS (a LAST_ACK_SUCCESS input stays, except at j*),
// LAST_ACK_SUCCESS for j* from WRITE or REPLAY. k_lookup finishes the non-matching elements, sets T (as max of ~i) and F
// and caches each matching element's ack_bv / state / op buffer index in pf; in k_ack_resolve
// j* (or, without a completion, F) applies the key's meta. T words carry the launch's epoch in
// their upper half, so a word of an earlier launch reads as empty and nothing is cleared (the
// epoch only wraps after 2^29 launches, when the runtime zeroes T with the F words' reset).
// Measured against u32 words with an 11-bit tag and a 1/2048 slice of T zeroed by every ACK
// launch: the slice memset is a kernel of its own (4.6 us), as long as the clear pass it replaced.
enum : uint8_t { kAkMatch = 1 };

__device__ __forceinline__ uint8_t ack_opcode(uint8_t in) { return in == kLastAckSuccess ? in : kAckSuccess; }

__device__ __forceinline__ uint8_t inv_opcode(uint8_t in, bool oog)
{
    return oog ? kInvOutOfGroup : (in == kOpInvAbort || in == kInvOutOfGroup) ? in : kInvSuccess;
}

__device__ __forceinline__ Ctx make_ctx(const BatchArgs &a)
{
    Ctx c;
    c.g = a.g;
    c.g_membership = a.g_membership;
    c.w_ack_init = a.w_ack_init;
    c.rw = nullptr;
    c.rws = nullptr;
    c.rw_done = nullptr;
    c.vc = nullptr;
    return c;
}

// The batch holding element i and its first element: i / stride, or for a packed launch the last
// batch whose offset is <= i (empty batches share their successor's offset)
__device__ __forceinline__ int32_t batch_of(const BatchArgs &a, int64_t i, int64_t &start)
{
    if (!a.offsets) {
        const int32_t b = (int32_t)(i / a.stride);
        start = (int64_t)b * a.stride;
        return b;
    }
    int lo = 0, hi = a.n_batches - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.offsets[mid] <= i) lo = mid; else hi = mid - 1;
    }
    start = a.offsets[lo];
    return lo;
}

__device__ __forceinline__ void elem_at(const BatchArgs &a, uint32_t i, uint8_t *&x, uint8_t &idx, Ctx &c)
{
    c.rw = nullptr;
    c.rws = nullptr;
    idx = 0;
    if (a.rw || !a.offsets) {  // packed INV / VAL elements need neither (exec_inv / exec_val)
        int64_t start;
        const int32_t b = batch_of(a, i, start);
        idx = (uint8_t)(i - start);
        c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
        c.rws = a.rws ? a.rws + (int64_t)b * (a.rw_stride / a.g.op_size) : nullptr;
        c.rwo = a.rwo ? a.rwo + (int64_t)b * (a.rw_stride / a.g.op_size) : nullptr;
    }
    x = a.elems + (int64_t)i * a.esz;
}

// the state mirror of a local launch: written by whichever pass finishes the element
__device__ __forceinline__ void note_state(const BatchArgs &a, int64_t i, const uint8_t *x)
{
    if (a.state_out) a.state_out[i] = x[9];
}

__device__ __forceinline__ uint64_t phys_of(const BatchArgs &a, uint32_t e) { return (uint64_t)e * a.g.entry_unit; }
__device__ __forceinline__ uint8_t *entry_of(const BatchArgs &a, uint32_t e) { return a.log + phys_of(a, e); }
// Live entries never overlap and are at least 64 B long, so their first 64-B lines are distinct.
// The F word of line l sits at l * odd mod 2^k (a bijection on the log's 2^k lines): keys that are
// neighbours in the log -- the hottest ids of a populated table are -- get F words on different
// lines, and memory-side atomics on one line serialise.
__device__ __forceinline__ uint32_t fw_index(const BatchArgs &a, uint64_t phys)
{
    return (uint32_t)(((phys >> 6) * 0x9E3779B1ull) & a.fw_mask);
}
__device__ __forceinline__ unsigned long long *fw_of(const BatchArgs &a, uint32_t e) { return a.fw + fw_index(a, phys_of(a, e)); }

__device__ __forceinline__ uint32_t first_cand(unsigned long long f, uint32_t rtag)
{
    return (uint32_t)(f >> 32) == ~rtag ? (uint32_t)f : kNone;
}

// F_r: atomicMin of ((~round tag) << 32 | element). The load filters most offers of a hot key:
// F only falls, and elements are dispatched roughly in element order.
__device__ __forceinline__ void offer(unsigned long long *f, uint32_t rtag, uint32_t i)
{
    const unsigned long long v = ((unsigned long long)(~rtag) << 32) | i;
    if (v < __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(f, v);
}

// Wave-aggregated atomicAdd(&arr[j], 1): one atomic per distinct j in the wave; each active lane
// gets its own ticket. All 64 lanes must call it.
__device__ __forceinline__ uint32_t agg_ticket(uint32_t *arr, uint32_t j, bool active)
{
    const int lane = threadIdx.x & 63;
    uint32_t ticket = 0;
    unsigned long long left = __ballot(active);
    while (left) {
        const int leader = __ffsll((long long)left) - 1;
        const uint32_t jl = __shfl(j, leader, 64);
        const unsigned long long m = left & __ballot(active && j == jl);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&arr[jl], (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        if ((m >> lane) & 1ull) ticket = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        left &= ~m;
    }
    return ticket;
}

// x: the element (global), or its LDS copy
template <int TYPE, int SV>
__device__ __forceinline__ void resolve_elem(const BatchArgs &a, uint32_t i, uint8_t *x, uint8_t *entry,
                                             VCopy *vc = nullptr)
{
    Ctx c = make_ctx(a);
    c.vc = vc;
    uint8_t *xg;
    uint8_t idx;
    elem_at(a, i, xg, idx, c);
    Meta m;
    meta_load(entry, m);
    Meta t = m;
    dispatch<SV>(TYPE, x, entry, idx, t, c);
    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
}

__device__ __forceinline__ uint8_t *shadow_of(const BatchArgs &a, uint32_t i)
{
    return a.shadow + (size_t)i * a.g.entry_size;
}

// entries and shadows are 8-byte aligned and a multiple of 8 long: 16-B words, then one 8-B word
__device__ __forceinline__ void copy_entry(uint8_t *dst, const uint8_t *src, uint32_t bytes)
{
    struct __attribute__((aligned(8))) W16 {
        uint64_t a, b;
    };
    uint32_t o = 0;
    for (; o + 16 <= bytes; o += 16) *reinterpret_cast<W16 *>(dst + o) = *reinterpret_cast<const W16 *>(src + o);
    if (o < bytes) *reinterpret_cast<uint64_t *>(dst + o) = *reinterpret_cast<const uint64_t *>(src + o);
}

// The round's first candidate of a key: S_r (read from src: the entry in round 0, the previous
// round's shadow later) -> S_{r+1}, written to the element's own shadow image, so the round's
// other elements, resolved concurrently, still read S_r. Later rounds read the shadow; the key's
// last shadow is committed to the entry once, by k_commit.
template <int TYPE, int SV>
__device__ __forceinline__ void apply_to_shadow(const BatchArgs &a, uint8_t *x, uint32_t i, const uint8_t *src)
{
    uint8_t *sh = shadow_of(a, i);
    Meta m;
    meta_load(src, m);
    if (SV == 31) {  // 64-B entries and shadows are 16-byte aligned
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(sh);
        const uint4 w0 = s4[0], w1 = s4[1], w2 = s4[2], w3 = s4[3];
        d4[0] = w0;
        d4[1] = w1;
        d4[2] = w2;
        d4[3] = w3;
    } else {
        copy_entry(sh, src, a.g.entry_size);
    }
    Ctx c = make_ctx(a);
    uint8_t *xg;
    uint8_t idx;
    elem_at(a, i, xg, idx, c);
    // x: the element's LDS copy (k_resolve0), or null: the element in global memory. Two calls,
    // not one on a select of the two, so each keeps its address space (no flat accesses).
    if (x) dispatch<SV>(TYPE, x, sh, idx, m, c);
    else dispatch<SV>(TYPE, xg, sh, idx, m, c);
    meta_store(sh, m);
}

// apply_to_shadow for big entries, by the whole wave (every lane calls it; cand: this lane's element
// is its key's first candidate, src its S_r): the wave copies S_r into the candidates' shadows
// (wave_block_copies), then each candidate runs its exec function on its shadow with the value
// copy recorded in vc (made by wave_value_copies after it), instead of one lane copying 320 + 287
// bytes in dependent steps while the rest of its wave waits.
__device__ __forceinline__ void wave_block_copies(uint8_t *dst, const uint8_t *src, uint32_t bytes);
template <int TYPE, int SV>
__device__ __forceinline__ void apply_to_shadow_wave(const BatchArgs &a, bool cand, uint32_t i, const uint8_t *src,
                                                     VCopy &vc, uint8_t *xl = nullptr, bool use_xl = false)
{
    uint8_t *sh = cand ? shadow_of(a, i) : nullptr;
    wave_block_copies(sh, src, a.g.entry_size);
    __threadfence_block();   // the shadows' bytes before any lane reads or rewrites them
    if (!cand) return;
    Meta m;
    meta_load(src, m);
    Ctx c = make_ctx(a);
    c.vc = &vc;
    uint8_t *xg;
    uint8_t idx;
    elem_at(a, i, xg, idx, c);
    if (use_xl) dispatch<SV>(TYPE, xl, sh, idx, m, c);   // xl: the element's patched copy (k_resolve0_direct)
    else dispatch<SV>(TYPE, xg, sh, idx, m, c);
    meta_store(sh, m);
}

// ------------------------------------------------------------------ k_lookup (+ round 0 candidates)
// Four lanes per element: each lane reads 16 bytes (two slots) of the element's 64-byte bucket,
// so one load instruction covers a whole bucket line per element. Slots are searched in the
// reference's order (first tag match wins, hermesKV.c:954-975). Each lane group carries
// kLookupPair elements through the three dependent loads (op header, bucket, log line) side by
// side, so twice as many loads are in flight per wave. A hit that would mutate its key's meta as
// it stands (S_0) offers itself as round 0's first candidate. The key compare and the meta load
// together once the slot is known; a candidate then loads its F word, which filters the offer (a
// hot key's later candidates see a smaller F and issue no atomic). Non-candidates never touch F:
// the batch is bound by random 64-B lines, and one less per element beats the shorter dependence
// chain of loading F beside the meta. The launch is split: a short head over the
// first kLookupHead elements gives every hot key a small F first, because at the start of one big
// launch some 10^5 elements are in flight before any F is set, and a hot key's candidates among
// them would all reach its F word (atomics on one address serialise).
//
// VAL batches finish here: hermes_exec_val (hermesKV.c:676-703) never changes a timestamp, so
// every VAL of a launch compares against its key's timestamp at launch start, sets VALID iff they
// match and reports VAL_SUCCESS whatever the state. The VALs of a key commute, and the matching
// ones all store the same state byte.
// 16 bytes at an 8-byte aligned address (op headers, log lines): one dwordx4 access
struct __attribute__((aligned(8))) U64x2 {
    uint64_t a, b;
};

// esz (a multiple of 8) bytes between 8-byte aligned buffers, 16 B per access
__device__ __forceinline__ void copy_elem(uint8_t *dst, const uint8_t *src, int32_t esz)
{
    for (int32_t o = 0; o + 16 <= esz; o += 16)
        *reinterpret_cast<U64x2 *>(dst + o) = *reinterpret_cast<const U64x2 *>(src + o);
    if (esz & 8) *reinterpret_cast<uint64_t *>(dst + esz - 8) = *reinterpret_cast<const uint64_t *>(src + esz - 8);
}

// bytes 8..15 of an op after its refill patch (second patch word pb, see patch_valid): opcode,
// ST_NEW, val_len; the timestamp (bytes 11..15) kept unless the patch resets it
__device__ __forceinline__ uint64_t patched_hdr(uint64_t h, uint64_t pb)
{
    const bool reset = ((pb >> 40) & 0xFFu) != 0;
    const uint64_t low = (pb & 0xFFu) | ((uint64_t)kNew << 8) | (((pb >> 8) & 0xFFu) << 16);
    return reset ? low : (low | (h & ~0xFFFFFFull));
}
__device__ __forceinline__ bool patch_valid(uint64_t pb);

// Local launches with RMWs: how a round-0 candidate (would_mutate against S_0) changes its key, from its
// header word h (bytes 8..15) and S_0 -- bits 0..1: 1 update_actions (a PUT, or an RMW from VALID;
// hermesKV.c:100-141), 2 a write replay (a GET, or an RMW from INVALID: :155-194), 3 anything else (an
// in-progress RMW's abort); bit 2 the RMW flag; bits 8..15 the op's val_len byte. The first two leave the
// key in an absorbing state for the rest of the launch (WRITE or REPLAY with the op buffer index set: every
// later GET, PUT and RMW stalls, and no in-progress RMW matches the new last-local-write timestamp), so the
// elements after F resolve against S_1 (after_first_rmw) in k_resolve0_direct instead of later rounds.
enum : uint16_t { kFkWrite = 1, kFkReplay = 2, kFkOther = 3 };
__device__ __forceinline__ uint16_t fk_kind(uint64_t h, const Meta &m0)
{
    const uint8_t oc = (uint8_t)h, st = (uint8_t)(h >> 8);
    uint16_t k = kFkOther;
    if (oc == kOpPut) k = kFkWrite;
    else if (oc == kOpGet) k = kFkReplay;
    else if (oc == kOpRmw && st != kInProgressRmw) k = m_state(m0) == kValid ? kFkWrite : kFkReplay;
    return (uint16_t)(k | (oc == kOpRmw ? 4u : 0u) | (((h >> 16) & 0xFFu) << 8));
}
// S_1 after F (kind fk, at batch index idx) from S_0, as update_actions / write_replay leave it
__device__ __forceinline__ Meta after_first_rmw(const BatchArgs &a, const Meta &m0, uint16_t fk, uint8_t idx)
{
    Meta m = m0;
    if ((fk & 3u) == kFkWrite) {
        const uint8_t rmw_flag = (fk >> 2) & 1u;
        m_set_val_len(m, (uint8_t)(((uint8_t)(fk >> 8) >> a.g.shift) + kOpMetaSize));
        m_set_rmw(m, rmw_flag);
        m_set_state(m, kWrite);
        m_set_obi(m, idx);
        const uint32_t step = (!a.g.rmw_enabled || rmw_flag == 1) ? 2u : 4u;
        const uint8_t node = (uint8_t)a.g.machine_id;
        m.llw_ver = m.ver + step;
        m.llw_cid = node;
        m_set_ack_bv(m, a.w_ack_init);
        m.ver += step;
        m_set_cid(m, node);
    } else {
        m_set_state(m, kReplay);
        m_set_obi(m, idx);
        m.llw_ver = m.ver;
        m.llw_cid = m_cid(m);
        m_set_ack_bv(m, a.w_ack_init);
    }
    return m;
}

constexpr int64_t kLookupHead = 8192;
constexpr int kLookupPair = 2;
// Four lanes (q = lane & 3) look up kLookupPair keys side by side: the 64-B bucket (16 B per
// lane), the reference's slot order (first tag match, hermesKV.c:954-975), the log window
// (:969-970), then each lane's 16 B of the 64-B log line (bytes 16q..16q+15). All four lanes of a
// group call it with the same arguments.
template <int P = kLookupPair>
__device__ __forceinline__ void lookup_pair(const BatchArgs &a, const uint64_t *key, const bool *probe, int q,
                                            int gbase, bool *ok, uint64_t *phys, uint4 *ln)
{
    uint4 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k)
        v[k] = probe[k] ? reinterpret_cast<const uint4 *>(a.index + ((key[k] & 0xFFFFFFFFFFFFULL) & a.g.bkt_mask) * 64u)[q]
                        : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint64_t s0 = (uint64_t)v[k].x | ((uint64_t)v[k].y << 32);
        const uint64_t s1 = (uint64_t)v[k].z | ((uint64_t)v[k].w << 32);
        const uint32_t tag = (uint32_t)(key[k] >> 48);
        const bool mt0 = probe[k] && (s0 & 1u) && ((uint32_t)(s0 >> 1) & 0x7FFFFFu) == tag;
        const bool mt1 = probe[k] && (s1 & 1u) && ((uint32_t)(s1 >> 1) & 0x7FFFFFu) == tag;
        const uint32_t g0 = (uint32_t)(__ballot(mt0) >> gbase) & 0xFu;
        const uint32_t g1 = (uint32_t)(__ballot(mt1) >> gbase) & 0xFu;
        uint32_t o = 0;  // bit 2*l + j: slot 2*l + j matches
#pragma unroll
        for (int l = 0; l < 4; ++l) o |= ((g0 >> l) & 1u) << (2 * l) | ((g1 >> l) & 1u) << (2 * l + 1);
        const int first = o ? __ffs(o) - 1 : 0;
        const uint64_t off = __shfl((first & 1) ? (s1 >> 24) : (s0 >> 24), first >> 1, 4);
        ok[k] = probe[k] && o && a.g.log_head - off < a.g.log_cap;
        phys[k] = off & a.g.log_mask;
    }
#pragma unroll
    for (int k = 0; k < P; ++k)
        ln[k] = ok[k] ? reinterpret_cast<const uint4 *>(a.log + phys[k])[q] : make_uint4(0u, 0u, 0u, 0u);
}

// lookup_pair that also loads each hit's F word beside its log line (lane q == 0; ~0 for a miss), so a
// key's F costs no dependent load after the line (k_local_fused)
template <int P>
__device__ __forceinline__ void lookup_pair_f(const BatchArgs &a, const uint64_t *key, const bool *probe, int q,
                                              int gbase, bool *ok, uint64_t *phys, uint4 *ln, unsigned long long *fwv)
{
    uint4 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k)
        v[k] = probe[k] ? reinterpret_cast<const uint4 *>(a.index + ((key[k] & 0xFFFFFFFFFFFFULL) & a.g.bkt_mask) * 64u)[q]
                        : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint64_t s0 = (uint64_t)v[k].x | ((uint64_t)v[k].y << 32);
        const uint64_t s1 = (uint64_t)v[k].z | ((uint64_t)v[k].w << 32);
        const uint32_t tag = (uint32_t)(key[k] >> 48);
        const bool mt0 = probe[k] && (s0 & 1u) && ((uint32_t)(s0 >> 1) & 0x7FFFFFu) == tag;
        const bool mt1 = probe[k] && (s1 & 1u) && ((uint32_t)(s1 >> 1) & 0x7FFFFFu) == tag;
        const uint32_t g0 = (uint32_t)(__ballot(mt0) >> gbase) & 0xFu;
        const uint32_t g1 = (uint32_t)(__ballot(mt1) >> gbase) & 0xFu;
        uint32_t o = 0;
#pragma unroll
        for (int l = 0; l < 4; ++l) o |= ((g0 >> l) & 1u) << (2 * l) | ((g1 >> l) & 1u) << (2 * l + 1);
        const int first = o ? __ffs(o) - 1 : 0;
        const uint64_t off = __shfl((first & 1) ? (s1 >> 24) : (s0 >> 24), first >> 1, 4);
        ok[k] = probe[k] && o && a.g.log_head - off < a.g.log_cap;
        phys[k] = off & a.g.log_mask;
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        ln[k] = ok[k] ? reinterpret_cast<const uint4 *>(a.log + phys[k])[q] : make_uint4(0u, 0u, 0u, 0u);
        fwv[k] = ok[k] && q == 0 ? a.fw[fw_index(a, phys[k])] : ~0ull;
    }
}


template <int P = kLookupPair>
__global__ __launch_bounds__(256) void k_lookup(BatchArgs a, int64_t i_begin, int64_t i_end)
{
    const int q = threadIdx.x & 3;
    const int lane = threadIdx.x & 63;
    const int gbase = lane & ~3;
    if (i_begin == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctr[kCtrFbM] = 0;
        a.ctr[kCtrFbL] = 0;
    }
    const bool vals_direct = a.type == kVals;
    int64_t gi[P];
    uint64_t key[P], hdr[P], tail[P];
    int probe[P];
    bool patched[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        gi[k] = i_begin + ((int64_t)blockIdx.x * P + k) * 64 + (threadIdx.x >> 2);
        uint64_t kk = 0, hh = 0;
        int p = 0;
        patched[k] = false;
        tail[k] = 0;
        if (gi[k] < i_end && q == 0) {
            const int32_t b = (int32_t)(gi[k] / a.stride);
            const int32_t idx = (int32_t)(gi[k] - (int64_t)b * a.stride);
            const bool counted = a.counts == nullptr || idx < a.counts[b];
            if (a.hx) {
                // patch_in_resolve: the element as its patch makes it (k_resolve0_direct writes the op), and
                // its op's last word -- on the line of the next op's header, which the next lane group reads
                const uint8_t *x = a.elems + gi[k] * a.esz;
                const U64x2 h = *reinterpret_cast<const U64x2 *>(x);
                const U64x2 pt = *reinterpret_cast<const U64x2 *>(a.patch + gi[k] * 16);
                tail[k] = *reinterpret_cast<const uint64_t *>(x + a.esz - 8);
                patched[k] = patch_valid(pt.b);
                kk = patched[k] ? pt.a : h.a;
                hh = patched[k] ? patched_hdr(h.b, pt.b) : h.b;
            }
            if (counted) {
                if (!a.hx) {
                    const U64x2 h = *reinterpret_cast<const U64x2 *>(a.elems + gi[k] * a.esz);
                    kk = h.a;
                    hh = h.b;
                }
                if (skip_elem_os(a.type, (uint8_t)hh, (uint8_t)(hh >> 8))) {
                    if (a.type == kInvs && a.ns_idx) {
                        int64_t start;  // packed: a search, for the rare membership-change INVs only
                        const int32_t bb = a.offsets ? batch_of(a, gi[k], start) : b;
                        atomicMax(&a.ns_idx[bb], a.offsets ? (int32_t)(gi[k] - start) : idx);
                    }
                } else {
                    p = 1;
                }
            }
        }
        key[k] = kk;
        hdr[k] = hh;
        probe[k] = p;
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int p = __shfl(probe[k], 0, 4);
        const uint64_t kk = __shfl(key[k], 0, 4);
        probe[k] = p;
        key[k] = kk;
    }
    // bucket, then the log line (lookup_pair: four lanes per element, 16 B each)
    bool ok[P];
    uint64_t phys[P], ekey[P];
    Meta m0[P];
    U64x2 ln[P];
    {
        bool pr[P];
        uint4 l4[P];
#pragma unroll
        for (int k = 0; k < P; ++k) pr[k] = probe[k] != 0;
        lookup_pair<P>(a, key, pr, q, gbase, ok, phys, l4);
#pragma unroll
        for (int k = 0; k < P; ++k)
            ln[k] = U64x2{(uint64_t)l4[k].x | ((uint64_t)l4[k].y << 32), (uint64_t)l4[k].z | ((uint64_t)l4[k].w << 32)};
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        ekey[k] = __shfl(ln[k].b, 0, 4);
        const uint64_t w45 = __shfl(ln[k].a, 1, 4), w67 = __shfl(ln[k].b, 1, 4);
        const uint32_t b32 = (uint32_t)__shfl(ln[k].a, 2, 4) & 0xFFu;
        m0[k].w4 = (uint32_t)w45;
        m0[k].w5 = (uint32_t)(w45 >> 32);
        m0[k].ver = (uint32_t)w67;
        m0[k].llw_cid = (uint8_t)(w67 >> 32);
        m0[k].llw_ver = (uint32_t)(w67 >> 40) | (b32 << 24);
    }
    if (q != 0) return;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (gi[k] >= i_end) continue;
        uint8_t *x = a.elems + gi[k] * a.esz;
        uint32_t e = kNone;
        uint8_t ifl = 0;
        if (ok[k] && ekey[k] == key[k]) {
            e = (uint32_t)(phys[k] / a.g.entry_unit);
            uint8_t *entry = a.log + phys[k];
            if (vals_direct) {
                const uint64_t its = pack_ts((uint32_t)(hdr[k] >> 32), (uint8_t)(hdr[k] >> 24));
                if (its == pack_ts(m0[k].ver, m_cid(m0[k])) && m_state(m0[k]) != kValid) entry[kEntryMetaOff] = kValid;
                x[8] = kValSuccess;
            } else if (a.ack_direct) {
                const uint64_t ats = pack_ts((uint32_t)(hdr[k] >> 32), (uint8_t)(hdr[k] >> 24));
                if (ats != pack_ts(m0[k].llw_ver, m0[k].llw_cid) || m_obi(m0[k]) == kObiEmpty) {
                    x[8] = ack_opcode((uint8_t)hdr[k]);
                } else {
                    ifl = kAkMatch;
                    const uint32_t w = fw_index(a, phys[k]);
                    const uint8_t snd = (uint8_t)(hdr[k] >> 8);
                    // F: the first match of a sender without a T word, or of any sender when the
                    // quorum is complete already (the first match then completes)
                    if (snd >= 8 || (uint8_t)(a.g_membership & ~m_ack_bv(m0[k])) == 0)
                        offer(a.fw + w, a.rtag0, (uint32_t)gi[k]);
                    if (snd < 8) {  // tagged with the launch: no clearing between launches
                        unsigned long long *t = a.ft + (size_t)w * 8 + snd;
                        const unsigned long long tv = ((unsigned long long)(a.rtag0 >> 3) << 32) | (0xFFFFFFFFu - (uint32_t)gi[k]);
                        if (tv > __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(t, tv);
                    }
                    a.pf[gi[k]] = (uint32_t)m_ack_bv(m0[k]) | ((uint32_t)m_state(m0[k]) << 8) | ((uint32_t)m_obi(m0[k]) << 16);
                }
            } else if (a.inv_direct) {
                const uint64_t its = pack_ts((uint32_t)(hdr[k] >> 32), (uint8_t)(hdr[k] >> 24));
                const uint64_t cur = pack_ts(m0[k].ver, m_cid(m0[k]));
                if (its < cur) {
                    x[8] = inv_opcode((uint8_t)hdr[k], false);
                } else if (its == cur) {
                    ifl = kIvEq | (m_state(m0[k]) == kWrite ? kIvWrite : 0);
                } else {
                    ifl = kIvRaise;
                    a.pf[gi[k]] = 0;  // "B is not A" flag, should this element be A
                    const uint32_t w = fw_index(a, phys[k]);
                    const unsigned long long xv = (its << 24) | (0x7FFFFFull - (uint64_t)gi[k]);
                    if (xv > __hip_atomic_load(a.fx + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(a.fx + w, xv);
                    if (m_state(m0[k]) == kWrite) offer(a.fw + w, a.rtag0, (uint32_t)gi[k]);
                }
            } else {
                uint64_t h2[2] = {0, hdr[k]};
                Ctx c = make_ctx(a);
                if (would_mutate(a.type, reinterpret_cast<const uint8_t *>(h2), m0[k], c)) {
                    if (a.fk) a.fk[gi[k]] = fk_kind(hdr[k], m0[k]);
                    const unsigned long long vv = ((unsigned long long)(~a.rtag0) << 32) | (uint32_t)gi[k];
                    unsigned long long *fw = a.fw + fw_index(a, phys[k]);
                    if (vv < __hip_atomic_load(fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(fw, vv);
                    // the seqlock byte is free at batch boundaries (concur_ctrl.h: the lock is held
                    // only inside one exec call): it tells k_resolve0 which keys have a candidate,
                    // so the others skip the F word; the key's commit clears it
                    if ((uint8_t)(m0[k].w5 >> 16) != a.ltag) entry[kEntryMetaOff + 4] = a.ltag;
                }
            }
        }
        if (patched[k]) {   // k_resolve0_direct writes the op's header from this word
            const uint64_t h = probe[k] && e == kNone ? (hdr[k] & ~0xFF00ull) | ((uint64_t)kMiss << 8) : hdr[k];
            *reinterpret_cast<U64x2 *>(a.hx + 2 * gi[k]) = U64x2{h, tail[k]};
        } else if (probe[k] && e == kNone) {
            x[9] = kMiss;
        }
        a.ent[gi[k]] = e;
        if (a.inv_direct || a.ack_direct) a.st[gi[k]] = ifl;
    }
}

// INV direct path: opcodes of the elements at or above ts_0, A marks itself, the other elements
// with ts M (or, without a raise, all of them) set Y. The load before each atomicMax filters the
// offers of a key with many INVs (Y only rises).
__global__ __launch_bounds__(256) void k_inv_resolve(BatchArgs a, int64_t i_begin, int64_t i_end)
{
    const int64_t i = i_begin + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= i_end) return;
    const uint8_t fl = a.st[i];
    if (fl == 0) return;
    const uint32_t w = fw_index(a, phys_of(a, a.ent[i]));
    uint8_t *x = a.elems + i * a.esz;
    const uint64_t hdr = *reinterpret_cast<const uint64_t *>(x + 8);
    const uint64_t its = pack_ts((uint32_t)(hdr >> 32), (uint8_t)(hdr >> 24));
    const unsigned long long X = a.fx[w];  // M and A are final (k_lookup)
    bool oog = false, y = false;
    if (X != 0) {  // some element raises the key's ts
        // in state WRITE, an element at ts_0 is out of group until the first raise P (offered by
        // every raising element of a key in state WRITE, so it exists)
        if (fl & kIvWrite) oog = (uint32_t)i < first_cand(a.fw[w], a.rtag0);
        const uint32_t ia = 0x7FFFFFu - (uint32_t)(X & 0x7FFFFFu);
        if ((uint32_t)i == ia) {
            a.st[i] = kIvApply;
            a.mem[i] = X;
        } else if (its == (uint64_t)(X >> 24)) {
            y = true;
            if (a.pf[ia] == 0) a.pf[ia] = 1;  // every writer stores the same value
        }
    } else {       // no raise: every flagged element of the key is at ts_0, B applies
        oog = (fl & kIvWrite) != 0;
        y = true;
        a.st[i] = kIvCand;
    }
    x[8] = inv_opcode((uint8_t)hdr, oog);
    if (y) {
        const unsigned long long yv = (unsigned long long)i + 1;
        if (yv > __hip_atomic_load(a.fy + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(a.fy + w, yv);
    }
}

// A of a raising key applies the key's meta to a 64-B entry (31-B values): entry bytes 16..63
// (meta, value) and the element's bytes 16..63 (flags, value) move as three 16-B words each, the
// new entry image is put together in registers.
__device__ __forceinline__ void inv_apply64(const BatchArgs &a, int64_t i, uint32_t w, uint8_t *entry,
                                            unsigned long long X)
{
    union Img {
        U64x2 q[3];
        uint64_t d[6];
    };
    Img en, el;
    const U64x2 *pe = reinterpret_cast<const U64x2 *>(entry + 16);
    const U64x2 *px = reinterpret_cast<const U64x2 *>(a.elems + i * a.esz + 16);
#pragma unroll
    for (int k = 0; k < 3; ++k) en.q[k] = pe[k];
    el.q[0] = px[0];  // the 56-B element ends at image byte 40: bytes 16..55 only
    el.q[1] = px[1];
    el.d[4] = *reinterpret_cast<const uint64_t *>(px + 2);
    el.d[5] = 0;
    int64_t b = i;
    if (a.pf[i]) {  // B is not A
        b = (int64_t)a.fy[w] - 1;
        a.fy[w] = 0;
    }
    const uint8_t lw = a.elems[b * a.esz + 9];
    Meta m;
    m.w4 = (uint32_t)en.d[0];
    m.w5 = (uint32_t)(en.d[0] >> 32);
    m.ver = (uint32_t)en.d[1];
    m.llw_cid = (uint8_t)(en.d[1] >> 32);
    m.llw_ver = (uint32_t)(en.d[1] >> 40) | ((uint32_t)(en.d[2] & 0xFFu) << 24);
    const uint64_t M = X >> 24;
    const uint8_t st = m_state(m);
    if (st == kValid) m_set_state(m, kInvalid);
    else if (st == kWrite || st == kReplay) m_set_state(m, kInvalidWrite);
    m_set_val_len(m, (uint8_t)a.g.kvs_value);
    m_set_rmw(m, (uint8_t)(el.d[0] & 1u));  // element byte 16: RMW_flag
    m_set_lwid(m, lw);
    m.ver = (uint32_t)(M >> 8);
    m_set_cid(m, (uint8_t)M);
    // value: element bytes 18..48 -> entry bytes 33..63, i.e. image byte 2 + k -> 17 + k: the
    // element image shifted up by 15 bytes = 120 bits (one word and 56 bits)
    uint64_t v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint64_t lo = k >= 2 ? el.d[k - 2] : 0, hi = k >= 1 ? el.d[k - 1] : 0;
        v[k] = (hi << 56) | (lo >> 8);
    }
    // bytes 0..15 of the image: meta (seqlock byte free), byte 16: llw_ver's top byte, 17..47: value
    Img out;
    out.d[0] = (uint64_t)m.w4 | ((uint64_t)(m.w5 & 0xFF00FFFFu) << 32);
    out.d[1] = (uint64_t)m.ver | ((uint64_t)m.llw_cid << 32) | ((uint64_t)m.llw_ver << 40);
    out.d[2] = (uint64_t)(uint8_t)(m.llw_ver >> 24) | (v[2] & ~0xFFull);
    out.d[3] = v[3];
    out.d[4] = v[4];
    out.d[5] = v[5];
    U64x2 *po = reinterpret_cast<U64x2 *>(entry + 16);
#pragma unroll
    for (int k = 0; k < 3; ++k) po[k] = out.q[k];
    a.fx[w] = 0;
}

// INV direct path: A (or, without a raise, B) applies its key's meta and clears X and Y.
template <int SV>
__global__ __launch_bounds__(256) void k_inv_commit(BatchArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t fl = a.st[i];
    if (fl != kIvApply && fl != kIvCand) return;
    const uint32_t e = a.ent[i];
    const uint32_t w = fw_index(a, phys_of(a, e));
    int64_t b = i;  // B
    if (fl == kIvCand) {
        if (a.fy[w] != (unsigned long long)i + 1) return;
        a.fy[w] = 0;
    }
    uint8_t *entry = entry_of(a, e);
    if (SV == 31 && fl == kIvApply) {  // 64-B entries: bytes 16..63 in and out as three 16-B words
        inv_apply64(a, i, w, entry, a.mem[i]);
        return;
    }
    Meta m;
    meta_load(entry, m);
    if (fl == kIvApply) {
        const unsigned long long X = a.mem[i];
        if (a.pf[i]) {
            b = (int64_t)a.fy[w] - 1;
            a.fy[w] = 0;
        }
        const uint8_t *xa = a.elems + i * a.esz;
        const uint64_t M = X >> 24;
        const uint8_t st = m_state(m);
        if (st == kValid) m_set_state(m, kInvalid);
        else if (st == kWrite || st == kReplay) m_set_state(m, kInvalidWrite);
        m_set_val_len(m, (uint8_t)a.g.kvs_value);
        m_set_rmw(m, e_rmw(xa));
        copy_value<SV>(entry + kEntryValueOff, xa + kOpValueOff, a.g.st_value);
        m.ver = (uint32_t)(M >> 8);
        m_set_cid(m, (uint8_t)M);
        a.fx[w] = 0;
    }
    m_set_lwid(m, a.elems[b * a.esz + 9]);
    meta_store(entry, m);
}

// ACK direct path: each matching element finds j*; j* (or, without a completion, F) applies the
// key's meta and completes the read_write_op slot. Nothing else reads the entry in this pass (the
// others use the cached S_0 fields), so the applier writes it here.
__global__ __launch_bounds__(256) void k_ack_resolve(BatchArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n || a.st[i] != kAkMatch) return;
    const uint32_t e = a.ent[i];
    const uint32_t w = fw_index(a, phys_of(a, e));
    const uint32_t c0 = a.pf[i];
    const uint8_t bv0 = (uint8_t)c0, st0 = (uint8_t)(c0 >> 8), obi0 = (uint8_t)(c0 >> 16);
    const U64x2 *tp = reinterpret_cast<const U64x2 *>(a.ft + (size_t)w * 8);
    uint32_t tv[8];  // 0xFFFFFFFF - (first match of the sender), 0: none in this launch
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const U64x2 p = tp[h];
        tv[2 * h] = (uint32_t)(p.a >> 32) == (a.rtag0 >> 3) ? (uint32_t)p.a : 0u;
        tv[2 * h + 1] = (uint32_t)(p.b >> 32) == (a.rtag0 >> 3) ? (uint32_t)p.b : 0u;
    }
    const uint8_t need = (uint8_t)(a.g_membership & ~bv0);
    // the first match of senders 0..7 (min T), and of any sender (with F; F is offered only by
    // matches from senders >= 8, or by every match when need is empty)
    uint32_t f = kNone;
#pragma unroll
    for (int s = 0; s < 8; ++s)
        if (tv[s] != 0) f = min(f, 0xFFFFFFFFu - tv[s]);
    uint32_t js = kNone;  // j*
    if (need == 0) {
        js = min(f, first_cand(a.fw[w], a.rtag0));  // F is read only here
    } else {
        uint32_t mx = 0;
        bool all = true;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (!((need >> s) & 1u)) continue;
            if (tv[s] == 0) all = false;
            else mx = max(mx, 0xFFFFFFFFu - tv[s]);
        }
        if (all) js = mx;
    }
    uint8_t *x = a.elems + i * a.esz;
    const bool done = (uint32_t)i == js;
    const bool wr = st0 == kWrite || st0 == kReplay;
    // j* overwrites the opcode (LAST_ACK_SUCCESS, or LAST_ACK_NO_BCAST -> ACK_SUCCESS), even a
    // LAST_ACK_SUCCESS input; the others keep a LAST_ACK_SUCCESS input
    x[8] = done ? (wr ? kLastAckSuccess : kAckSuccess) : ack_opcode(x[8]);
    if (!(done || (js == kNone && (uint32_t)i == f))) return;
    // the applier: ack_bv, and with a completion the state, op buffer index and read_write_op
    uint8_t bv = bv0;
#pragma unroll
    for (int s = 0; s < 8; ++s)
        if (tv[s] != 0 && (js == kNone || 0xFFFFFFFFu - tv[s] <= js)) bv |= (uint8_t)(1u << s);
    uint8_t *entry = entry_of(a, e);
    Meta m;
    meta_load(entry, m);
    m_set_ack_bv(m, bv);
    if (done) {
        if (st0 == kInvalidWrite) m_set_state(m, kInvalid);
        else if (wr) m_set_state(m, kValid);
        else if (st0 != kValid && st0 != kInvalid && a.error_flags) atomicOr(a.error_flags, 2u);
        m_set_obi(m, kObiEmpty);
        if (a.rw) {
            int64_t start;
            const int64_t b = batch_of(a, i, start);
            uint8_t *rw = a.rw + b * a.rw_stride + (size_t)obi0 * a.g.op_size;
            const uint8_t oc = rw[8];
            const uint8_t ns = oc == kOpGet ? kNew : oc == kOpPut ? kPutComplete : oc == kOpRmw ? kRmwComplete : rw[9];
            rw[9] = ns;
            if (a.rws) a.rws[b * (a.rw_stride / a.g.op_size) + obi0] = ns;
        }
    }
    meta_store(entry, m);
}

// ------------------------------------------------------------------ rounds (passes over all elements)
// Candidates of round r >= 1: pending elements against S_r, which round r-1's first candidate left
// in its shadow. Aggregated per key in LDS over kCandPer * 256 elements (see k_lookup).
constexpr int kCandPer = 4;
constexpr int kCandSlots = 2048;  // >= 2 * kCandPer * 256: the probe always ends
template <int TYPE>
__global__ __launch_bounds__(256) void k_cand(BatchArgs a, int r)
{
    __shared__ uint32_t lk[kCandSlots], lv[kCandSlots];
    for (int j = threadIdx.x; j < kCandSlots; j += 256) {
        lk[j] = kNone;
        lv[j] = kNone;
    }
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * 256 * kCandPer;
#pragma unroll
    for (int k = 0; k < kCandPer; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        if (i >= a.n) break;
        if (a.st[i] != kStPend) continue;
        Meta m;
        meta_load(shadow_of(a, a.pf[i]), m);
        uint64_t h2[2] = {0, ld64(a.elems + i * a.esz + 8)};
        Ctx c = make_ctx(a);
        if (!would_mutate(TYPE, reinterpret_cast<const uint8_t *>(h2), m, c)) continue;
        const uint32_t fi = fw_index(a, phys_of(a, a.ent[i]));
        uint32_t h = (fi * 0x9E3779B1u) >> 21;
        for (;;) {
            const uint32_t old = atomicCAS(&lk[h], kNone, fi);
            if (old == kNone || old == fi) {
                atomicMin(&lv[h], (uint32_t)i);
                break;
            }
            h = (h + 1) & (kCandSlots - 1);
        }
    }
    __syncthreads();
    const uint32_t rtag = a.rtag0 + (uint32_t)r;
    for (int j = threadIdx.x; j < kCandSlots; j += 256)
        if (lk[j] != kNone) offer(a.fw + lk[j], rtag, lv[j]);
}

// Round 0's resolve over every element, on LDS copies of the block's contiguous op slab (copied
// in and out with 16-B accesses, so the byte-wise result writes never reach memory one by one).
// Before F_0 (or no candidate) -> resolved now; F_0 -> applied to its shadow; after -> pending.
template <int TYPE, int SV, int BP>
__global__ __launch_bounds__(BP) void k_resolve0(BatchArgs a)
{
    extern __shared__ uint4 sops[];
    // 64-B entries: each thread reads bytes 16..63 (meta + value) in three 16-B accesses; the meta
    // comes from registers, the value from the thread's LDS copy
    constexpr bool kStage = SV == 31;
    __shared__ U64x2 sent[kStage ? 3 * BP : 1];
    const int64_t i0 = (int64_t)blockIdx.x * BP;
    const int cnt = a.n - i0 < BP ? (int)(a.n - i0) : BP;
    // the element's entry id and meta load while the block copies its op slab in
    const uint32_t e = (int)threadIdx.x < cnt ? a.ent[i0 + threadIdx.x] : kNone;
    Meta m{};
    if (e != kNone) {
        if (kStage) {
            const U64x2 *p = reinterpret_cast<const U64x2 *>(entry_of(a, e));
            const U64x2 l1 = p[1], l2 = p[2], l3 = p[3];
            m.w4 = (uint32_t)l1.a;
            m.w5 = (uint32_t)(l1.a >> 32);
            m.ver = (uint32_t)l1.b;
            m.llw_cid = (uint8_t)(l1.b >> 32);
            m.llw_ver = (uint32_t)(l1.b >> 40) | ((uint32_t)(l2.a & 0xFFu) << 24);
            sent[3 * threadIdx.x] = l1;
            sent[3 * threadIdx.x + 1] = l2;
            sent[3 * threadIdx.x + 2] = l3;
        } else {
            meta_load(entry_of(a, e), m);
        }
    }
    // what the non-mutating elements read the entry value from (bytes below 16 are never read)
    uint8_t *rentry = kStage ? reinterpret_cast<uint8_t *>(&sent[3 * threadIdx.x]) - 16 : entry_of(a, e);
    const uint32_t bytes = (uint32_t)cnt * (uint32_t)a.esz;  // a multiple of 8
    // big ops (312 B): only the elements that hit move through LDS (message slabs are mostly
    // padding); 8-B words, each inside one element
    constexpr bool kLive = BP == 128;
    __shared__ uint8_t live[kLive ? BP : 1];
    const uint32_t ew = (uint32_t)a.esz / 8u;
    if (kLive) {
        live[threadIdx.x] = e != kNone;
        __syncthreads();
        const uint64_t *src = reinterpret_cast<const uint64_t *>(a.elems + i0 * a.esz);
        uint64_t *s8 = reinterpret_cast<uint64_t *>(sops);
        for (uint32_t w = threadIdx.x; w < bytes / 8; w += BP)
            if (live[w / ew]) s8[w] = src[w];
    } else {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.elems + i0 * a.esz);
        for (uint32_t w = threadIdx.x; w < bytes / 16; w += BP) sops[w] = src[w];
        if ((bytes & 8) && threadIdx.x == 0)
            reinterpret_cast<uint64_t *>(sops)[bytes / 8 - 1] = reinterpret_cast<const uint64_t *>(src)[bytes / 8 - 1];
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < cnt) {
        const int64_t i = i0 + t;
        uint8_t st = kStDone;
        if (e != kNone) {
            // only keys flagged by k_lookup can have a first candidate
            const uint32_t f = (uint8_t)(m.w5 >> 16) == a.ltag ? first_cand(*fw_of(a, e), a.rtag0) : kNone;
            if (f == kNone || (uint32_t)i < f) {
                Ctx c = make_ctx(a);
                uint8_t *xg;
                uint8_t idx;
                elem_at(a, (uint32_t)i, xg, idx, c);
                Meta tm = m;
                dispatch<SV>(TYPE, reinterpret_cast<uint8_t *>(sops) + (uint32_t)t * a.esz, rentry, idx, tm, c);
                if (a.error_flags && !meta_equal(tm, m)) atomicOr(a.error_flags, 1u);
            } else if ((uint32_t)i == f) {
                apply_to_shadow<TYPE, SV>(a, reinterpret_cast<uint8_t *>(sops) + (uint32_t)t * a.esz, (uint32_t)i,
                                          entry_of(a, e));
                st = kStCommit;
            } else if (a.rounds == 0) {  // after the key's only mutation: absorbing state
                Ctx c = make_ctx(a);
                uint8_t *xg;
                uint8_t idx;
                elem_at(a, (uint32_t)i, xg, idx, c);
                const Meta m1 = after_first<TYPE>(a, m, f, 0);
                Meta tm = m1;
                dispatch<SV>(TYPE, reinterpret_cast<uint8_t *>(sops) + (uint32_t)t * a.esz, rentry, idx, tm, c);
                if (a.error_flags && !meta_equal(tm, m1)) atomicOr(a.error_flags, 1u);
            } else {
                a.pf[i] = f;
                st = kStPend;
            }
        }
        a.st[i] = st;
        // big ops move through LDS only when they hit (kLive); the others are in memory unchanged
        note_state(a, i, kLive && e == kNone ? a.elems + i * a.esz
                                              : reinterpret_cast<const uint8_t *>(sops) + (uint32_t)t * a.esz);
    }
    __syncthreads();
    if (kLive) {
        uint64_t *dst = reinterpret_cast<uint64_t *>(a.elems + i0 * a.esz);
        const uint64_t *s8 = reinterpret_cast<const uint64_t *>(sops);
        for (uint32_t w = threadIdx.x; w < bytes / 8; w += BP)
            if (live[w / ew]) dst[w] = s8[w];
        return;
    }
    uint4 *dst = reinterpret_cast<uint4 *>(a.elems + i0 * a.esz);
    for (uint32_t w = threadIdx.x; w < bytes / 16; w += BP) dst[w] = sops[w];
    if ((bytes & 8) && threadIdx.x == 0)
        reinterpret_cast<uint64_t *>(dst)[bytes / 8 - 1] = reinterpret_cast<const uint64_t *>(sops)[bytes / 8 - 1];
}

// k_resolve0 for big ops (312 B) in place: one thread per element on its global copy, no LDS, so
// occupancy is bound by registers instead of by 312 B of LDS per element (local and ACK launches)
// The value copies the wave's exec calls recorded (Ctx::vc), made by the whole wave: byte k of a
// value by lane k % 64, so each instruction moves 64 consecutive bytes. kVcBatch values at a time:
// all their loads are issued before the first store, so a wave waits one memory latency per
// kVcBatch values instead of one per value. Every lane of the wave
// calls it.
#ifndef HKV_VC_BATCH_N
#define HKV_VC_BATCH_N 4
#endif
constexpr int kVcBatch = HKV_VC_BATCH_N;
template <int VB>
__device__ __forceinline__ void wave_value_copies_n(const VCopy &v, uint32_t n)
{
    const int lane = threadIdx.x & 63;
    unsigned long long todo = __ballot(v.dst != nullptr);
    while (todo) {
        uint8_t *dp[VB];
        const uint8_t *sp[VB];
#pragma unroll
        for (int u = 0; u < VB; ++u) {   // the next VB recorded copies (todo is the same in every lane)
            dp[u] = nullptr;
            sp[u] = nullptr;
            if (todo) {
                const int j = __ffsll((long long)todo) - 1;
                todo &= todo - 1;
                const uint64_t d = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)v.dst, j, 64) |
                                   ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)v.dst >> 32), j, 64) << 32);
                const uint64_t s = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)v.src, j, 64) |
                                   ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)v.src >> 32), j, 64) << 32);
                dp[u] = reinterpret_cast<uint8_t *>(d);
                sp[u] = reinterpret_cast<const uint8_t *>(s);
            }
        }
        uint8_t b[VB][5];
#pragma unroll
        for (int u = 0; u < VB; ++u)
#pragma unroll
            for (int r = 0; r < 5; ++r) {   // values up to 320 B; all loads before the stores
                const uint32_t k = (uint32_t)lane + 64u * r;
                b[u][r] = sp[u] && k < n ? sp[u][k] : 0;
            }
#pragma unroll
        for (int u = 0; u < VB; ++u)
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                const uint32_t k = (uint32_t)lane + 64u * r;
                if (dp[u] && k < n) dp[u][k] = b[u][r];
            }
    }
}

// bytes [lo, hi) of the 8-byte word v to the 8-byte aligned p, in aligned 1/2/4-byte stores (the
// word's other bytes are other fields: op header, entry meta)
__device__ __forceinline__ void store_word_part(uint8_t *p, uint64_t v, uint32_t lo, uint32_t hi)
{
    for (uint32_t b = lo; b < hi;) {
        if ((b & 3) == 0 && b + 4 <= hi) {
            *reinterpret_cast<uint32_t *>(p + b) = (uint32_t)(v >> (8 * b));
            b += 4;
        } else if ((b & 1) == 0 && b + 2 <= hi) {
            *reinterpret_cast<uint16_t *>(p + b) = (uint16_t)(v >> (8 * b));
            b += 2;
        } else {
            p[b] = (uint8_t)(v >> (8 * b));
            b += 1;
        }
    }
}

// wave_value_copies_n by 8-byte words: lane k stores the destination's aligned word k (the two end
// words byte-exact), built from the aligned source words k and k + 1 (the latter from lane k + 1), so
// a 287-byte value is 37 lanes of one load and one store instead of five byte instructions each way
// (the op value sits at byte 18 and the entry value at byte 33, so the two ends differ mod 8). Only
// source words holding a byte of the value are loaded.
template <int VB>
__device__ __forceinline__ void wave_value_words_n(const VCopy &v, uint32_t n)
{
    const uint32_t lane = threadIdx.x & 63;
    unsigned long long todo = __ballot(v.dst != nullptr);
    while (todo) {
        uint8_t *dp[VB];
        const uint8_t *sp[VB];
        uint32_t fl[VB];
#pragma unroll
        for (int u = 0; u < VB; ++u) {
            dp[u] = nullptr;
            sp[u] = nullptr;
            fl[u] = 0;
            if (todo) {
                const int j = __ffsll((long long)todo) - 1;
                todo &= todo - 1;
                const uint64_t d = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)v.dst, j, 64) |
                                   ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)v.dst >> 32), j, 64) << 32);
                const uint64_t s = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)v.src, j, 64) |
                                   ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)v.src >> 32), j, 64) << 32);
                dp[u] = reinterpret_cast<uint8_t *>(d);
                sp[u] = reinterpret_cast<const uint8_t *>(s);
                fl[u] = (uint32_t)__shfl((int)v.fill, j, 64);
            }
        }
        uint64_t w[VB];
#pragma unroll
        for (int u = 0; u < VB; ++u) {   // all loads before the stores
            // destination word k takes the source bytes from base + 8k; aligned source word j is at ab + 8j
            const uintptr_t s = (uintptr_t)sp[u], d0 = (uintptr_t)dp[u] & 7u;
            const uintptr_t ab = (s - d0) & ~(uintptr_t)7;
            const uintptr_t wa = ab + 8u * lane;
            w[u] = 0;
            if (fl[u]) w[u] = 0x0101010101010101ull * (uint8_t)fl[u];   // every word (any shift of it is itself)
            else if (sp[u] && wa + 8 > s && wa < s + n) w[u] = *reinterpret_cast<const uint64_t *>(wa);
        }
#pragma unroll
        for (int u = 0; u < VB; ++u) {
            const uint64_t hi_w = (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)w[u], 1, 64) |
                                  ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(w[u] >> 32), 1, 64) << 32);
            if (!dp[u]) continue;
            const uint32_t d0 = (uint32_t)((uintptr_t)dp[u] & 7u);
            const uint32_t r = (uint32_t)(((uintptr_t)sp[u] - d0) & 7u);
            const uint32_t nw = (d0 + n + 7u) >> 3;
            if (lane >= nw) continue;
            const uint64_t val = r ? (w[u] >> (8 * r)) | (hi_w << (64 - 8 * r)) : w[u];
            uint8_t *dw = dp[u] - d0 + 8u * lane;
            const uint32_t lo = lane == 0 ? d0 : 0u;
            const uint32_t hi = lane == nw - 1 ? d0 + n - 8u * (nw - 1) : 8u;
            if (lo == 0 && hi == 8) *reinterpret_cast<uint64_t *>(dw) = val;
            else store_word_part(dw, val, lo, hi);
        }
    }
}

#ifndef HKV_FULL_HDR
#define HKV_FULL_HDR 1
#endif
#ifndef HKV_VC_WORDS
#define HKV_VC_WORDS 1
#endif
__device__ __forceinline__ void wave_value_copies(const VCopy &v, uint32_t n, int batch)
{
    if (HKV_VC_WORDS && n <= 8 * 62) {   // nw + 1 <= 64 source words
        if (batch == 1) wave_value_words_n<1>(v, n);
        else wave_value_words_n<kVcBatch>(v, n);
        return;
    }
    if (batch == 1) wave_value_copies_n<1>(v, n);
    else wave_value_copies_n<kVcBatch>(v, n);
}

// Whole-wave copies of `bytes` (a multiple of 8, 8-byte aligned ends) recorded one per lane (dst
// null: none): C = bytes / 16 rounded up lanes per copy move 16 B each, 64 / C copies per
// instruction, and kBcRounds instructions' loads are issued before their stores. Every lane of the
// wave calls it.
constexpr int kBcRounds = 2;
__device__ __forceinline__ void wave_block_copies(uint8_t *dst, const uint8_t *src, uint32_t bytes)
{
    struct __attribute__((aligned(8))) W16 {
        uint64_t a, b;
    };
    const int lane = threadIdx.x & 63;
    const int C = (int)((bytes + 15) / 16);
    const int per = 64 / C;
    const int slot = lane / C, ch = lane - slot * C;
    unsigned long long todo = __ballot(dst != nullptr);
    while (todo) {
        W16 v[kBcRounds];
        uint8_t *dp[kBcRounds];
        bool half[kBcRounds];
#pragma unroll
        for (int r = 0; r < kBcRounds; ++r) {
            int mine = -1;
            for (int k = 0; k < per; ++k) {   // this instruction's copies, lane order (todo is uniform)
                if (!todo) break;
                const int j = __ffsll((long long)todo) - 1;
                todo &= todo - 1;
                if (k == slot) mine = j;
            }
            const int sl = mine < 0 ? 0 : mine;
            const uint64_t d = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)dst, sl, 64) |
                               ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)dst >> 32), sl, 64) << 32);
            const uint64_t sa = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(uintptr_t)src, sl, 64) |
                                ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)src >> 32), sl, 64) << 32);
            dp[r] = mine >= 0 && slot < per ? reinterpret_cast<uint8_t *>(d) + 16 * ch : nullptr;
            half[r] = 16 * ch + 16 > (int)bytes;
            const uint8_t *sp = reinterpret_cast<const uint8_t *>(sa) + 16 * ch;
            v[r] = W16{0, 0};
            if (dp[r]) {
                if (half[r]) v[r].a = *reinterpret_cast<const uint64_t *>(sp);
                else v[r] = *reinterpret_cast<const W16 *>(sp);
            }
        }
#pragma unroll
        for (int r = 0; r < kBcRounds; ++r) {
            if (!dp[r]) continue;
            if (half[r]) *reinterpret_cast<uint64_t *>(dp[r]) = v[r].a;
            else *reinterpret_cast<W16 *>(dp[r]) = v[r];
        }
    }
}

// patch_in_resolve (big local launches with refill patches, a.hx set; launch_batch): k_lookup read each
// patch beside the op's header, so a patched element runs its exec function on a copy of its op's first 24
// bytes in LDS -- key and header word as patched (k_lookup), flags from the patch -- and this pass writes the
// op once: its header from the copy, a write's value fill (a copy with no source to load), the GET values
// the exec functions copy, and the pad bytes after the value from the op's last word (k_lookup), so the op's
// 64-byte blocks are written whole (a block written with holes costs HBM a read-modify-write:
// tools/write_bench.hip). The refill's own pass over the slab (k_refill_st_w) goes, and this pass reads
// no op line: the header came with k_lookup's read, a write's value is the patch's fill byte.
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, src, 64) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64) << 32);
}
// Ops whose every byte is known (k_resolve0_direct's whole ones: key h0, header h1, flags and fill byte fl, the
// fill, the last word lw; nw 8-byte words) written by the whole wave: (nw + 1) / 2 lanes per op, 16 B each, so
// one store instruction writes 64 / that many ops contiguously. Every lane calls it.
__device__ __forceinline__ void wave_whole_ops(uint8_t *xg, bool whole, uint64_t h0, uint64_t h1, uint32_t fl, uint64_t lw,
                                               uint32_t nw)
{
    const int lane = threadIdx.x & 63;
    const int C = (int)((nw + 1) / 2);
    const int per = 64 / C;
    const int slot = lane / C, ch = lane - slot * C;
    unsigned long long todo = __ballot(whole);
    while (todo) {
        int mine = -1;
        for (int k = 0; k < per; ++k) {   // (todo is the same in every lane)
            if (!todo) break;
            const int j = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            if (k == slot) mine = j;
        }
        const int sl = mine < 0 ? 0 : mine;
        const uint64_t d = shfl_u64((uint64_t)(uintptr_t)xg, sl), a0 = shfl_u64(h0, sl), a1 = shfl_u64(h1, sl);
        const uint64_t l = shfl_u64(lw, sl);
        const uint32_t f = (uint32_t)__shfl((int)fl, sl, 64);
        if (mine < 0 || slot >= per) continue;
        const uint64_t pat = 0x0101010101010101ull * ((f >> 16) & 0xFFu);
        auto word = [&](uint32_t k) {
            return k == 0 ? a0 : k == 1 ? a1 : k == 2 ? ((uint64_t)(f & 0xFFFFu) | (pat << 16)) : k == nw - 1 ? l : pat;
        };
        const uint32_t k0 = 2u * (uint32_t)ch;
        uint8_t *p = reinterpret_cast<uint8_t *>(d) + 8u * k0;
        if (k0 + 1 < nw) *reinterpret_cast<U64x2 *>(p) = U64x2{word(k0), word(k0 + 1)};
        else *reinterpret_cast<uint64_t *>(p) = word(k0);
    }
}

// waves per SIMD k_resolve0_direct is compiled for (its registers: 512 / waves). At 8 it fits 64 VGPRs
// instead of 127 (4 waves per SIMD): configs[2] fresh 0.736-0.741 -> 0.772-0.782 G ops/s (gpurun_out/r06s;
// in round 5's kernel, before the patches, it was level)
#ifndef HKV_R0D_WAVES
#define HKV_R0D_WAVES 8
#endif
#define HKV_R0D_ATTR __attribute__((amdgpu_waves_per_eu(HKV_R0D_WAVES, 8)))
template <int TYPE, int SV>
__global__ __launch_bounds__(256) HKV_R0D_ATTR void k_resolve0_direct(BatchArgs a)
{
    constexpr bool kPir = TYPE == kLocal && SV != 31;
    __shared__ uint64_t sop[kPir ? 256 * 3 : 1];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool in = i < a.n;
    const uint32_t e = in ? a.ent[i] : kNone;
    U64x2 pt{0, 0}, hw{0, 0};
    if (kPir && a.hx && in) {   // beside the entry id: one trip
        pt = *reinterpret_cast<const U64x2 *>(a.patch + i * 16);
        hw = *reinterpret_cast<const U64x2 *>(a.hx + 2 * i);
    }
    const bool pd = kPir && a.hx && in && patch_valid(pt.b);
    const uint32_t fb = (uint32_t)(pt.b >> 32) & 0xFFu;   // a patched element's value fill byte (0: none)
    uint64_t *cop = &sop[kPir ? threadIdx.x * 3 : 0];
    if (pd) {
        cop[0] = pt.a;
        cop[1] = hw.a;
        cop[2] = ((pt.b >> 16) & 0xFFFFull) | (fb ? (0x0101010101010101ull * fb) << 16 : 0ull);
    }
    uint8_t st = kStDone;
    uint8_t *xg = nullptr;
    uint8_t idx = 0;
    Ctx c = make_ctx(a);
    // big values: the exec calls record their value copy, made by the whole wave afterwards (the
    // key's entry is not written in this pass -- its first candidate writes its own shadow -- and
    // the op is this lane's own)
    VCopy vc{nullptr, nullptr};
    if (SV != 31 && a.g.st_value <= 320) c.vc = &vc;
    // a key's first candidate applies itself to its shadow by the whole wave (apply_to_shadow_wave)
    const bool wave_shadow = SV != 31 && a.g.st_value <= 320;
    bool cand = false;
    if (in) elem_at(a, (uint32_t)i, xg, idx, c);
    // the op the exec functions see: the LDS copy of a patched one, else the op (two calls, so each keeps
    // its address space instead of flat accesses)
    uint8_t *xl = reinterpret_cast<uint8_t *>(cop);
    if (e != kNone) {
        Meta m;
        meta_load(entry_of(a, e), m);
        const uint32_t f = (uint8_t)(m.w5 >> 16) == a.ltag ? first_cand(*fw_of(a, e), a.rtag0) : kNone;
        // elements after F: resolved here when F's mutation is absorbing (no RMWs: always; with RMWs: F's kind)
        uint16_t fkf = 0;
        if (TYPE == kLocal && a.fk && f != kNone && (uint32_t)i > f) fkf = a.fk[f];
        const bool after_abs = (uint32_t)i > f && f != kNone && (a.rounds == 0 || (fkf & 3u) == kFkWrite ||
                                                                  (fkf & 3u) == kFkReplay);
        if (f == kNone || (uint32_t)i < f || after_abs) {
            Meta m0 = m;
            if (after_abs) {
                if (a.rounds == 0) {
                    m0 = after_first<TYPE>(a, m, f, 0);
                } else {
                    int64_t fs;
                    batch_of(a, f, fs);
                    m0 = after_first_rmw(a, m, fkf, (uint8_t)(f - fs));
                }
            }
            Meta tm = m0;
            if (pd) dispatch<SV>(TYPE, xl, entry_of(a, e), idx, tm, c);
            else dispatch<SV>(TYPE, xg, entry_of(a, e), idx, tm, c);
            if (a.error_flags && !meta_equal(tm, m0)) atomicOr(a.error_flags, 1u);
        } else if ((uint32_t)i == f) {
            if (wave_shadow) cand = true;
            else apply_to_shadow<TYPE, SV>(a, nullptr, (uint32_t)i, entry_of(a, e));
            st = kStCommit;
        } else {
            a.pf[i] = f;
            st = kStPend;
        }
    }
    if (wave_shadow) apply_to_shadow_wave<TYPE, SV>(a, cand, (uint32_t)i, cand ? entry_of(a, e) : nullptr, vc, xl, pd);
    bool whole = false;   // a patched op whose every byte is known here: written whole by its lane
    if (pd) {
        uint8_t *cv = reinterpret_cast<uint8_t *>(cop) + kOpValueOff;
        if (vc.dst == cv) vc.dst = xg + kOpValueOff;
        if (vc.src == cv) {
            vc.src = fb ? nullptr : xg + kOpValueOff;
            vc.fill = fb ? 0x100u | fb : 0u;
        }
        whole = fb && vc.dst != xg + kOpValueOff;   // (a value the exec copies into the op replaces the fill)
    }
    if (SV != 31) wave_value_copies(vc, a.g.st_value, kVcBatch);
    if (kPir && a.hx) {
        // a whole op: key, header, flags, the value fill and the pad after it (launch_batch: at most 8 bytes,
        // in the op's last word), written by the wave, three ops a store instruction, so every 64-byte block
        // of the op is complete in L2 before it goes to HBM (whole ops stored by their own lane, 16 bytes
        // at a time: 4 % slower at configs[2])
        const uint32_t vend = kOpValueOff + a.g.st_value, w0 = (uint32_t)a.esz - 8u;
        const uint64_t pat = 0x0101010101010101ull * fb;
        const uint32_t nlow = vend - w0;
        const uint64_t lmask = nlow >= 8 ? ~0ull : (1ull << (8 * nlow)) - 1ull;
        wave_whole_ops(xg, whole, cop[0], cop[1], ((uint32_t)cop[2] & 0xFFFFu) | (fb << 16),
                       (pat & lmask) | (hw.b & ~lmask), (uint32_t)a.esz / 8u);
    }
    if (!in) return;
    a.st[i] = st;
    if (pd) {
        const uint64_t h0 = cop[0], h1 = cop[1], h2 = cop[2];
        const uint32_t vend = kOpValueOff + a.g.st_value, w0 = (uint32_t)a.esz - 8u;
        if (!whole) {   // the header from the copy, then the pad bytes after the value
            uint64_t *o = reinterpret_cast<uint64_t *>(xg);
            o[0] = h0;
            o[1] = h1;
            *reinterpret_cast<uint16_t *>(xg + 16) = (uint16_t)h2;
            if (vend < (uint32_t)a.esz) store_word_part(xg + w0, hw.b, vend - w0, 8u);
        }
        if (a.state_out) a.state_out[i] = (uint8_t)(h1 >> 8);
        return;
    }
    note_state(a, i, xg);
#if HKV_FULL_HDR
    // the op's first three and last 8-byte words stored again as they now stand, so that with the value a
    // GET copied the slab's lines are written whole (a line written with holes costs HBM a read-modify-write:
    // tools/write_bench.hip, 4M 312-byte ops with an 8-byte hole each 495 us against 241 us whole)
    if (SV != 31 && (a.esz & 7) == 0 && a.esz >= 32) {
        __threadfence_block();   // the wave's value copies before the loads
        uint64_t *o = reinterpret_cast<uint64_t *>(xg);
        const uint64_t h0 = o[0], h1 = o[1], h2 = o[2], t = o[a.esz / 8 - 1];
        o[0] = h0;
        o[1] = h1;
        o[2] = h2;
        o[a.esz / 8 - 1] = t;
    }
#endif
}

// ------------------------------------------------------------------ local launches: direct path
// Local batches without RMWs, 56-B ops and 64-B entries (configs[1]). Under these, an element's
// key can only be mutated by a PUT (hermes_exec_write) from VALID/INVALID, or by a GET replay
// from INVALID (hermes_exec_read -> write replay), and its first mutation leaves the key in an
// absorbing state (WRITE/REPLAY, see absorbing_state). So every element's result is fixed by S_0
// and by F, its key's first mutating element:
//   i < F (or no F): the exec function against S_0;  i = F: S_0 -> its shadow;  i > F: against WRITE.
// Three passes instead of lookup + re-reading every op and entry line:
//   k_local_pre    the PUTs only (one op header per element, then bucket + log line per PUT):
//                  every PUT that mutates S_0 offers F and tags its entry's seqlock byte;
//   k_local_fused  every element: op slab through LDS, bucket, log line (the whole 64-B entry, four
//                  lanes) -- F is final for every key not INVALID at S_0, so each element resolves
//                  right there, F applies itself to its shadow, and the slab is written back once;
//                  elements of INVALID keys (where GET replays may mutate: they offer F here) wait;
//   k_local_deferred  those waiting elements, against the final F.
// k_commit then installs the shadows. Measured against k_lookup + k_resolve0: the entry line and
// the op slab are read once instead of twice.
// work-skipping timing modes of k_local_pre (tools/dbg_modes.sh): compiled in only with
// -DHKV_DEBUG_MODES; the default build folds every test to false
#ifdef HKV_DEBUG_MODES
#define HKV_DBG_ON(a, bit) (((a).dbg & (bit)) != 0)
#else
#define HKV_DBG_ON(a, bit) false
#endif
// Round 5: 2048 elements per block (512 threads), a 2048-slot table: each block looks up and offers
// each of its PUT keys once, so doubling the block removes the second lookup of the keys two 1024-element
// halves shared, and the two head elements per thread instead of four cut registers. Same box, 3 x 20
// steps (gpurun_out/r05v): prepass 76.1 -> 64.2 us, 4.25-4.29 -> 4.27-4.36 G ops/s; 1536 (86 us), 4096 (78 us),
// a 2048-element head (79 us) and a 4096-slot table (111 us) were slower
#ifndef HKV_PRE_ELEMS
#define HKV_PRE_ELEMS 2048
#endif
constexpr int kPreElems = HKV_PRE_ELEMS;   // elements per k_local_pre block (HKV_PRE_ELEMS: a build macro for A/B)
constexpr int kPreThreads = kPreElems / 4; // four of its own elements per thread
#ifndef HKV_PRE_HEAD_ELEMS
#define HKV_PRE_HEAD_ELEMS 1024
#endif
constexpr int kPreHead = HKV_PRE_HEAD_ELEMS;   // launch head whose PUT keys every block knows
#ifndef HKV_PRE_HASH_SLOTS
#define HKV_PRE_HASH_SLOTS 2048
#endif
constexpr int kPreHash = HKV_PRE_HASH_SLOTS;   // LDS slots of a (key -> first PUT) table (a power of two)
constexpr int kLfElems = 32;             // elements per k_local_fused block (one wave)
enum { kCtrDefer = 3 };
enum : uint8_t { kStDefer = 3 };

// The key (bytes 8..15) and the meta (bytes 16..32) of a log line held 16 B per lane, in every lane
__device__ __forceinline__ uint64_t line_key_meta(const uint4 &ln, Meta &m)
{
    const uint64_t ek = (uint64_t)(uint32_t)__shfl((int)ln.z, 0, 4) | ((uint64_t)(uint32_t)__shfl((int)ln.w, 0, 4) << 32);
    m.w4 = (uint32_t)__shfl((int)ln.x, 1, 4);
    m.w5 = (uint32_t)__shfl((int)ln.y, 1, 4);
    m.ver = (uint32_t)__shfl((int)ln.z, 1, 4);
    const uint32_t w7 = (uint32_t)__shfl((int)ln.w, 1, 4);
    const uint32_t b32 = (uint32_t)__shfl((int)ln.x, 2, 4) & 0xFFu;
    m.llw_cid = (uint8_t)w7;
    m.llw_ver = (w7 >> 8) | (b32 << 24);
    return ek;
}

// element i lies inside its batch's count (launches are under 2^31 elements: 32-bit division,
// and none at all without counts)
__device__ __forceinline__ bool in_count(const BatchArgs &a, uint32_t i)
{
    if (!a.counts) return true;
    const uint32_t b = i / (uint32_t)a.stride;
    return (int32_t)(i - b * (uint32_t)a.stride) < a.counts[b];
}

// ---- pending header writes (hkv_batch_desc.d_patch, HKV_PATCH_BYTES per element): the second
// 8-B word of a patch holds opcode (bits 0..7), val_len (8..15), flags (16..31), the value fill
// byte (32..39), ts reset (40..47) and valid (48..55).
__device__ __forceinline__ bool patch_valid(uint64_t pb) { return ((pb >> 48) & 0xFFu) != 0; }

// the key of element i as the launch sees it (patched or not)
__device__ __forceinline__ uint64_t elem_key(const BatchArgs &a, int64_t i)
{
    if (a.patch && a.patch[i * 16 + 14]) return *reinterpret_cast<const uint64_t *>(a.patch + i * 16);
    return *reinterpret_cast<const uint64_t *>(a.elems + i * a.esz);
}

// a patch applied to the 16-B chunk q (bytes 16q..16q+15) of a 56-B op with a 31-B value
__device__ __forceinline__ uint4 patch_chunk(uint4 w, int q, uint64_t pa, uint64_t pb)
{
    const uint32_t fill = (uint32_t)((pb >> 32) & 0xFFu) * 0x01010101u;
    const bool vfill = fill != 0, reset = ((pb >> 40) & 0xFFu) != 0;
    if (q == 0) {
        w.x = (uint32_t)pa;
        w.y = (uint32_t)(pa >> 32);
        // opcode, ST_NEW, val_len; ts.cid (byte 11) and ts.version (12..15) kept unless reset
        w.z = (uint32_t)(pb & 0xFFu) | ((uint32_t)kNew << 8) | ((uint32_t)((pb >> 8) & 0xFFu) << 16) |
              (reset ? 0u : (w.z & 0xFF000000u));
        if (reset) w.w = 0;
    } else if (q == 1) {
        const uint32_t flags = (uint32_t)((pb >> 16) & 0xFFFFu);
        w.x = flags | (vfill ? (fill & 0xFFFF0000u) : (w.x & 0xFFFF0000u));
        if (vfill) w.y = w.z = w.w = fill;
    } else if (q == 2) {
        if (vfill) w.x = w.y = w.z = w.w = fill;
    } else if (vfill) {  // bytes 48..55: byte 48 is the value's last
        w.x = (w.x & 0xFFFFFF00u) | (fill & 0xFFu);
    }
    return w;
}

// Every other path: the patches go into the ops first (one thread per element), then the launch
// runs as usual
__global__ __launch_bounds__(256) void k_apply_patch(uint8_t *elems, const uint8_t *patch, int64_t n, int32_t esz,
                                                     uint32_t st_value)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const U64x2 p = *reinterpret_cast<const U64x2 *>(patch + i * 16);
    if (!patch_valid(p.b)) return;
    uint8_t *x = elems + i * esz;
    *reinterpret_cast<uint64_t *>(x) = p.a;
    x[8] = (uint8_t)p.b;
    x[9] = kNew;
    x[10] = (uint8_t)(p.b >> 8);
    if ((p.b >> 40) & 0xFFu) {
        x[11] = 0;
        *reinterpret_cast<uint32_t *>(x + 12) = 0;
    }
    *reinterpret_cast<uint16_t *>(x + 16) = (uint16_t)(p.b >> 16);
    const uint8_t fill = (uint8_t)(p.b >> 32);
    if (fill)
        for (uint32_t k = 0; k < st_value; ++k) x[kOpValueOff + k] = fill;
}

__device__ __forceinline__ uint32_t pre_slot(uint64_t key)
{
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - __builtin_ctz(kPreHash))) & (kPreHash - 1);
}

// (key -> smallest element) in an LDS table of kPreHash slots, key ~0 the empty mark; false when the
// key cannot go in (key ~0 itself, or a full table)
__device__ __forceinline__ bool pre_insert(uint64_t *hk, uint32_t *hv, uint64_t key, uint32_t i, bool &created,
                                           uint32_t &slot)
{
    created = false;
    if (key == ~0ull) return false;
    uint32_t sl = pre_slot(key);
    for (int n = 0; n < kPreHash; ++n) {
        const unsigned long long old = atomicCAS((unsigned long long *)&hk[sl], ~0ull, key);
        if (old == ~0ull || old == key) {
            created = old == ~0ull;
            atomicMin(&hv[sl], i);
            slot = sl;
            return true;
        }
        sl = (sl + 1) & (kPreHash - 1);
    }
    return false;
}

// a key into an LDS set of kPreHash slots (the head's PUT keys: only membership is asked)
__device__ __forceinline__ void pre_insert_key(uint64_t *hk, uint64_t key)
{
    if (key == ~0ull) return;
    uint32_t sl = pre_slot(key);
    for (int n = 0; n < kPreHash; ++n) {
        const unsigned long long old = atomicCAS((unsigned long long *)&hk[sl], ~0ull, key);
        if (old == ~0ull || old == key) return;
        sl = (sl + 1) & (kPreHash - 1);
    }
}

// The PUTs of kPreElems elements offer F. Whether a PUT mutates S_0 depends on S_0 alone
// (hermes_exec_write: VALID or INVALID and no op buffer index), so either every PUT of a key is a
// candidate or none is, and F is the key's first PUT or nothing. So each block looks up each key
// once, for its first PUT (an LDS table of the block's PUT keys). A Zipf-hot key's PUTs are spread
// over every block, and all blocks of the launch are in flight together: every block also reads the
// keys of the PUTs among the launch's first kPreHead elements (before its own; headers only,
// L2-resident after the first block) and drops its keys that have a PUT there -- an earlier block
// offers that one. Four keys per lane group are in flight; the offer is a plain atomicMin.
#ifndef HKV_PRE_PAIR
#define HKV_PRE_PAIR 4
#endif
constexpr int kPrePair = HKV_PRE_PAIR;   // keys per lane group in flight in the prepass's lookups (a build macro for A/B)
#ifdef HKV_PRE_WAVES
#define HKV_PRE_ATTR __attribute__((amdgpu_waves_per_eu(HKV_PRE_WAVES)))
#else
#define HKV_PRE_ATTR
#endif
// No seqlock-byte tags (round 5): k_local_fused loads every hit's F word beside its log line and needs
// no mark of the keys that have one
#ifdef HKV_PRE_NUM_SGPR
#define HKV_PRE_SGPR_ATTR __attribute__((amdgpu_num_sgpr(HKV_PRE_NUM_SGPR)))
#else
#define HKV_PRE_SGPR_ATTR
#endif
template <int HEAD = kPreHead>
__global__ __launch_bounds__(kPreThreads) HKV_PRE_ATTR HKV_PRE_SGPR_ATTR void k_local_pre(BatchArgs a)
{
    __shared__ uint64_t hk[kPreHash], gk[kPreHash];  // the block's PUT keys, the head's
    __shared__ uint32_t hv[kPreHash];
    __shared__ uint32_t dl[kPreElems];               // distinct keys: slots of hk, or ~index (no slot)
    __shared__ uint32_t nd;
    const int tid = threadIdx.x, q = tid & 3, gbase = (tid & 63) & ~3;
    if (tid == 0) {
        nd = 0;
        if (blockIdx.x == 0) a.ctr[kCtrDefer] = 0;
    }
    for (int j = tid; j < kPreHash; j += kPreThreads) {
        hk[j] = ~0ull;
        gk[j] = ~0ull;
        hv[j] = kNone;
    }
    if (HKV_DBG_ON(a, 8)) return;
    const int64_t i0 = (int64_t)blockIdx.x * kPreElems;
    const int64_t head_end = HKV_DBG_ON(a, 4) ? 0 : i0 < HEAD ? i0 : HEAD;  // the head: elements before the block's own
    // PUTs that are not skipped (hermes_skip_op, hermesKV.c:709-769). Reading every op header is a
    // pass over the whole op slab; with the caller's opcode mirror only the PUTs' headers are read
    // (the others read element 0's, one cached line; k_local_fused checks the mirror against every
    // element's opcode). Loads are unconditional and all issued before the first is used.
    constexpr int kOwnK = kPreElems / kPreThreads, kAllK = kOwnK + (HEAD + kPreThreads - 1) / kPreThreads;
    U64x2 h[kAllK];
    bool in[kAllK];
    uint8_t opm[kAllK];
    U64x2 pt[kAllK];
#pragma unroll
    for (int k = 0; k < kAllK; ++k) {
        const bool own = k < kOwnK;
        const int64_t i = own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid;
        in[k] = i < a.n && (own || i < head_end);
        opm[k] = a.opc ? a.opc[in[k] ? i : 0] : (uint8_t)kOpPut;
    }
    if (a.patch) {
        // the patches first: a refilled PUT's patch holds all the prepass needs (key, opcode, ST_NEW),
        // so only the PUTs kept from the last round read their op header (a second dependent load
        // for them, against a third of the op slab's lines fetched for nothing)
#pragma unroll
        for (int k = 0; k < kAllK; ++k) {
            const bool own = k < kOwnK;
            const int64_t i = own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid;
            pt[k] = in[k] && opm[k] == kOpPut ? *reinterpret_cast<const U64x2 *>(a.patch + i * 16) : U64x2{0, 0};
        }
#pragma unroll
        for (int k = 0; k < kAllK; ++k) {
            const bool own = k < kOwnK;
            const int64_t i = own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid;
            h[k] = *reinterpret_cast<const U64x2 *>(a.elems + (in[k] && opm[k] == kOpPut && !patch_valid(pt[k].b) ? i : 0) * 56);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kAllK; ++k) {
            const bool own = k < kOwnK;
            const int64_t i = own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid;
            h[k] = *reinterpret_cast<const U64x2 *>(a.elems + (in[k] && opm[k] == kOpPut ? i : 0) * 56);
            pt[k] = U64x2{0, 0};
        }
    }
#pragma unroll
    for (int k = 0; k < kAllK; ++k)
        if (patch_valid(pt[k].b)) {   // a patched element: its key and opcode, state ST_NEW
            h[k].a = pt[k].a;
            h[k].b = (h[k].b & ~0xFFFFull) | (pt[k].b & 0xFFu) | ((uint64_t)kNew << 8);
        }
#pragma unroll
    for (int k = 0; k < kAllK; ++k) {
        const bool own = k < kOwnK;
        const int64_t i = own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid;
        // a non-PUT read element 0's raw header, which a patch may have made stale: only the
        // mirror's PUTs take part
        in[k] = in[k] && opm[k] == kOpPut && in_count(a, (uint32_t)i);
    }
    if (HKV_DBG_ON(a, 16)) {
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < kAllK; ++k) acc += h[k].a ^ h[k].b;
        if (acc == 0x1234567ull) a.ctr[7] = 1;
        return;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kAllK; ++k) {
        const bool own = k < kOwnK;
        const uint32_t i = (uint32_t)(own ? i0 + k * kPreThreads + tid : (int64_t)(k - kOwnK) * kPreThreads + tid);
        const uint64_t key = h[k].a;
        if (!(in[k] && (uint8_t)h[k].b == kOpPut && !skip_elem_os(kLocal, kOpPut, (uint8_t)(h[k].b >> 8)))) continue;
        bool created;
        uint32_t sl;
        if (own) {
            const bool in_table = pre_insert(hk, hv, key, i, created, sl);
            if (!in_table || created) {  // a key's first arrival lists it (no slot: it offers for itself)
                dl[atomicAdd(&nd, 1u)] = in_table ? sl : ~i;
            }
        } else {
            pre_insert_key(gk, key);
        }
    }
    __syncthreads();
    const Ctx c = make_ctx(a);
    const uint64_t hput[2] = {0, (uint64_t)kOpPut};
    const uint32_t cnt = HKV_DBG_ON(a, 2) ? 0 : nd;
    for (uint32_t base = 0; base < cnt; base += (kPreThreads / 4) * kPrePair) {
        uint64_t key[kPrePair];
        bool probe[kPrePair], ok[kPrePair];
        uint32_t idx[kPrePair];
        uint64_t phys[kPrePair];
        uint4 ln[kPrePair];
#pragma unroll
        for (int k = 0; k < kPrePair; ++k) {
            const uint32_t j = base + k * (kPreThreads / 4) + (tid >> 2);
            probe[k] = j < cnt;
            const uint32_t d = probe[k] ? dl[j] : 0u;
            idx[k] = !probe[k] ? kNone : d < (uint32_t)kPreHash ? hv[d] : ~d;
            key[k] = !probe[k] ? 0 : d < (uint32_t)kPreHash ? hk[d] : elem_key(a, (int64_t)idx[k]);
            if (probe[k] && head_end > 0 && key[k] != ~0ull) {  // a head PUT of the key comes first
                uint32_t sl = pre_slot(key[k]);
                for (int n = 0; n < kPreHash; ++n) {
                    const uint64_t g = gk[sl];
                    if (g == ~0ull) break;
                    if (g == key[k]) {
                        probe[k] = false;
                        break;
                    }
                    sl = (sl + 1) & (kPreHash - 1);
                }
            }
        }
        lookup_pair<kPrePair>(a, key, probe, q, gbase, ok, phys, ln);
#pragma unroll
        for (int k = 0; k < kPrePair; ++k) {
            Meta m0;
            const uint64_t ek = line_key_meta(ln[k], m0);
            if (q != 0 || !ok[k] || ek != key[k]) continue;
            if (!would_mutate(kLocal, reinterpret_cast<const uint8_t *>(hput), m0, c) || HKV_DBG_ON(a, 1)) continue;
            atomicMin(a.fw + fw_index(a, phys[k]), ((unsigned long long)(~a.rtag0) << 32) | idx[k]);
        }
    }
}

// exec_read / exec_write (hermesKV.c:251-356, with the skew optimisations of :196-238) for a local op
// of the direct path (RMWs off) that leaves its key's meta m as it is: the caller has excluded the
// branches that change it (update_actions, write replays) -- the element is not its key's first
// mutating element, so would_mutate is false against S_0, or m is the key's meta after that first write
// -- and only the element's own bytes move, without the generic dispatch's meta updates. An element
// that would mutate after all raises error flag bit 0, as the generic path's meta check does.
__device__ __forceinline__ void local_resolve_nm(const BatchArgs &a, uint8_t *x, const uint8_t *ent, const Meta &m)
{
    const uint8_t oc = x[8], st = m_state(m);
    const bool obi_empty = m_obi(m) == kObiEmpty;
    bool mut = false;
    if (oc == kOpGet) {
        if (st == kValid) {
            copy_value<31>(x + kOpValueOff, ent + kEntryValueOff, 31);
            x[9] = kGetComplete;
            x[10] = (uint8_t)((m_val_len(m) >> a.g.shift) - kOpMetaSize);
        } else if (st == kInvalidWrite || st == kWrite || st == kReplay) {
            x[9] = kGetStall;
        } else {
            x[9] = kEmpty;
            if (st == kInvalid) {   // hermes_check_membership_n_write_replay_actions, hermesKV.c:179-194
                const uint8_t lw = m_lwid(m);
                if (lw < 8 && ((a.g_membership >> lw) & 1u)) x[9] = kGetStall;
                else mut = obi_empty;
            }
        }
        if (a.g.skew & kSkewReadComplete) hot_read_complete(x, m.ver, m_cid(m));
    } else if (oc == kOpPut) {
        mut = (st == kValid || st == kInvalid) && obi_empty;
        x[9] = kPutStall;
        if (a.g.skew & kSkewWriteCoalesce) {   // as exec_write (hkv_exec.h)
            const uint32_t cv = m.ver & 0xFFFFu;
            uint32_t over = ld32(x + 12);
            if (st != kReplay && over == 0) {
                st32(x + 12, cv);
                over = cv;
            }
            if (over > 0 && over + 1u < cv) x[9] = kPutComplete;
        }
    }
    if (mut && a.error_flags) atomicOr(a.error_flags, 1u);
}

// Every element, F final (except on INVALID keys): see the section comment. One wave per block and
// nothing shared beyond it. The lookup runs four lanes per element (each lane holds 16 B of the op
// and of the log line); the wave-private LDS copies of op and entry are then resolved one element
// per lane, so the exec code's branches are paid once per 32 elements; the ops go back whole.
// Every hit's F word is loaded beside its log line; the word alone says whether this launch's prepass
// offered a first candidate for the key (first_cand)
// SGPR budget of the local launch's kernels (HKV_LOCAL_NUM_SGPR, a build macro for A/B): waves are admitted
// per SIMD by ~800 SGPRs / (ceil(sgpr/16) * 16 + 16) (MI355X_MICROARCH.md, "Residency"), so 92 SGPRs allow
// 7 waves and 80 allow 8
#ifndef HKV_LOCAL_NUM_SGPR
#define HKV_LOCAL_NUM_SGPR 80   // round 6: local launch 353-355 -> 341-351 us (gpurun_out/r06c), 7 -> 8 waves per SIMD
#endif
#if HKV_LOCAL_NUM_SGPR > 0
#define HKV_LOCAL_SGPR_ATTR __attribute__((amdgpu_num_sgpr(HKV_LOCAL_NUM_SGPR)))
#else
#define HKV_LOCAL_SGPR_ATTR
#endif
// NW waves per block (round 6): each wave works on its own 32 elements as before, and after the block's
// barrier the stage bytes and the state mirror of all NW * 32 elements go out as whole 64-byte blocks (a
// wave's 32 bytes alone are half a block, which HBM writes with a read-modify-write: tools/calib_bench.hip,
// 16-B random writes 2.4x the time of 64-B ones).
#ifndef HKV_LF_WAVES
#define HKV_LF_WAVES 2
#endif
constexpr int kLfWaves = HKV_LF_WAVES;   // waves per k_local_fused block (a build macro for A/B)
template <int P, int NW>
__global__ __launch_bounds__(64 * NW) HKV_LOCAL_SGPR_ATTR void k_local_fused(BatchArgs a)
{
    constexpr int E = 16 * P;   // elements per wave: P per lane group
    constexpr int EB = E * NW;  // elements per block
    __shared__ uint4 sops_b[NW][E * 4];   // 64 B per op (56 used)
    __shared__ uint4 sln_b[NW][E * 4];
    __shared__ unsigned long long sfw_b[NW][E];
    __shared__ uint32_t sent_b[NW][E];    // entry id of a hit, kNone otherwise
    __shared__ uint8_t sprb_b[NW][E];     // probed (not skipped)
    __shared__ uint32_t sst[EB / 4], sstate[EB / 4];   // the block's stage bytes and state mirror
    __shared__ uint32_t sdef[EB];
    __shared__ uint32_t ndef;
    const int w = threadIdx.x >> 6, tid = threadIdx.x & 63, q = tid & 3, gbase = tid & ~3;
    uint4 *sops = sops_b[w], *sln = sln_b[w];
    unsigned long long *sfw = sfw_b[w];
    uint32_t *sent = sent_b[w];
    uint8_t *sprb = sprb_b[w];
    const int64_t ib = (int64_t)blockIdx.x * EB, i0 = ib + (int64_t)w * E;
    if (threadIdx.x == 0) ndef = 0;
    uint64_t key[P];
    bool probe[P], ok[P], live[P];
    uint64_t phys[P];
    uint4 ln[P], op[P];
    int te[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        te[k] = k * 16 + (tid >> 2);
        const int64_t i = i0 + te[k];
        live[k] = i < a.n;
        op[k] = make_uint4(0u, 0u, 0u, 0u);
        if (live[k]) {
            const uint8_t *xg = a.elems + i * 56 + 16 * q;
            U64x2 p{0, 0};
            if (a.patch) p = *reinterpret_cast<const U64x2 *>(a.patch + i * 16);
            if (q < 3) {
                op[k] = *reinterpret_cast<const uint4 *>(xg);
            } else {
                const uint64_t t = *reinterpret_cast<const uint64_t *>(xg);
                op[k].x = (uint32_t)t;
                op[k].y = (uint32_t)(t >> 32);
            }
            if (patch_valid(p.b)) op[k] = patch_chunk(op[k], q, p.a, p.b);
        }
        sops[te[k] * 4 + q] = op[k];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        // lane 0 of the group holds op bytes 0..15: the key and the header
        key[k] = (uint64_t)(uint32_t)__shfl((int)op[k].x, 0, 4) | ((uint64_t)(uint32_t)__shfl((int)op[k].y, 0, 4) << 32);
        const uint32_t h0 = (uint32_t)__shfl((int)op[k].z, 0, 4);
        probe[k] = false;
        if (live[k] && !HKV_DBG_ON(a, 128))
            probe[k] = in_count(a, (uint32_t)(i0 + te[k])) && !skip_elem_os(kLocal, (uint8_t)h0, (uint8_t)(h0 >> 8));
    }
    unsigned long long fwv[P];   // a hit's F word, loaded beside its log line
    if (HKV_DBG_ON(a, 512)) {   // (timing modes) no F loads
        lookup_pair<P>(a, key, probe, q, gbase, ok, phys, ln);
#pragma unroll
        for (int k = 0; k < P; ++k) fwv[k] = ~0ull;
    } else {
        lookup_pair_f<P>(a, key, probe, q, gbase, ok, phys, ln, fwv);
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        Meta m;
        const uint64_t ek = line_key_meta(ln[k], m);
        const bool hit = ok[k] && ek == key[k];
        // keys INVALID at S_0 take their F after this pass (k_local_deferred)
        const unsigned long long f = hit && m_state(m) != kInvalid && q == 0 ? fwv[k] : ~0ull;
        if (hit) sln[te[k] * 4 + q] = ln[k];
        if (q == 0) {
            sfw[te[k]] = f;
            sent[te[k]] = hit ? (uint32_t)(phys[k] / a.g.entry_unit) : kNone;
            sprb[te[k]] = probe[k];
        }
    }
    __syncthreads();
    if (tid < E && i0 + tid < a.n && !HKV_DBG_ON(a, 64)) {
        const int64_t i = i0 + tid;
        uint8_t *x = reinterpret_cast<uint8_t *>(&sops[tid * 4]);
        uint8_t *ent = reinterpret_cast<uint8_t *>(&sln[tid * 4]);
        const uint32_t e = sent[tid];
        uint8_t st = kStDone;
        if (e != kNone) {
            Ctx c = make_ctx(a);
            Meta m;
            meta_load(ent, m);
            const bool wm = would_mutate(kLocal, x, m, c);
            if (m_state(m) == kInvalid) {
                // GET replays may mutate: they offer F now, and the key's elements resolve later
                if (wm) {
                    const uint64_t ph = phys_of(a, e);
                    offer(a.fw + fw_index(a, ph), a.rtag0, (uint32_t)i);
                    if ((uint8_t)(m.w5 >> 16) != a.ltag) a.log[ph + kEntryMetaOff + 4] = a.ltag;
                }
                st = kStDefer;
                sdef[atomicAdd(&ndef, 1u)] = (uint32_t)i;
            } else {
                const uint32_t f = first_cand(sfw[tid], a.rtag0);
                // a mutating element must have offered itself in k_local_pre
                if (wm && (f == kNone || f > (uint32_t)i) && a.error_flags) atomicOr(a.error_flags, 4u);
                if ((uint32_t)i == f) {
                    apply_to_shadow<kLocal, 31>(a, x, (uint32_t)i, ent);
                    st = kStCommit;
                } else {
                    // F of a key that is not INVALID is its first PUT (k_local_pre)
                    local_resolve_nm(a, x, ent, f != kNone && (uint32_t)i > f ? after_first<kLocal>(a, m, f, 1) : m);
                }
            }
        } else if (sprb[tid]) {
            x[9] = kMiss;
        }
        // k_local_pre read only the PUTs the caller's opcode mirror names
        if (a.opc && sprb[tid] && x[8] == kOpPut && a.opc[i] != kOpPut && a.error_flags) atomicOr(a.error_flags, 8u);
        if (!HKV_DBG_ON(a, 1024)) a.ent[i] = e;
        // a deferred element's state byte is written again by k_local_deferred, after this pass
        reinterpret_cast<uint8_t *>(sst)[w * E + tid] = st;
        reinterpret_cast<uint8_t *>(sstate)[w * E + tid] = x[9];
    }
    __syncthreads();
    // the block's stage bytes and state mirror as whole blocks (a partial last block byte by byte)
    if (!HKV_DBG_ON(a, 1024) && !HKV_DBG_ON(a, 64)) {
        if (ib + EB <= a.n && ((uintptr_t)a.state_out & 3) == 0) {   // (st is 256-byte aligned)
            if ((int)threadIdx.x < EB / 4) {
                reinterpret_cast<uint32_t *>(a.st + ib)[threadIdx.x] = sst[threadIdx.x];
                if (a.state_out) reinterpret_cast<uint32_t *>(a.state_out + ib)[threadIdx.x] = sstate[threadIdx.x];
            }
        } else if ((int)threadIdx.x < EB && ib + threadIdx.x < a.n) {
            a.st[ib + threadIdx.x] = reinterpret_cast<const uint8_t *>(sst)[threadIdx.x];
            if (a.state_out) a.state_out[ib + threadIdx.x] = reinterpret_cast<const uint8_t *>(sstate)[threadIdx.x];
        }
    }
    // the waiting elements (keys INVALID at S_0: rare), appended once per block
    if (ndef && threadIdx.x == 0) {
        const uint32_t base = atomicAdd(&a.ctr[kCtrDefer], ndef);
        for (uint32_t j = 0; j < ndef; ++j) a.fbl[base + j] = sdef[j];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!live[k] || HKV_DBG_ON(a, 256)) continue;
        uint8_t *xg = a.elems + (i0 + te[k]) * 56 + 16 * q;
        const uint4 v = sops[te[k] * 4 + q];
        if (q < 3) *reinterpret_cast<uint4 *>(xg) = v;
        else *reinterpret_cast<uint64_t *>(xg) = (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
}

// ------------------------------------------------------------------ launches with unique keys
// HKV_BATCH_UNIQUE: no key appears twice among the launch's elements, so every element is its key's
// only one and sees S_0 in any serial order: after k_lookup's lookup (four lanes per element, two
// elements per lane group) lane 0 of the group runs the exec function on the element and the entry
// in place and stores the meta back -- one pass, each entry line read and written once. (INV
// launches: a peer's round slab, see hermeskv.h.) With check_unique every element also swaps its
// index into its key's F word, tagged with the launch; finding the launch's tag there means a
// second element of the key (error bit 4).
template <int TYPE, int SV, int P = kLookupPair>
__global__ __launch_bounds__(256) void k_unique(BatchArgs a)
{
    const int q = threadIdx.x & 3;
    const int gbase = (threadIdx.x & 63) & ~3;
    int64_t gi[P];
    uint64_t key[P], hdr[P];
    bool probe[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        gi[k] = ((int64_t)blockIdx.x * P + k) * 64 + (threadIdx.x >> 2);
        uint64_t kk = 0, hh = 0;
        bool p = false;
        if (gi[k] < a.n && q == 0) {
            int64_t start = 0;
            int32_t b = 0;
            bool in = true;
            if (a.offsets) {
                b = batch_of(a, gi[k], start);
            } else {
                b = (int32_t)(gi[k] / a.stride);
                start = (int64_t)b * a.stride;
                in = a.counts == nullptr || gi[k] - start < a.counts[b];
            }
            if (in) {
                const U64x2 h = *reinterpret_cast<const U64x2 *>(a.elems + gi[k] * a.esz);
                kk = h.a;
                hh = h.b;
                if (skip_elem_os(TYPE, (uint8_t)hh, (uint8_t)(hh >> 8))) {
                    if (TYPE == kInvs && a.ns_idx) atomicMax(&a.ns_idx[b], (int32_t)(gi[k] - start));
                } else {
                    p = true;
                }
            }
        }
        key[k] = (uint64_t)(uint32_t)__shfl((int)(uint32_t)kk, 0, 4) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(kk >> 32), 0, 4) << 32);
        probe[k] = __shfl((int)p, 0, 4) != 0;
        hdr[k] = hh;
    }
    bool ok[P];
    uint64_t phys[P];
    uint4 ln[P];
    lookup_pair<P>(a, key, probe, q, gbase, ok, phys, ln);
    Meta m[P];
    uint64_t ek[P];
#pragma unroll
    for (int k = 0; k < P; ++k) ek[k] = line_key_meta(ln[k], m[k]);
    if (q != 0) return;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!probe[k]) continue;
        uint8_t *x = a.elems + gi[k] * a.esz;
        if (!(ok[k] && ek[k] == key[k])) {
            x[9] = kMiss;
            continue;
        }
        if (a.check_unique) {
            const unsigned long long v = ((unsigned long long)(~a.rtag0) << 32) | (uint32_t)gi[k];
            const unsigned long long old = atomicExch(a.fw + fw_index(a, phys[k]), v);
            if ((uint32_t)(old >> 32) == ~a.rtag0 && a.error_flags) atomicOr(a.error_flags, 16u);
        }
        uint8_t *entry = a.log + phys[k];
        Ctx c = make_ctx(a);
        uint8_t idx = 0;
        if (TYPE == kAcks) {   // the element's batch: its read_write_ops and their state mirror
            uint8_t *xx;
            elem_at(a, (uint32_t)gi[k], xx, idx, c);
        }
        Meta t = m[k];
        dispatch<SV>(TYPE, x, entry, idx, t, c);
        if (!meta_equal(t, m[k])) meta_store(entry, t);
    }
}

// k_unique for 64-B entries: the lookup as in k_local_fused (one wave per block, four lanes per
// element, each holding 16 B of the element and of the entry line), both staged in LDS, then one
// lane per element runs the exec function on the LDS copies; each lane writes back its 16-B chunks
// of the element and of the entry line that changed. The exec code touches LDS only, and the
// global writes are whole 16-B words.
__device__ __forceinline__ uint4 load_chunk(const uint8_t *x, int q, int32_t esz)
{
    if (16 * q + 16 <= esz) return *reinterpret_cast<const uint4 *>(x + 16 * q);
    if (16 * q + 8 <= esz) {
        const uint64_t t = *reinterpret_cast<const uint64_t *>(x + 16 * q);
        return make_uint4((uint32_t)t, (uint32_t)(t >> 32), 0u, 0u);
    }
    return make_uint4(0u, 0u, 0u, 0u);
}

__device__ __forceinline__ bool chunk_equal(const uint4 &a, const uint4 &b)
{
    return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}

template <int TYPE, int P = kLookupPair>
__global__ __launch_bounds__(64) void k_unique_lds(BatchArgs a)
{
    constexpr int E = 16 * P;   // elements per wave: P per lane group
    __shared__ uint4 sops[E * 4];
    __shared__ uint4 sln[E * 4];
    __shared__ uint32_t sent[E];
    __shared__ uint8_t sprb[E];
    const int tid = threadIdx.x, q = tid & 3, gbase = tid & ~3;
    const int64_t i0 = (int64_t)blockIdx.x * E;
    const int64_t n_live = a.offsets ? (int64_t)a.offsets[a.n_batches] : a.n;   // packed: past the last offset
    uint64_t key[P];
    bool probe[P], ok[P], live[P];
    uint64_t phys[P];
    uint4 ln[P], op[P];
    int te[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        te[k] = k * 16 + (tid >> 2);
        const int64_t i = i0 + te[k];
        live[k] = i < a.n && i < n_live;
        op[k] = live[k] ? load_chunk(a.elems + i * a.esz, q, a.esz) : make_uint4(0u, 0u, 0u, 0u);
        sops[te[k] * 4 + q] = op[k];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        key[k] = (uint64_t)(uint32_t)__shfl((int)op[k].x, 0, 4) | ((uint64_t)(uint32_t)__shfl((int)op[k].y, 0, 4) << 32);
        const uint32_t h0 = (uint32_t)__shfl((int)op[k].z, 0, 4);
        probe[k] = false;
        const int64_t i = i0 + te[k];
        if (live[k] && (a.offsets || in_count(a, (uint32_t)i))) {
            if (!skip_elem_os(TYPE, (uint8_t)h0, (uint8_t)(h0 >> 8))) {
                probe[k] = true;
            } else if (TYPE == kInvs && a.ns_idx && q == 0) {
                int64_t start;
                const int32_t b = batch_of(a, i, start);
                atomicMax(&a.ns_idx[b], (int32_t)(i - start));
            }
        }
    }
    lookup_pair<P>(a, key, probe, q, gbase, ok, phys, ln);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        Meta m;
        const uint64_t ek = line_key_meta(ln[k], m);
        const bool hit = ok[k] && ek == key[k];
        sln[te[k] * 4 + q] = ln[k];
        if (q == 0) {
            sent[te[k]] = hit ? (uint32_t)(phys[k] / a.g.entry_unit) : kNone;
            sprb[te[k]] = probe[k];
        }
    }
    __syncthreads();
    if (tid < E && i0 + tid < n_live) {
        const int64_t i = i0 + tid;
        uint8_t *x = reinterpret_cast<uint8_t *>(&sops[tid * 4]);
        uint8_t *ent = reinterpret_cast<uint8_t *>(&sln[tid * 4]);
        const uint32_t e = sent[tid];
        if (e != kNone) {
            if (a.check_unique) {
                const unsigned long long v = ((unsigned long long)(~a.rtag0) << 32) | (uint32_t)i;
                const unsigned long long old = atomicExch(a.fw + fw_index(a, phys_of(a, e)), v);
                if ((uint32_t)(old >> 32) == ~a.rtag0 && a.error_flags) atomicOr(a.error_flags, 16u);
            }
            Ctx c = make_ctx(a);
            int done = -1;
            if (TYPE == kAcks) c.rw_done = &done;   // the batch is found only for a completion
            Meta m;
            meta_load(ent, m);
            Meta t = m;
            dispatch<31>(TYPE, x, ent, 0, t, c);
            if (!meta_equal(t, m)) meta_store(ent, t);
            if (TYPE == kAcks && done >= 0 && a.rw) {   // its read_write_ops slot and state mirror
                uint8_t *xx;
                uint8_t idx;
                elem_at(a, (uint32_t)i, xx, idx, c);
                complete_rw_slot(c, done);
            }
        } else if (sprb[tid]) {
            x[9] = kMiss;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!live[k]) continue;
        uint4 w = sops[te[k] * 4 + q];
        if (TYPE == kInvs && a.ack_out) {
            // the ACK callbacks (ack_skip_or_get_sender_id, ack_copy_and_modify_elem,
            // ack_modify_elem_after_send; the k_marshal_acks of hkv_workload.hip) on the element as the
            // batch left it: the header chunk is lane 0's, the INV leaves as ST_EMPTY once answered
            uint8_t *y = a.ack_out + (i0 + te[k]) * a.ack_out_size;
            const uint32_t hz = sops[te[k] * 4].z;
            const uint8_t oc = (uint8_t)hz;
            const bool full = oc == kOpInvAbort && a.ack_out_size >= (uint32_t)a.esz;
            if (oc == kInvSuccess || full) {
                uint4 c = w;
                if (q == 0)
                    c.z = (hz & ~0xFFFFu) | (oc == kInvSuccess ? kOpAck : kOpInvAbort) |
                          ((uint32_t)(uint8_t)a.g.machine_id << 8);
                if (q == 0 || (full && 16 * q < a.esz)) {
                    if (16 * q + 16 <= a.esz || q == 0) *reinterpret_cast<uint4 *>(y + 16 * q) = c;
                    else *reinterpret_cast<uint64_t *>(y + 16 * q) = (uint64_t)c.x | ((uint64_t)c.y << 32);
                }
            } else if (q == 0) {
                y[8] = kEmpty;
            }
            if (q == 0 && (oc == kInvSuccess || oc == kOpInvAbort || oc == kOpMembChange))
                w.z = (w.z & ~0xFFu) | kEmpty;
        }
        if (!chunk_equal(w, op[k])) {
            uint8_t *xg = a.elems + (i0 + te[k]) * a.esz + 16 * q;
            if (16 * q + 16 <= a.esz) *reinterpret_cast<uint4 *>(xg) = w;
            else *reinterpret_cast<uint64_t *>(xg) = (uint64_t)w.x | ((uint64_t)w.y << 32);
        }
        if (ok[k] && q > 0) {   // bytes 0..15 of a log line (the MICA key) never change
            const uint4 l = sln[te[k] * 4 + q];
            if (!chunk_equal(l, ln[k])) reinterpret_cast<uint4 *>(a.log + phys[k])[q] = l;
        }
    }
}

// HKV_BATCH_ROWS: k_unique_lds over positions instead of elements. Position j holds element j of
// every row, all of one key (or holes, opcode 0): the four lanes of a position load its element of
// every row and look the key up once, one lane applies the row elements in row order to the LDS copy
// of the entry -- exactly the rows' launches one after another, since each row holds the key once --
// and each element and the entry line are written back where they changed. An ACK's completion finds
// its read_write_ops once per position (the rows share the batch layout).
#ifdef HKV_ROWS_NUM_SGPR
#define HKV_ROWS_SGPR_ATTR __attribute__((amdgpu_num_sgpr(HKV_ROWS_NUM_SGPR)))
#else
#define HKV_ROWS_SGPR_ATTR
#endif
template <int TYPE, int RMAX, int CH, int P = kLookupPair>
#ifdef HKV_ROWS_WAVES   // (A/B builds) waves per SIMD k_unique_rows is compiled for
#define HKV_ROWS_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(HKV_ROWS_WAVES, 8)))
#else
#define HKV_ROWS_WAVES_ATTR
#endif
__global__ __launch_bounds__(64) HKV_ROWS_SGPR_ATTR HKV_ROWS_WAVES_ATTR void k_unique_rows(BatchArgs a)
{
    constexpr int E = 16 * P;   // positions per wave: P per lane group
    // CH: 16-B chunks of an element held in LDS (1 for 16-B ACKs, 4 for 56-B INVs)
    __shared__ uint4 sops[RMAX][E * CH];
    __shared__ uint4 sln[E * 4];
    __shared__ uint32_t sent[E];
    __shared__ uint8_t spart[E];   // bit r: row r's element takes part (present, in count, not skipped)
    const int tid = threadIdx.x, q = tid & 3, gbase = tid & ~3;
    const int64_t i0 = (int64_t)blockIdx.x * E;
    const int R = a.n_rows < RMAX ? a.n_rows : RMAX;
    // packed rows may end before the stride: elements past the last batch offset are in no batch
    const int64_t n_live = a.offsets ? (int64_t)a.offsets[a.n_batches] : a.n;
    uint64_t key[P];
    bool probe[P], ok[P], live[P];
    uint64_t phys[P];
    uint4 ln[P], op[RMAX][P];
    uint32_t part[P];
    int te[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        te[k] = k * 16 + (tid >> 2);
        const int64_t i = i0 + te[k];
        live[k] = i < a.n && i < n_live && (a.offsets || in_count(a, (uint32_t)i));
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            const bool on = live[k] && r < R && r != a.skip_row;
            op[r][k] = on && q < CH ? load_chunk(a.elems + (r * a.row_stride + i) * a.esz, q, a.esz)
                                    : make_uint4(0u, 0u, 0u, 0u);
            if (q < CH) sops[r][te[k] * CH + q] = op[r][k];
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        uint64_t kk = 0;
        uint32_t p = 0;
        bool mismatch = false;
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            const uint64_t kr = (uint64_t)(uint32_t)__shfl((int)op[r][k].x, 0, 4) |
                                ((uint64_t)(uint32_t)__shfl((int)op[r][k].y, 0, 4) << 32);
            const uint32_t h0 = (uint32_t)__shfl((int)op[r][k].z, 0, 4);
            if (!live[k] || r >= R || r == a.skip_row || (uint8_t)h0 == 0) continue;   // a hole
            if (skip_elem_os(TYPE, (uint8_t)h0, (uint8_t)(h0 >> 8))) continue;
            if (p && kr != kk) mismatch = true;
            if (!p) kk = kr;
            p |= 1u << r;
        }
        if (mismatch && q == 0 && a.error_flags) atomicOr(a.error_flags, 16u);
        key[k] = kk;
        part[k] = mismatch ? 0u : p;
        probe[k] = part[k] != 0;
    }
    lookup_pair<P>(a, key, probe, q, gbase, ok, phys, ln);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        Meta m;
        const uint64_t ek = line_key_meta(ln[k], m);
        const bool hit = ok[k] && ek == key[k];
        sln[te[k] * 4 + q] = ln[k];
        if (q == 0) {
            sent[te[k]] = hit ? (uint32_t)(phys[k] / a.g.entry_unit) : kNone;
            spart[te[k]] = (uint8_t)part[k];
        }
    }
    __syncthreads();
    if (tid < E && i0 + tid < n_live) {
        const int64_t i = i0 + tid;
        uint8_t *ent = reinterpret_cast<uint8_t *>(&sln[tid * 4]);
        const uint32_t e = sent[tid];
        const uint32_t p = spart[tid];
        if (e != kNone && p) {
            if (a.check_unique) {
                const unsigned long long v = ((unsigned long long)(~a.rtag0) << 32) | (uint32_t)i;
                const unsigned long long old = atomicExch(a.fw + fw_index(a, phys_of(a, e)), v);
                if ((uint32_t)(old >> 32) == ~a.rtag0 && a.error_flags) atomicOr(a.error_flags, 16u);
            }
            Ctx c = make_ctx(a);
            int done = -1;
            if (TYPE == kAcks) c.rw_done = &done;   // the batch is found only for a completion
            Meta m;
            meta_load(ent, m);
            Meta t = m;
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if ((p >> r) & 1u) dispatch<31>(TYPE, reinterpret_cast<uint8_t *>(&sops[r][tid * CH]), ent, 0, t, c);
            if (!meta_equal(t, m)) meta_store(ent, t);
            if (TYPE == kAcks && done >= 0 && a.rw) {
                uint8_t *xx;
                uint8_t idx;
                elem_at(a, (uint32_t)i, xx, idx, c);
                complete_rw_slot(c, done);
            }
        } else {
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if ((p >> r) & 1u) reinterpret_cast<uint8_t *>(&sops[r][tid * CH])[9] = kMiss;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!live[k]) continue;
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            if (r >= R || r == a.skip_row || q >= CH) continue;
            uint4 w = sops[r][te[k] * CH + q];
            if (TYPE == kAcks && CH == 1 && a.ack_out) {
                // the VAL callbacks (hermes_worker.c:122-157, as shipped): an element whose opcode is not
                // ACK_SUCCESS, MEMBERSHIP_CHANGE or EMPTY is sent as a VAL from this machine, every
                // non-empty one leaves empty; a hole (opcode 0) is no element
                const uint8_t oc = (uint8_t)w.z;
                uint4 v = make_uint4(0u, 0u, (uint32_t)kEmpty, 0u);
                if (oc != 0 && oc != kAckSuccess && oc != kOpMembChange && oc != kEmpty)
                    v = make_uint4(w.x, w.y, (w.z & ~0xFFFFu) | (uint32_t)kOpVal | ((uint32_t)(uint8_t)a.g.machine_id << 8), w.w);
                *reinterpret_cast<uint4 *>(a.ack_out + (r * a.row_stride + i0 + te[k]) * 16) = v;
                if (oc != 0 && oc != kEmpty) w.z = (w.z & ~0xFFu) | (uint32_t)kEmpty;
            }
            if (!chunk_equal(w, op[r][k])) {
                uint8_t *xg = a.elems + (r * a.row_stride + i0 + te[k]) * a.esz + 16 * q;
                if (16 * q + 16 <= a.esz) *reinterpret_cast<uint4 *>(xg) = w;
                else *reinterpret_cast<uint64_t *>(xg) = (uint64_t)w.x | ((uint64_t)w.y << 32);
            }
        }
        if (ok[k] && q > 0) {   // bytes 0..15 of a log line (the MICA key) never change
            const uint4 l = sln[te[k] * 4 + q];
            if (!chunk_equal(l, ln[k])) reinterpret_cast<uint4 *>(a.log + phys[k])[q] = l;
        }
    }
}

// k_unique for big objects (320-B entries, elements of up to 320 B: configs[2]): the same one pass,
// with each element and its whole entry staged in LDS by the element's four lanes (16-B chunks,
// coalesced), so the exec code -- 287-byte value copies included -- runs on LDS copies, and only the
// 16-B chunks that changed go back. One wave per kUbElems elements.
constexpr int kUbElems = 16;
constexpr int kUbChunks = 20;   // 320 B
template <int TYPE>
__global__ __launch_bounds__(64) void k_unique_big(BatchArgs a)
{
    // elements and entries in LDS; each lane keeps the chunks it loaded in registers (what changed goes
    // back), so a wave's LDS is 10 KB and four waves fit a SIMD
    __shared__ uint4 sx[kUbElems * kUbChunks];
    __shared__ uint4 se[kUbElems * kUbChunks];
    constexpr int kPerLane = (kUbChunks + 3) / 4;
    uint4 x0[kPerLane], e0[kPerLane];
    const int tid = threadIdx.x, q = tid & 3, el = tid >> 2, gbase = tid & ~3;
    const int64_t i = (int64_t)blockIdx.x * kUbElems + el;
    const bool live = i < a.n;
    const int nch = (a.esz + 15) / 16;
    uint8_t *xg = a.elems + i * a.esz;
#pragma unroll
    for (int u = 0; u < kPerLane; ++u) {
        const int c = q + 4 * u;
        const uint4 v = live && c < nch ? load_chunk(xg, c, a.esz) : make_uint4(0u, 0u, 0u, 0u);
        if (c < nch) sx[el * kUbChunks + c] = v;
        x0[u] = v;
    }
    const uint4 c0 = sx[el * kUbChunks];   // the element's key and header (every lane of the group)
    const uint64_t key = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
    bool probe = false;
    if (live && (a.offsets || in_count(a, (uint32_t)i))) {
        if (!skip_elem_os(TYPE, (uint8_t)c0.z, (uint8_t)(c0.z >> 8))) {
            probe = true;
        } else if (TYPE == kInvs && a.ns_idx && q == 0) {
            int64_t start;
            const int32_t b = batch_of(a, i, start);
            atomicMax(&a.ns_idx[b], (int32_t)(i - start));
        }
    }
    bool ok;
    uint64_t phys;
    uint4 ln;
    lookup_pair<1>(a, &key, &probe, q, gbase, &ok, &phys, &ln);
    Meta m0;
    const uint64_t ek = line_key_meta(ln, m0);
    const bool hit = ok && ek == key;
#pragma unroll
    for (int u = 0; u < kPerLane; ++u) e0[u] = make_uint4(0u, 0u, 0u, 0u);
    if (hit) {
        const uint4 *eg = reinterpret_cast<const uint4 *>(a.log + phys);
#pragma unroll
        for (int u = 0; u < kPerLane; ++u) {
            const int c = q + 4 * u;
            if (c >= kUbChunks) continue;
            const uint4 v = c < 4 ? ln : eg[c];
            se[el * kUbChunks + c] = v;
            e0[u] = v;
        }
    }
    __syncthreads();
    if (q == 0 && live) {
        uint8_t *x = reinterpret_cast<uint8_t *>(&sx[el * kUbChunks]);
        uint8_t *ent = reinterpret_cast<uint8_t *>(&se[el * kUbChunks]);
        if (hit) {
            if (a.check_unique) {
                const unsigned long long v = ((unsigned long long)(~a.rtag0) << 32) | (uint32_t)i;
                const unsigned long long old = atomicExch(a.fw + fw_index(a, phys), v);
                if ((uint32_t)(old >> 32) == ~a.rtag0 && a.error_flags) atomicOr(a.error_flags, 16u);
            }
            Ctx c = make_ctx(a);
            int done = -1;
            if (TYPE == kAcks) c.rw_done = &done;   // the batch is found only for a completion
            Meta m;
            meta_load(ent, m);
            Meta t = m;
            dispatch<287>(TYPE, x, ent, 0, t, c);
            if (!meta_equal(t, m)) meta_store(ent, t);
            if (TYPE == kAcks && done >= 0 && a.rw) {   // its read_write_ops slot and state mirror
                uint8_t *xx;
                uint8_t idx;
                elem_at(a, (uint32_t)i, xx, idx, c);
                complete_rw_slot(c, done);
            }
        } else if (probe) {
            x[9] = kMiss;
        }
    }
    __syncthreads();
    if (live) {
        const uint32_t hz = sx[el * kUbChunks].z;   // the element's opcode after the batch (byte 8)
        const uint8_t oc = (uint8_t)hz;
        if (TYPE == kInvs && a.ack_out) {
            // the ACK callbacks on the element as the batch left it (as in k_unique_lds): an INV_SUCCESS
            // answers with its header, an OP_INV_ABORT with the whole element when the ACK slot holds it
            uint8_t *y = a.ack_out + i * a.ack_out_size;
            const bool full = oc == kOpInvAbort && a.ack_out_size >= (uint32_t)a.esz;
            if (oc == kInvSuccess || full) {
                for (int c = q; c < (full ? nch : 1); c += 4) {
                    uint4 w = sx[el * kUbChunks + c];
                    if (c == 0)
                        w.z = (hz & ~0xFFFFu) | (oc == kInvSuccess ? kOpAck : kOpInvAbort) |
                              ((uint32_t)(uint8_t)a.g.machine_id << 8);
                    if (16 * c + 16 <= a.esz || c == 0) *reinterpret_cast<uint4 *>(y + 16 * c) = w;
                    else *reinterpret_cast<uint64_t *>(y + 16 * c) = (uint64_t)w.x | ((uint64_t)w.y << 32);
                }
            } else if (q == 0) {
                y[8] = kEmpty;
            }
        }
#pragma unroll
        for (int u = 0; u < kPerLane; ++u) {
            const int c = q + 4 * u;
            if (c >= nch) continue;
            uint4 w = sx[el * kUbChunks + c];
            if (TYPE == kInvs && a.ack_out && c == 0 && (oc == kInvSuccess || oc == kOpInvAbort || oc == kOpMembChange))
                w.z = (w.z & ~0xFFu) | kEmpty;   // answered (ack_modify_elem_after_send)
            if (chunk_equal(w, x0[u])) continue;
            if (16 * c + 16 <= a.esz) *reinterpret_cast<uint4 *>(xg + 16 * c) = w;
            else *reinterpret_cast<uint64_t *>(xg + 16 * c) = (uint64_t)w.x | ((uint64_t)w.y << 32);
        }
    }
    if (hit) {   // bytes 0..15 of an entry (the MICA key) never change
        uint4 *eg = reinterpret_cast<uint4 *>(a.log + phys);
#pragma unroll
        for (int u = 0; u < kPerLane; ++u) {
            const int c = q + 4 * u;
            if (c >= kUbChunks) continue;
            const uint4 w = se[el * kUbChunks + c];
            if (c > 0 && !chunk_equal(w, e0[u])) eg[c] = w;
        }
    }
}

// Elements of keys that were INVALID at S_0, against their key's final F (k_resolve0_direct's rules)
__global__ __launch_bounds__(256) void k_local_deferred(BatchArgs a)
{
    const uint32_t nd = a.ctr[kCtrDefer];
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < nd; j += gridDim.x * 256u) {
        const uint32_t i = a.fbl[j];
        const uint32_t e = a.ent[i];
        uint8_t *xg;
        uint8_t idx;
        Ctx c = make_ctx(a);
        elem_at(a, i, xg, idx, c);
        Meta m;
        meta_load(entry_of(a, e), m);
        const uint32_t f = first_cand(*fw_of(a, e), a.rtag0);
        uint8_t st = kStDone;
        if (f == kNone || i < f) {
            Meta tm = m;
            dispatch<31>(kLocal, xg, entry_of(a, e), idx, tm, c);
            if (a.error_flags && !meta_equal(tm, m)) atomicOr(a.error_flags, 1u);
        } else if (i == f) {
            apply_to_shadow<kLocal, 31>(a, nullptr, i, entry_of(a, e));
            st = kStCommit;
        } else {
            const Meta m1 = after_first<kLocal>(a, m, f, 0);
            Meta tm = m1;
            dispatch<31>(kLocal, xg, entry_of(a, e), idx, tm, c);
            if (a.error_flags && !meta_equal(tm, m1)) atomicOr(a.error_flags, 1u);
        }
        a.st[i] = st;
        note_state(a, i, xg);
    }
}

// Round r >= 1 resolve over the pending elements (sparse: direct global access), against S_r in
// the shadow of round r-1's first candidate of the element's key.
// After the last round, elements still pending go to the fallback list.
template <int TYPE, int SV>
__global__ __launch_bounds__(256) void k_resolve(BatchArgs a, int r)
{
    // 16-B messages (ACKs, VALs): the element is dispatched on an LDS copy, one 16-B access in and
    // one out instead of the exec functions' byte-wise global accesses. (A 56-B op costs more to
    // write back whole than the one or two bytes an INV changes.)
    extern __shared__ uint64_t sx[];
    const bool kStage = SV == 31 && a.esz <= 16;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool left = false;
    // big values: copied a wave per value after the exec calls (see k_resolve0_direct); the shadow
    // they read (round r-1's first candidate's) is not written in this round
    VCopy vc{nullptr, nullptr};
    VCopy *vcp = SV != 31 && a.g.st_value <= 320 ? &vc : nullptr;
    const bool wave_shadow = SV != 31 && vcp;   // see k_resolve0_direct
    bool cand = false;
    uint32_t prev = 0;
    if (i < a.n && a.st[i] == kStPend) {
        const uint32_t e = a.ent[i];
        const uint32_t f = first_cand(*fw_of(a, e), a.rtag0 + (uint32_t)r);
        prev = a.pf[i];  // S_r lives in the shadow of round r-1's first candidate
        if (f == kNone || (uint32_t)i <= f) {
            uint8_t *xg = a.elems + i * a.esz;
            uint8_t *xl = reinterpret_cast<uint8_t *>(sx) + threadIdx.x * (uint32_t)a.esz;
            if (kStage) copy_elem(xl, xg, a.esz);
            if ((uint32_t)i != f) {
                if (kStage) resolve_elem<TYPE, SV>(a, (uint32_t)i, xl, shadow_of(a, prev));
                else resolve_elem<TYPE, SV>(a, (uint32_t)i, xg, shadow_of(a, prev), vcp);
                a.st[i] = kStDone;
            } else {
                if (wave_shadow) cand = true;
                else apply_to_shadow<TYPE, SV>(a, kStage ? xl : nullptr, (uint32_t)i, shadow_of(a, prev));
                a.st[prev] = kStDone;  // superseded
                a.st[i] = kStCommit;
            }
            if (kStage) copy_elem(xg, xl, a.esz);
            if (!cand) note_state(a, i, kStage ? xl : xg);
        } else {
            a.pf[i] = f;  // after the last round: identifies the key's run in k_fb_exec
            left = r == a.rounds;
        }
    }
    if (wave_shadow) {
        apply_to_shadow_wave<TYPE, SV>(a, cand, (uint32_t)i, cand ? shadow_of(a, prev) : nullptr, vc);
        if (cand) note_state(a, i, a.elems + i * a.esz);
    }
    if (SV != 31) wave_value_copies(vc, a.g.st_value, kVcBatch);
    if (r == a.rounds) {  // wave-aggregated append (uniform branch)
        const uint32_t t = agg_ticket(&a.ctr[kCtrFbL], 0u, left);
        if (left) a.fbl[t] = (uint32_t)i;
    }
}

// ------------------------------------------------------------------ fallback
__device__ __forceinline__ uint32_t pow2ceil(uint32_t c) { return c <= 1 ? 1u : 1u << (32 - __clz(c - 1)); }

// Final commit of a launch: every key's last shadow becomes its entry.
template <int SV>
__global__ __launch_bounds__(256) void k_commit(BatchArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (SV != 31) {  // big entries: copied by the whole wave, 16 B per lane, several entries per step
        const bool mine = i < a.n && a.st[i] == kStCommit;
        const uint32_t e = mine ? a.ent[i] : 0u;
        wave_block_copies(mine ? entry_of(a, e) : nullptr, mine ? shadow_of(a, (uint32_t)i) : nullptr,
                          a.g.entry_size);
        return;
    }
    if (i >= a.n || a.st[i] != kStCommit) return;
    uint8_t *dst = entry_of(a, a.ent[i]);
    const uint8_t *src = shadow_of(a, (uint32_t)i);
    if (SV == 31) {  // 64-B entries and shadows are 16-byte aligned
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        const uint4 w0 = s4[0], w1 = s4[1], w2 = s4[2], w3 = s4[3];
        d4[0] = w0;
        d4[1] = w1;
        d4[2] = w2;
        d4[3] = w3;
    } else {
        copy_entry(dst, src, a.g.entry_size);
    }
}

// k_commit for 64-B entries over few commits (the local direct path: one per key a PUT first
// wrote): each wave takes 1024 elements, reads their stage bytes 16 per lane, lists the committing
// ones in LDS (a wave-wide prefix sum of the per-lane counts), then copies their shadows 16
// entries at a time, four lanes per entry. One wave per 1024 elements instead of one thread per
// element: k_commit's cost was its 4M threads, not its copies.
constexpr int kCwElems = 1024;
__global__ __launch_bounds__(256) void k_commit_w(BatchArgs a)
{
    __shared__ uint32_t lst[4][kCwElems];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e0 = ((int64_t)blockIdx.x * 4 + w) * kCwElems + 16 * lane;
    uint32_t m = 0;
    if (e0 + 16 <= a.n) {   // st is 256-byte aligned and e0 a multiple of 16
        const uint4 s4 = *reinterpret_cast<const uint4 *>(a.st + e0);
        const uint32_t sw[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int b = 0; b < 16; ++b)
            if (((sw[b >> 2] >> (8 * (b & 3))) & 0xFFu) == kStCommit) m |= 1u << b;
    } else {
        for (int b = 0; b < 16; ++b)
            if (e0 + b < a.n && a.st[e0 + b] == kStCommit) m |= 1u << b;
    }
    const uint32_t c = __popc(m);
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, d, 64);
        if (lane >= d) incl += v;
    }
    const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
    for (uint32_t pos = incl - c; m; m &= m - 1) lst[w][pos++] = (uint32_t)e0 + (uint32_t)(__ffs(m) - 1);
    __syncthreads();
    const int q = lane & 3;
    for (uint32_t j = (uint32_t)(lane >> 2); j < total; j += 16) {
        const uint32_t i = lst[w][j];
        const uint4 v = reinterpret_cast<const uint4 *>(shadow_of(a, i))[q];
        reinterpret_cast<uint4 *>(entry_of(a, a.ent[i]))[q] = v;
    }
}

constexpr int kFbThreads = 1024;
constexpr int kFbPerThread = 8;
constexpr int kFbChunk = kFbThreads * kFbPerThread;
constexpr int kFbLds = 8192;    // (F_R, element) pairs sorted in LDS
constexpr int kFbSerial = 32;   // runs up to this long are applied by one thread

__device__ __forceinline__ int block_min(int v, int *lds)
{
    for (int o = 32; o > 0; o >>= 1) {
        const int u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = lds[0];
#pragma unroll
    for (int w = 1; w < kFbThreads / 64; ++w) r = lds[w] < r ? lds[w] : r;
    return r;
}

// ascending bitonic sort of n (a power of two) words, by the whole workgroup
__device__ void bitonic_sort(unsigned long long *s, uint32_t n)
{
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
                const uint32_t u = t ^ j;
                if (u > t) {
                    const unsigned long long x = s[t], y = s[u];
                    if ((x > y) == ((t & k) == 0)) {
                        s[t] = y;
                        s[u] = x;
                    }
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
}

// Elements still pending after the last round (the fallback list), after k_commit: every such
// element's key had a first candidate F_R in the last round, whose index it holds in pf. Workgroup
// b owns the keys with F_R % gridDim == b: it gathers their members as (F_R, element) pairs (LDS,
// or a region of mem beyond kFbLds pairs), sorts them (each key is then one run in element order)
// and finishes each run from the committed entry with first-candidate passes: repeat {block min
// of the first candidate f against the shared meta; resolve members before f on private copies;
// barrier; f applies; barrier} over chunks of kFbChunk members until a chunk has no candidate.
template <int TYPE, int SV>
__global__ __launch_bounds__(kFbThreads) void k_fb_exec(BatchArgs a)
{
    __shared__ unsigned long long srt[kFbLds];
    __shared__ Meta sm;
    __shared__ int red[kFbThreads / 64];
    __shared__ uint32_t lcnt, loff;
    const int tid = threadIdx.x;
    const uint32_t nl = a.ctr[kCtrFbL];
    if (nl == 0) return;  // uniform
    const uint32_t G = gridDim.x, me = blockIdx.x;
    if (tid == 0) lcnt = 0;
    __syncthreads();
    for (uint32_t j = tid; j < nl; j += kFbThreads)
        if (a.pf[a.fbl[j]] % G == me) atomicAdd(&lcnt, 1u);
    __syncthreads();
    const uint32_t cnt = lcnt, p2 = pow2ceil(cnt);
    if (cnt == 0) return;  // uniform
    unsigned long long *ord = srt;
    if (p2 > (uint32_t)kFbLds) {
        if (tid == 0) loff = atomicAdd(&a.ctr[kCtrFbM], p2);
        __syncthreads();
        ord = a.mem + loff;
    }
    __syncthreads();
    if (tid == 0) lcnt = 0;
    __syncthreads();
    for (uint32_t j = tid; j < nl; j += kFbThreads) {
        const uint32_t i = a.fbl[j], f = a.pf[i];
        if (f % G == me) ord[atomicAdd(&lcnt, 1u)] = ((unsigned long long)f << 32) | i;
    }
    for (uint32_t j = cnt + tid; j < p2; j += kFbThreads) ord[j] = ~0ull;
    __threadfence_block();
    __syncthreads();
    bitonic_sort(ord, p2);
    Ctx c = make_ctx(a);
    // serial tier: the head of a run of at most kFbSerial members applies it alone, in order
    for (uint32_t p = tid; p < cnt; p += kFbThreads) {
        const uint32_t kf = (uint32_t)(ord[p] >> 32);
        if (p > 0 && (uint32_t)(ord[p - 1] >> 32) == kf) continue;
        uint32_t re = p + 1;
        while (re < cnt && re - p <= (uint32_t)kFbSerial && (uint32_t)(ord[re] >> 32) == kf) ++re;
        if (re - p > (uint32_t)kFbSerial) continue;
        uint8_t *entry = entry_of(a, a.ent[(uint32_t)ord[p]]);
        Meta m;
        meta_load(entry, m);
        for (uint32_t q = p; q < re; ++q) {
            uint8_t *x;
            uint8_t idx;
            elem_at(a, (uint32_t)ord[q], x, idx, c);
            dispatch<SV>(TYPE, x, entry, idx, m, c);
            note_state(a, (uint32_t)ord[q], x);
        }
        meta_store(entry, m);
    }
    __syncthreads();
    for (uint32_t rs = 0; rs < cnt;) {  // longer runs: one at a time, by the whole workgroup
        const uint32_t key_f = (uint32_t)(ord[rs] >> 32);
        if (tid == 0) {
            uint32_t re = rs + 1;
            while (re < cnt && (uint32_t)(ord[re] >> 32) == key_f) ++re;
            loff = re;
            if (re - rs > (uint32_t)kFbSerial) meta_load(entry_of(a, a.ent[(uint32_t)ord[rs]]), sm);
        }
        __threadfence_block();
        __syncthreads();
        const uint32_t re = loff;
        if (re - rs <= (uint32_t)kFbSerial) {  // uniform: done by the serial tier
            __syncthreads();
            rs = re;
            continue;
        }
        uint8_t *entry = entry_of(a, a.ent[(uint32_t)ord[rs]]);
        for (uint32_t base = rs; base < re; base += kFbChunk) {
            uint32_t pending = 0;
#pragma unroll
            for (int j = 0; j < kFbPerThread; ++j)
                if (base + j * kFbThreads + tid < re) pending |= 1u << j;
            for (;;) {
                const Meta m = sm;
                int mine = kFbChunk;
#pragma unroll
                for (int j = kFbPerThread - 1; j >= 0; --j) {
                    if (!(pending >> j & 1u)) continue;
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, (uint32_t)ord[base + j * kFbThreads + tid], x, idx, c);
                    if (would_mutate(TYPE, x, m, c)) mine = j * kFbThreads + tid;
                }
                const int f = block_min(mine, red);
#pragma unroll
                for (int j = 0; j < kFbPerThread; ++j) {
                    const int pos = j * kFbThreads + tid;
                    if (!(pending >> j & 1u) || pos >= f) continue;
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, (uint32_t)ord[base + pos], x, idx, c);
                    Meta t = m;
                    dispatch<SV>(TYPE, x, entry, idx, t, c);
                    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
                    note_state(a, (uint32_t)ord[base + pos], x);
                    pending &= ~(1u << j);
                }
                __syncthreads();  // every read of the entry value precedes the mutation
                if (f < kFbChunk && (f % kFbThreads) == tid) {
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, (uint32_t)ord[base + f], x, idx, c);
                    Meta mm = m;
                    dispatch<SV>(TYPE, x, entry, idx, mm, c);
                    note_state(a, (uint32_t)ord[base + f], x);
                    pending &= ~(1u << (f / kFbThreads));
                    sm = mm;
                }
                __threadfence_block();
                __syncthreads();
                if (f >= kFbChunk) break;
            }
        }
        if (tid == 0) meta_store(entry, sm);
        __threadfence_block();
        __syncthreads();
        rs = re;
    }
}

// ------------------------------------------------------------------ small launches
// Launches of at most kSmallMax elements (the drop-in entry point's combined host batches, a
// few hundred to a few thousand elements) run in ONE workgroup and ONE kernel: the launch-wide
// latency of the multi-kernel engine (lookup, resolve, commit passes) is what bounds them, not
// bandwidth. The same rounds, with the workgroup's barriers instead of kernel boundaries:
//   lookup     every element (four per thread) as hermesKV.c:938-993; entry ids in LDS
//   round r    pending elements test would_mutate against their key's entry as it stands
//              (S_r); candidates lower their key's F in an LDS hash table (entry id -> F);
//              barrier; elements before F (or of keys without one) resolve on private copies of
//              S_r; barrier; F applies to the entry itself (S_r -> S_{r+1}); barrier.
//   after kSmallRounds rounds, keys still mutating are finished serially: the smallest pending
//   element of each key walks its key's pending elements in element order.
// Exactness is the engine's (would_mutate sound, checked through *error_flags).
constexpr int kSmallMax = (int)kSmallMaxElems;
constexpr int kSmallThreads = 1024;
constexpr int kSmallPer = kSmallMax / kSmallThreads;
constexpr int kSmallSlots = 2 * kSmallMax;
constexpr int kSmallRounds = 8;

__device__ __forceinline__ uint32_t small_slot(uint32_t *hkey, uint32_t e)
{
    uint32_t h = (e * 0x9E3779B1u) >> (32 - 13);  // kSmallSlots = 2^13
    for (;;) {
        const uint32_t old = atomicCAS(&hkey[h], kNone, e);
        if (old == kNone || old == e) return h;
        h = (h + 1) & (kSmallSlots - 1);
    }
}

// Where element i of a small launch lives. Uniform launches: n_batches batches of one type at
// `stride` elements each (hkv_batch_async). Mixed launches (the combining submit of the host entry
// point): batches of any type back to back, each described by a SmallBatch header, element i in
// the batch b with bstart[b] <= i < bstart[b + 1].
struct SmallView {
    uint8_t *x;
    uint8_t idx;      // op buffer index (local batches: < 256)
    int32_t pos;      // the element's position in its batch (INV batches run to 900 and beyond)
    int type;
    int b;
    bool live;
};

template <bool MIXED>
__device__ __forceinline__ SmallView small_at(const BatchArgs &a, const int32_t *bstart, const SmallBatch *bh,
                                              int i, Ctx &c)
{
    SmallView v;
    if (!MIXED) {
        const int32_t b = i / a.stride, idx = i - b * a.stride;
        v.x = a.elems + (int64_t)i * a.esz;
        v.idx = (uint8_t)idx;
        v.pos = idx;
        v.type = a.type;
        v.b = b;
        v.live = a.counts == nullptr || idx < a.counts[b];
        c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
        c.rws = a.rws ? a.rws + (int64_t)b * (a.rw_stride / a.g.op_size) : nullptr;
        c.rwo = a.rwo ? a.rwo + (int64_t)b * (a.rw_stride / a.g.op_size) : nullptr;
        return v;
    }
    int lo = 0, hi = a.n_batches;  // the last b with bstart[b] <= i
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (bstart[mid] <= i) lo = mid;
        else hi = mid;
    }
    const SmallBatch &h = bh[lo];
    const int idx = i - bstart[lo];
    v.x = a.dev_region + h.elem_off + (int64_t)idx * h.esz;
    v.idx = (uint8_t)idx;
    v.pos = idx;
    v.type = h.type;
    v.b = lo;
    v.live = true;
    c.g_membership = h.g_membership;
    c.w_ack_init = h.w_ack_init;
    c.rw = h.rw_off >= 0 ? a.dev_region + h.rw_off : nullptr;
    c.rws = nullptr;
    return v;
}

template <int SV, bool MIXED>
__global__ __launch_bounds__(kSmallThreads) void k_small(BatchArgs a)
{
    extern __shared__ uint32_t lds[];
    uint32_t *eid = lds;                          // [kSmallMax] entry id, kNone: skipped / missing / done
    uint32_t *hkey = eid + kSmallMax;             // [kSmallSlots] entry id of the slot
    uint32_t *hf = hkey + kSmallSlots;            // [kSmallSlots] the key's first candidate this round
    int32_t *ns = reinterpret_cast<int32_t *>(hf + kSmallSlots);      // [kSmallMax] per batch: last membership change
    uint16_t *slot = reinterpret_cast<uint16_t *>(ns + kSmallMax);    // [kSmallMax]
    __shared__ int32_t bstart[kSmallMaxBatches + 1];
    __shared__ SmallBatch bh[MIXED ? kSmallMaxBatches : 1];
    const int tid = threadIdx.x;
    const int n = (int)a.n;
    if (a.prof && tid == 0) a.prof[0] = wall_clock64();
    if (a.region_bytes) {  // staged in host memory: bring the launch's region into HBM (the
                           // dispatch's system-scope acquire drops any line an earlier launch left)
        const uint4 *src = reinterpret_cast<const uint4 *>(a.host_src);
        uint4 *dst = reinterpret_cast<uint4 *>(a.dev_region);
        for (uint64_t w = tid; w < a.region_bytes / 16; w += kSmallThreads) dst[w] = src[w];
        __threadfence_block();
    }
    for (int j = tid; j < kSmallSlots; j += kSmallThreads) {
        hkey[j] = kNone;
        hf[j] = kNone;
    }
    for (int j = tid; j < a.n_batches && j < kSmallMax; j += kSmallThreads) ns[j] = -1;
    if (MIXED) {
        __syncthreads();  // the copied-in headers
        const SmallBatch *g = reinterpret_cast<const SmallBatch *>(a.dev_region);
        for (int j = tid; j < a.n_batches; j += kSmallThreads) bh[j] = g[j];
        if (tid == 0) {
            int32_t acc = 0;
            for (int j = 0; j < a.n_batches; ++j) {
                bstart[j] = acc;
                acc += g[j].count;
            }
            bstart[a.n_batches] = acc;
        }
    }
    __syncthreads();
    if (a.prof && tid == 0) a.prof[1] = wall_clock64();
    Ctx c = make_ctx(a);
    // lookup (hermesKV.c:938-993); a hit reads the key and its meta S_0 from the log line at once
    Meta m0[kSmallPer];
    uint32_t pend = 0;  // bit k: element tid + k * kSmallThreads is pending
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int i = tid + k * kSmallThreads;
        if (i >= n) continue;
        uint32_t e = kNone;
        const SmallView v = small_at<MIXED>(a, bstart, bh, i, c);
        if (v.live) {
            const U64x2 h = *reinterpret_cast<const U64x2 *>(v.x);
            if (skip_elem_os(v.type, (uint8_t)h.b, (uint8_t)(h.b >> 8))) {
                if (v.type == kInvs) atomicMax(&ns[v.b], v.pos);   // hermes_skip_inv: the last one wins
            } else {
                const uint64_t key = h.a;
                const uint4 *bk = reinterpret_cast<const uint4 *>(a.index + ((key & 0xFFFFFFFFFFFFULL) & a.g.bkt_mask) * 64u);
                const uint4 q0 = bk[0], q1 = bk[1], q2 = bk[2], q3 = bk[3];
                const uint64_t sl[8] = {(uint64_t)q0.x | ((uint64_t)q0.y << 32), (uint64_t)q0.z | ((uint64_t)q0.w << 32),
                                        (uint64_t)q1.x | ((uint64_t)q1.y << 32), (uint64_t)q1.z | ((uint64_t)q1.w << 32),
                                        (uint64_t)q2.x | ((uint64_t)q2.y << 32), (uint64_t)q2.z | ((uint64_t)q2.w << 32),
                                        (uint64_t)q3.x | ((uint64_t)q3.y << 32), (uint64_t)q3.z | ((uint64_t)q3.w << 32)};
                const uint32_t tag = (uint32_t)(key >> 48);
                int hit = -1;
#pragma unroll
                for (int q = 7; q >= 0; --q)
                    if ((sl[q] & 1u) && ((uint32_t)(sl[q] >> 1) & 0x7FFFFFu) == tag) hit = q;
                if (hit >= 0) {
                    const uint64_t off = sl[hit] >> 24;
                    if (a.g.log_head - off < a.g.log_cap) {
                        const uint64_t phys = off & a.g.log_mask;
                        const U64x2 *ln = reinterpret_cast<const U64x2 *>(a.log + phys);
                        const U64x2 l0 = ln[0], l1 = ln[1], l2 = ln[2];  // key at 8, meta at 16..32
                        if (l0.b == key) {
                            e = (uint32_t)(phys / a.g.entry_unit);
                            m0[k].w4 = (uint32_t)l1.a;
                            m0[k].w5 = (uint32_t)(l1.a >> 32);
                            m0[k].ver = (uint32_t)l1.b;
                            m0[k].llw_cid = (uint8_t)(l1.b >> 32);
                            m0[k].llw_ver = (uint32_t)(l1.b >> 40) | ((uint32_t)(l2.a & 0xFFu) << 24);
                        }
                    }
                }
                if (e == kNone) v.x[9] = kMiss;
            }
        }
        eid[i] = e;
        if (e != kNone) {
            slot[i] = (uint16_t)small_slot(hkey, e);
            pend |= 1u << k;
        }
    }
    __syncthreads();
    if (a.prof && tid == 0) a.prof[2] = wall_clock64();
    bool any = true;
    for (int r = 0;; ++r) {
        any = __syncthreads_or(pend != 0);
        if (!any || r == kSmallRounds) break;
        // round 0 tests S_0 from the lookup's registers, later rounds the entry as it now stands
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {  // candidates of round r
            if (!(pend >> k & 1u)) continue;
            const int i = tid + k * kSmallThreads;
            const SmallView v = small_at<MIXED>(a, bstart, bh, i, c);
            if (r > 0) meta_load(entry_of(a, eid[i]), m0[k]);
            if (would_mutate(v.type, v.x, m0[k], c)) atomicMin(&hf[slot[i]], (uint32_t)i);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {  // before the key's candidate: S_r, unchanged
            if (!(pend >> k & 1u)) continue;
            const int i = tid + k * kSmallThreads;
            if (hf[slot[i]] <= (uint32_t)i) continue;
            const SmallView v = small_at<MIXED>(a, bstart, bh, i, c);
            Meta t = m0[k];
            dispatch<SV>(v.type, v.x, entry_of(a, eid[i]), v.idx, t, c);
            if (a.error_flags && !meta_equal(t, m0[k])) atomicOr(a.error_flags, 1u);
            pend &= ~(1u << k);
        }
        __threadfence_block();
        __syncthreads();  // every read of S_r precedes the mutation
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {  // the candidate: S_r -> S_{r+1}
            if (!(pend >> k & 1u)) continue;
            const int i = tid + k * kSmallThreads;
            if (hf[slot[i]] != (uint32_t)i) continue;
            const SmallView v = small_at<MIXED>(a, bstart, bh, i, c);
            uint8_t *entry = entry_of(a, eid[i]);
            Meta m = m0[k];
            dispatch<SV>(v.type, v.x, entry, v.idx, m, c);
            meta_store(entry, m);
            hf[slot[i]] = kNone;
            pend &= ~(1u << k);
        }
        __threadfence_block();
    }
    if (a.prof && tid == 0) a.prof[3] = wall_clock64();
    if (any) {  // keys that kept mutating: the first pending element of each key finishes it in order
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {
            const int i = tid + k * kSmallThreads;
            if (i < n && !(pend >> k & 1u)) eid[i] = kNone;   // done: no longer part of any key's walk
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k)
            if (pend >> k & 1u) atomicMin(&hf[slot[tid + k * kSmallThreads]], (uint32_t)(tid + k * kSmallThreads));
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSmallPer; ++k) {
            const int i = tid + k * kSmallThreads;
            if (!(pend >> k & 1u) || hf[slot[i]] != (uint32_t)i) continue;
            const uint32_t e = eid[i];
            uint8_t *entry = entry_of(a, e);
            Meta m;
            meta_load(entry, m);
            for (int j = i; j < n; ++j) {
                if (eid[j] != e) continue;
                const SmallView v = small_at<MIXED>(a, bstart, bh, j, c);
                dispatch<SV>(v.type, v.x, entry, v.idx, m, c);
            }
            meta_store(entry, m);
        }
    }
    // hermes_skip_dispatcher's *node_suspected = value[0] of each INV batch's last membership change
    if (MIXED) {
        __syncthreads();
        for (int b = tid; b < a.n_batches; b += kSmallThreads) {
            const SmallBatch &h = bh[b];
            if (h.type == kInvs && h.ns_off >= 0 && ns[b] >= 0)
                *reinterpret_cast<int32_t *>(a.dev_region + h.ns_off) =
                    a.dev_region[h.elem_off + (int64_t)ns[b] * h.esz + kOpValueOff];
        }
    } else if (a.type == kInvs && a.node_suspected) {
        __syncthreads();
        for (int b = tid; b < a.n_batches; b += kSmallThreads)
            if (ns[b] >= 0) a.node_suspected[b] = a.elems[((int64_t)b * a.stride + ns[b]) * a.esz + kOpValueOff];
    }
    if (!MIXED && a.state_out) {
        __syncthreads();
        for (int i = tid; i < n; i += kSmallThreads) a.state_out[i] = a.elems[(int64_t)i * a.esz + 9];
    }
    if (a.prof && tid == 0) a.prof[4] = wall_clock64();
    if (a.region_bytes) {  // results back to the host staging, then the completion flag
        __threadfence_block();  // one workgroup wrote the region: its CU's caches see it
        __syncthreads();
        // System-scope stores (sc0 sc1) write through L2 to the host, and a thread's vmcnt counts
        // them done once they are visible there: each thread waits for its own, then the flag
        // follows the barrier. A __threadfence_system() instead writes back all of L2, every entry
        // this launch dirtied included (~10 us); plain stores would sit in L2 and reach the host
        // later, over the set's next use.
        const unsigned long long *src = reinterpret_cast<const unsigned long long *>(a.dev_region);
        unsigned long long *dst = reinterpret_cast<unsigned long long *>(a.host_dst);
        for (uint64_t w = tid; w < a.region_bytes / 8; w += kSmallThreads)
            __hip_atomic_store(dst + w, src[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) __hip_atomic_store(a.done_flag, a.done_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (a.prof && tid == 0) a.prof[5] = wall_clock64();
}

int launch_small(const BatchArgs &a0, hipStream_t s)
{
    // HKV_SMALL_PROF=N: every N-th launch records its phase timestamps and prints the running
    // average (debug; synchronises the stream)
    static const int prof_every = getenv("HKV_SMALL_PROF") ? atoi(getenv("HKV_SMALL_PROF")) : 0;
    static unsigned long long *prof = nullptr;
    static long prof_n = 0;
    static double prof_sum[5] = {0, 0, 0, 0, 0};
    BatchArgs a = a0;
    a.prof = nullptr;
    const bool sample = prof_every > 0 && (++prof_n % prof_every) == 0;
    if (sample) {
        if (!prof && hipHostMalloc((void **)&prof, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -3;
        a.prof = prof;
    }
    const size_t lds = (size_t)4 * (2 * kSmallMax + 2 * kSmallSlots) + (size_t)2 * kSmallMax;
    auto setup = [&](const void *f, int k) {
        static bool done[6] = {false, false, false, false, false, false};
        if (!done[k]) {
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return false;
            done[k] = true;
        }
        return true;
    };
#define HKV_SMALL(V, M)                                                                   \
    do {                                                                                  \
        if (!setup((const void *)k_small<V, M>, (V == 31 ? 0 : V == 287 ? 1 : 2) + (M ? 3 : 0))) return -3; \
        hipLaunchKernelGGL((k_small<V, M>), dim3(1), dim3(kSmallThreads), lds, s, a);        \
    } while (0)
    const bool mixed = a.hdr != nullptr;
    if (a.g.st_value == 31) {
        if (mixed) HKV_SMALL(31, true);
        else HKV_SMALL(31, false);
    } else if (a.g.st_value == 287) {
        if (mixed) HKV_SMALL(287, true);
        else HKV_SMALL(287, false);
    } else {
        if (mixed) HKV_SMALL(0, true);
        else HKV_SMALL(0, false);
    }
#undef HKV_SMALL
    if (sample) {
        hipStreamSynchronize(s);
        static long k = 0;
        ++k;
        for (int p = 0; p < 5; ++p) prof_sum[p] += (double)(prof[p + 1] - prof[p]) * 10.0 / 1000.0;  // 100 MHz ticks -> us
        fprintf(stderr, "[hkv] k_small phases (us, avg of %ld): copy-in+init %.2f lookup %.2f rounds %.2f fallback %.2f copy-out %.2f\n", k,
                prof_sum[0] / k, prof_sum[1] / k, prof_sum[2] / k, prof_sum[3] / k, prof_sum[4] / k);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------ partitioned host launches
// The combining submit's launches on 64-B entries (HostPartLaunch, hkv_internal.h). Workgroup g
// takes partition g of every batch: all elements of its keys, in element order, and no other
// workgroup's. So the k_small rounds run per workgroup with no communication at all, and a
// launch's latency stays that of one partition however many callers it combines:
//   load    its slice of each batch straight from the callers' pinned buffers into LDS (one
//           thread per element, four 16-B loads), with each element's position in its batch
//   lookup  one thread per element (hermesKV.c:938-993): bucket, tag probe, wrap, the whole
//           64-B entry line into LDS; the elements of one entry share the copy of its first one
//   rounds  k_small's element-order rounds on the LDS copies (candidates lower their key's F,
//           elements before F resolve on private metas, F applies to the shared copy); after
//           kHpRounds the first pending element of a key finishes it serially
//   store   changed entry lines back to HBM (the 48 bytes after the MICA key), every element back
//           to its caller's buffer with system-scope stores, then flags[g] = seq
// A completing ACK marks its read_write_ops slot in the caller's pinned copy directly (one byte,
// system scope); node_suspected is the host's (hermes_skip_inv depends on the element alone).
constexpr int kHpThreads = kPartCap;          // one element per thread
constexpr int kHpSlots = 2 * kPartCap;        // entry-id hash slots
constexpr int kHpRounds = 8;
constexpr int kHpWords = kPartCap * 8 / kHpThreads;   // 8-byte words of elements per thread (esz <= 64)

__device__ __forceinline__ uint32_t hp_slot(uint32_t *hkey, uint32_t e)
{
    uint32_t h = (e * 0x9E3779B1u) >> (32 - 9);   // kHpSlots = 2^9
    for (;;) {
        const uint32_t old = atomicCAS(&hkey[h], kNone, e);
        if (old == kNone || old == e) return h;
        h = (h + 1) & (kHpSlots - 1);
    }
}

// Host memory the callers rewrite between launches is read with system-scope (uncached) loads: the
// serving kernel (k_hserve) outlives many launches, so no kernel start invalidates stale lines for it.
__device__ __forceinline__ uint64_t ld_sys64(const void *p)
{
    return __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys32(const void *p)
{
    return __hip_atomic_load(reinterpret_cast<const uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys_u16(const uint16_t *p)   // 2-byte aligned
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    return (ld_sys32(reinterpret_cast<const void *>(a & ~(uintptr_t)3)) >> (8 * (a & 2))) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t ld_sys_u8(const uint8_t *p)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    return (ld_sys32(reinterpret_cast<const void *>(a & ~(uintptr_t)3)) >> (8 * (a & 3))) & 0xFFu;
}

// exec_ack's read_write_ops completion of slot `done` in a caller's pinned copy (hermesKV.c:660-668).
// pre: bytes 8..11 of slot pre_slot, read ahead (hp_rw_ahead); a slot of another opcode keeps its state,
// so it is not written at all.
__device__ __forceinline__ void hp_complete_rw(uint8_t *rw, int done, uint32_t op_size, uint32_t pre = 0, int pre_slot = -1)
{
    uint8_t *w = rw + (size_t)done * op_size;
    const uint8_t oc = done == pre_slot ? (uint8_t)pre : (uint8_t)ld_sys_u8(w + 8);
    if (oc != kOpGet && oc != kOpPut && oc != kOpRmw) return;
    const uint8_t ns = oc == kOpGet ? kNew : oc == kOpPut ? kPutComplete : kRmwComplete;
    __hip_atomic_store(w + 9, ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// An ACK's read_write_ops slot is the entry's op-buffer index (exec_ack): its opcode is read right after
// the lookup, so the read overlaps the rounds instead of following them -- from the opcodes the caller
// staged in device memory (rwo), else from byte 8 of the slot in the pinned copy (over PCIe)
__device__ __forceinline__ void hp_rw_ahead(const uint8_t *rw, const uint8_t *rwo, const uint8_t *line, uint32_t op_size,
                                            uint32_t &pre, int &pre_slot)
{
    Meta m;
    meta_load(line, m);
    const int ob = m_obi(m);
    if (ob == kObiEmpty) return;
    pre = rwo ? ld_sys_u8(rwo + ob) : ld_sys_u8(rw + (size_t)ob * op_size + 8);
    pre_slot = ob;
}

// The LDS of one partition's work (both kernels)
struct HpLds {
    uint4 sel[kPartCap * 4];        // elements (64 B per slot, esz used)
    uint4 sln[kPartCap * 4];        // entry lines; a key's elements use its first slot's
    HostPartHdr bh[kPartMaxB];
    int32_t base[kPartMaxB + 1], lo[kPartMaxB], wbase[kPartMaxB + 1];
    uint16_t prow[2][kPartMaxB];    // part[g][*], part[g + 1][*]
    uint32_t hkey[kHpSlots], hmin[kHpSlots], hf[kHpSlots];
    uint8_t sdirty[kPartCap], spend[kPartCap];
    uint16_t shs[kPartCap];
    int cmd;
    int32_t nb;
    int32_t nm;                     // k_hserve: launches taken in this pass
    int32_t sb[kPartMaxB + 1];      // ... their first batches (sb[nm]: all of them)
};

// The batch ranges of partition g (bh, prow in LDS): per-batch slot and word offsets (one wave)
__device__ __forceinline__ void hp_scan(HpLds &L, int nb)
{
    const int tid = threadIdx.x;
    if (tid < 64) {
        int32_t c = 0, cw = 0;
        if (tid < nb) {
            const int32_t a0 = L.prow[0][tid], a1 = L.prow[1][tid];
            L.lo[tid] = a0;
            c = a1 - a0;
            cw = c * (L.bh[tid].esz / 8);
        }
        int32_t incl = c, inclw = cw;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t v = __shfl_up(incl, d, 64), vw = __shfl_up(inclw, d, 64);
            if (tid >= d) {
                incl += v;
                inclw += vw;
            }
        }
        if (tid < nb) {
            L.base[tid + 1] = incl;
            L.wbase[tid + 1] = inclw;
        }
        if (tid == 0) {
            L.base[0] = 0;
            L.wbase[0] = 0;
        }
    }
}

__device__ __forceinline__ int hp_batch_of(const int32_t *offs, int nb, int v)   // the last b with offs[b] <= v
{
    int l = 0, h = nb;
    while (h - l > 1) {
        const int mid = (l + h) >> 1;
        if (offs[mid] <= v) l = mid;
        else h = mid;
    }
    return l;
}

// Partition g of one launch whose headers and ranges are in L (after hp_scan and a barrier):
// load, lookup, rounds, store back, then flags[g] = seq. See the section comment.
__device__ void hp_partition(const HostPartCommon &p, HpLds &L, int g, int nb, uint32_t seq)
{
    const int tid = threadIdx.x;
    const bool pr = p.prof && g == 0 && tid == 0;
    if (pr) p.prof[1] = wall_clock64();
    for (int j = tid; j < kHpSlots; j += kHpThreads) {
        L.hkey[j] = kNone;
        L.hmin[j] = kNone;
        L.hf[j] = kNone;
    }
    const int P = L.base[nb];   // at most kPartCap (the host's check)
    const int s = tid;
    const bool live = s < P;
    const int b = live ? hp_batch_of(L.base, nb, s) : 0;
    const HostPartHdr &hd = L.bh[b];
    const int64_t j = live ? (int64_t)L.lo[b] + (s - L.base[b]) : 0;
    // the elements: each batch's slice is contiguous in its caller's buffer, so consecutive lanes
    // copy consecutive 8-byte words of it (coalesced requests over PCIe), all loads in flight at once
    const uint16_t pos = live ? (uint16_t)ld_sys_u16(reinterpret_cast<const uint16_t *>(hd.pos) + j) : (uint16_t)0;
    {
        const int TW = L.wbase[nb];   // at most kPartCap * 8
        uint64_t w[kHpWords];
        int dst[kHpWords];
#pragma unroll
        for (int r = 0; r < kHpWords; ++r) {
            const int idx = tid + r * kHpThreads;
            dst[r] = -1;
            w[r] = 0;
            if (idx < TW) {
                const int l = hp_batch_of(L.wbase, nb, idx);
                const int per = L.bh[l].esz / 8, wi = idx - L.wbase[l];
                w[r] = ld_sys64(reinterpret_cast<const uint8_t *>(L.bh[l].elems) + ((int64_t)L.lo[l] * L.bh[l].esz + 8 * wi));
                dst[r] = (L.base[l] + wi / per) * 8 + wi % per;
            }
        }
#pragma unroll
        for (int r = 0; r < kHpWords; ++r)
            if (dst[r] >= 0) reinterpret_cast<uint64_t *>(L.sel)[dst[r]] = w[r];
    }
    __syncthreads();
    uint8_t *x = reinterpret_cast<uint8_t *>(&L.sel[s * 4]);
    Ctx c;
    c.g = p.g;
    c.g_membership = hd.g_membership;
    c.w_ack_init = hd.w_ack_init;
    c.rw = reinterpret_cast<uint8_t *>(hd.rw);
    c.rws = nullptr;
    c.rw_done = nullptr;
    c.vc = nullptr;
    const int type = hd.type;
    // lookup (hermesKV.c:938-993)
    uint32_t e = kNone;
    uint64_t phys = 0;
    if (live && !skip_elem_os(type, x[8], x[9])) {
        const uint64_t key = *reinterpret_cast<const uint64_t *>(x);
        const uint4 *bk = reinterpret_cast<const uint4 *>(p.index + ((key & 0xFFFFFFFFFFFFULL) & p.g.bkt_mask) * 64u);
        const uint4 q0 = bk[0], q1 = bk[1], q2 = bk[2], q3 = bk[3];
        const uint64_t sl[8] = {(uint64_t)q0.x | ((uint64_t)q0.y << 32), (uint64_t)q0.z | ((uint64_t)q0.w << 32),
                                (uint64_t)q1.x | ((uint64_t)q1.y << 32), (uint64_t)q1.z | ((uint64_t)q1.w << 32),
                                (uint64_t)q2.x | ((uint64_t)q2.y << 32), (uint64_t)q2.z | ((uint64_t)q2.w << 32),
                                (uint64_t)q3.x | ((uint64_t)q3.y << 32), (uint64_t)q3.z | ((uint64_t)q3.w << 32)};
        const uint32_t tag = (uint32_t)(key >> 48);
        int hit = -1;
#pragma unroll
        for (int q = 7; q >= 0; --q)
            if ((sl[q] & 1u) && ((uint32_t)(sl[q] >> 1) & 0x7FFFFFu) == tag) hit = q;
        if (hit >= 0) {
            const uint64_t off = sl[hit] >> 24;
            if (p.g.log_head - off < p.g.log_cap) {
                phys = off & p.g.log_mask;
                const uint4 *ln = reinterpret_cast<const uint4 *>(p.log + phys);
                const uint4 l0 = ln[0], l1 = ln[1], l2 = ln[2], l3 = ln[3];
                if (((uint64_t)l0.z | ((uint64_t)l0.w << 32)) == key) {
                    e = (uint32_t)(phys / p.g.entry_unit);
                    L.sln[s * 4 + 0] = l0;
                    L.sln[s * 4 + 1] = l1;
                    L.sln[s * 4 + 2] = l2;
                    L.sln[s * 4 + 3] = l3;
                }
            }
        }
        if (e == kNone) x[9] = kMiss;
    }
    uint32_t rw_pre = 0;
    int rw_pre_slot = -1;
    if (type == kAcks && hd.rw && e != kNone)
        hp_rw_ahead(reinterpret_cast<const uint8_t *>(hd.rw), reinterpret_cast<const uint8_t *>(hd.rwo),
                    reinterpret_cast<const uint8_t *>(&L.sln[s * 4]), p.g.op_size, rw_pre, rw_pre_slot);
    if (pr) p.prof[2] = wall_clock64();
    uint32_t hs = 0;
    if (e != kNone) {
        hs = hp_slot(L.hkey, e);
        atomicMin(&L.hmin[hs], (uint32_t)s);
    }
    __syncthreads();
    const int cs = e != kNone ? (int)L.hmin[hs] : s;   // the slot whose line copy the key's elements share
    uint8_t *ent = reinterpret_cast<uint8_t *>(&L.sln[cs * 4]);
    const uint8_t idx = (uint8_t)pos;
    bool pend = e != kNone, dirty = false;
    int done = -1;
    c.rw_done = type == kAcks ? &done : nullptr;
    bool any = true;
    for (int r = 0;; ++r) {
        any = __syncthreads_or(pend);
        if (!any || r == kHpRounds) break;
        Meta m;
        if (pend) {
            meta_load(ent, m);
            if (would_mutate(type, x, m, c)) atomicMin(&L.hf[hs], (uint32_t)s);
        }
        __syncthreads();
        if (pend && L.hf[hs] > (uint32_t)s) {   // before the key's candidate: S_r, unchanged
            Meta t = m;
            dispatch<31>(type, x, ent, idx, t, c);
            if (p.error_flags && !meta_equal(t, m)) atomicOr(p.error_flags, 1u);
            pend = false;
        }
        __syncthreads();   // every read of S_r precedes the mutation
        if (pend && L.hf[hs] == (uint32_t)s) {  // the candidate: S_r -> S_{r+1}
            dispatch<31>(type, x, ent, idx, m, c);
            meta_store(ent, m);
            L.hf[hs] = kNone;
            dirty = true;
            pend = false;
        }
    }
    if (any) {  // keys that kept mutating: each key's first pending element finishes it in order
        L.spend[s] = pend;
        L.shs[s] = (uint16_t)hs;
        __syncthreads();   // (every F of the last round was reset to kNone when it applied)
        if (pend) atomicMin(&L.hf[hs], (uint32_t)s);
        __syncthreads();
        if (pend && L.hf[hs] == (uint32_t)s) {
            Meta m;
            meta_load(ent, m);
            for (int k = s; k < P; ++k) {
                if (!L.spend[k] || L.shs[k] != (uint16_t)hs) continue;   // hash slot = entry = key
                uint8_t *xk = reinterpret_cast<uint8_t *>(&L.sel[k * 4]);
                Ctx ck = c;
                int dk = -1;
                ck.rw_done = type == kAcks ? &dk : nullptr;
                const int l = hp_batch_of(L.base, nb, k);   // the element's own batch
                ck.g_membership = L.bh[l].g_membership;
                ck.w_ack_init = L.bh[l].w_ack_init;
                ck.rw = reinterpret_cast<uint8_t *>(L.bh[l].rw);
                const int64_t jk = (int64_t)L.lo[l] + (k - L.base[l]);
                const uint8_t ik = (uint8_t)ld_sys_u16(reinterpret_cast<const uint16_t *>(L.bh[l].pos) + jk);
                dispatch<31>(L.bh[l].type, xk, ent, ik, m, ck);
                if (dk >= 0 && ck.rw) hp_complete_rw(ck.rw, dk, p.g.op_size);
            }
            meta_store(ent, m);
            dirty = true;
        }
    }
    // a completing ACK of the rounds marks its read_write_ops slot (exec_ack left it to us)
    if (done >= 0 && c.rw) hp_complete_rw(c.rw, done, p.g.op_size, rw_pre, rw_pre_slot);
    if (pr) p.prof[3] = wall_clock64();
    L.sdirty[s] = 0;
    __syncthreads();
    if (dirty) L.sdirty[cs] = 1;
    __syncthreads();
    // the changed entry lines back to HBM (bytes 16..63: the MICA key never changes)
    if (live && e != kNone && cs == s && L.sdirty[s]) {
        uint4 *dst = reinterpret_cast<uint4 *>(p.log + phys);
        dst[1] = L.sln[s * 4 + 1];
        dst[2] = L.sln[s * 4 + 2];
        dst[3] = L.sln[s * 4 + 3];
    }
    // every element back to its caller (consecutive lanes, consecutive words), then the flag (see
    // k_small's copy-out)
    for (int w = tid; w < L.wbase[nb]; w += kHpThreads) {
        const int l = hp_batch_of(L.wbase, nb, w);
        const int per = L.bh[l].esz / 8, wi = w - L.wbase[l];
        const uint64_t ob = L.bh[l].out ? L.bh[l].out : L.bh[l].elems;
        unsigned long long *d = reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(ob) +
                                                                       (int64_t)L.lo[l] * L.bh[l].esz) + wi;
        __hip_atomic_store(d, (unsigned long long)reinterpret_cast<const uint64_t *>(L.sel)[(L.base[l] + wi / per) * 8 + wi % per],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (pr) p.prof[4] = wall_clock64();
    if (tid == 0) {
        __hip_atomic_store(p.flags + g, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// One launch, its headers in the kernel arguments
__global__ __launch_bounds__(kHpThreads) void k_hpart(HostPartLaunch p)
{
    __shared__ HpLds L;
    const int tid = threadIdx.x, g = blockIdx.x, nb = p.n_batches;
    if (p.c.prof && g == 0 && tid == 0) p.c.prof[0] = wall_clock64();
    if (tid < nb) {
        L.bh[tid] = p.hdr[tid];
        L.prow[0][tid] = p.part[g][tid];
        L.prow[1][tid] = p.part[g + 1][tid];
    }
    __syncthreads();
    hp_scan(L, nb);
    __syncthreads();
    hp_partition(p.c, L, g, nb, p.seq);
}

// The serving kernel: workgroup g takes partition g of every launch published in the pinned ring,
// in order, from p.start[g] on -- no kernel launch per combined batch. Thread 0 polls the next
// slot's seq (uncached, backing off with s_sleep); the workgroup leaves when the host raises *stop,
// after idle_ticks without a launch, or once life_ticks have passed (then between launches), and
// records p.epoch in exited[g] so the host knows to launch a new server for what it publishes next.
__global__ __launch_bounds__(kHpThreads) void k_hserve(HostServeLaunch p)
{
    __shared__ HpLds L;
    const int tid = threadIdx.x, g = blockIdx.x;
    uint32_t next = p.start[g];
    const uint64_t t0 = wall_clock64();
    uint64_t idle_since = t0;
    for (;;) {
        const HostRingSlot *sl = p.ring + (next % (uint32_t)p.ring_n);
        constexpr int HW = (int)(sizeof(HostPartHdr) / 8);
        if (p.spec) {   // thread 0 polls alone; the scan below runs beside the first launch's header loads
            if (tid == 0) {
                int cmd = 0;
                for (;;) {
                    if (ld_sys32(&sl->seq) == next) {
                        cmd = 1;
                        break;
                    }
                    const uint64_t now = wall_clock64();
                    if (ld_sys32(p.stop) || now - idle_since > p.idle_ticks || now - t0 > p.life_ticks) {
                        cmd = 2;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
                L.cmd = cmd;
            }
            __syncthreads();
            if (L.cmd == 2) break;
        }
        if (tid < 64) {
            int cmd = 1;
            if (!p.spec) {
                if (tid == 0) {
                    for (;;) {
                        if (ld_sys32(&sl->seq) == next) {
                            cmd = 1;
                            break;
                        }
                        const uint64_t now = wall_clock64();
                        if (ld_sys32(p.stop) || now - idle_since > p.idle_ticks || now - t0 > p.life_ticks) {
                            cmd = 2;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(4);
                    }
                    L.cmd = cmd;
                }
                cmd = __shfl(cmd, 0);
            }
            if (cmd == 1) {   // this launch and the ones published after it while their batches fit: lane k
                              // reads launch next + k's seq and batch count, all loads in flight together
                const HostRingSlot *sk = p.ring + ((next + (uint32_t)tid) % (uint32_t)p.ring_n);
                const bool in = tid < p.merge;
                const uint32_t sq = in && tid > 0 ? ld_sys32(&sk->seq) : next;
                // the count only once the seq is seen (the host writes a slot's contents before its seq)
                const int nbk = in && sq == next + (uint32_t)tid ? (int)ld_sys32(&sk->n_batches) : 0;
                int incl = nbk;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int v = __shfl_up(incl, d, 64);
                    if (tid >= d) incl += v;
                }
                const bool ok = in && sq == next + (uint32_t)tid && (tid == 0 || incl <= kPartMaxB);
                const uint64_t stop = __ballot(!ok);   // the first launch not taken (lane 0 always is)
                const int nm = stop ? __ffsll((long long)stop) - 1 : 64;
                if (tid < nm) L.sb[tid + 1] = incl;
                if (tid == 0) {
                    L.sb[0] = 0;
                    L.nm = nm;
                }
            }
        } else if (p.spec) {   // launch `next` is published: all kPartMaxB of its headers and rows g, g + 1
            const int u = tid - 64;
            if (u < HW * kPartMaxB) {
                reinterpret_cast<uint64_t *>(L.bh)[u] = ld_sys64(reinterpret_cast<const uint64_t *>(sl->hdr) + u);
            } else if (u < HW * kPartMaxB + 2 * kPartMaxB) {
                const int q = u - HW * kPartMaxB, row = q / kPartMaxB, b = q % kPartMaxB;
                L.prow[row][b] = (uint16_t)ld_sys_u16(&sl->part[g + row][b]);
            }
        }
        __syncthreads();
        if (L.cmd == 2) break;
        const bool pr = p.c.prof && g == 0 && tid == 0;
        const uint64_t t_seen = pr ? wall_clock64() : 0;
        const int nm = L.nm, nbt = L.sb[nm];
        // the headers (8 bytes per thread) and part rows g and g + 1 (2 bytes per thread) of every launch
        // taken, its batches after the previous launch's (p.spec: the first launch's came beside the scan)
        const int bfrom = p.spec ? L.sb[1] : 0;
        if (bfrom < nbt) {
            if (tid >= HW * bfrom && tid < HW * nbt) {
                const int b = tid / HW;
                int k = 0;
                while (L.sb[k + 1] <= b) ++k;
                const HostRingSlot *sk = p.ring + ((next + (uint32_t)k) % (uint32_t)p.ring_n);
                reinterpret_cast<uint64_t *>(L.bh)[tid] =
                    ld_sys64(reinterpret_cast<const uint64_t *>(sk->hdr) + (tid - HW * L.sb[k]));
            } else if (tid >= 128 && tid < 128 + 2 * nbt) {
                const int q = tid - 128, row = q / nbt, b = q % nbt;
                if (b >= bfrom) {
                    int k = 0;
                    while (L.sb[k + 1] <= b) ++k;
                    const HostRingSlot *sk = p.ring + ((next + (uint32_t)k) % (uint32_t)p.ring_n);
                    L.prow[row][b] = (uint16_t)ld_sys_u16(&sk->part[g + row][b - L.sb[k]]);
                }
            }
            __syncthreads();
        }
        if (tid == 0) {   // partition g of the taken launches within kPartCap elements (the first always is)
            int k = 1, tot = 0;
            for (int b = 0; b < L.sb[1]; ++b) tot += L.prow[1][b] - L.prow[0][b];
            for (; k < nm; ++k) {
                int c = 0;
                for (int b = L.sb[k]; b < L.sb[k + 1]; ++b) c += L.prow[1][b] - L.prow[0][b];
                if (tot + c > kPartCap) break;
                tot += c;
            }
            L.nm = k;
        }
        __syncthreads();
        const int taken = L.nm, nb = L.sb[taken];
        hp_scan(L, nb);
        __syncthreads();
        hp_partition(p.c, L, g, nb, next + (uint32_t)taken - 1u);
        if (pr) {   // HKV_PART_PROF: workgroup 0's phase sums over the launches it served (debug)
            unsigned long long *q = p.c.prof;
            q[8] += t_seen - idle_since;
            q[9] += q[1] - t_seen;
            q[10] += q[2] - q[1];
            q[11] += q[3] - q[2];
            q[12] += q[4] - q[3];
            q[13] += 1;
        }
        next += (uint32_t)taken;
        idle_since = wall_clock64();
        __syncthreads();   // LDS reuse by the next launch
    }
    if (tid == 0) __hip_atomic_store(p.exited + g, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static unsigned long long *g_serve_prof = nullptr;
static void serve_prof_print()
{
    const unsigned long long *q = g_serve_prof;
    const double n = q[13] ? (double)q[13] : 1.0;
    fprintf(stderr, "[hkv] k_hserve phases (us, avg of %llu launches, workgroup 0): wait %.2f headers %.2f load+lookup %.2f "
            "rounds %.2f store %.2f\n", q[13], q[8] / n / 100.0, q[9] / n / 100.0, q[10] / n / 100.0, q[11] / n / 100.0,
            q[12] / n / 100.0);
}

int launch_host_serve(const HostServeLaunch &sl0, hipStream_t s)
{
    HostServeLaunch sl = sl0;
    if (getenv("HKV_PART_PROF")) {   // (debug) phase sums, printed at exit
        if (!g_serve_prof) {
            if (hipHostMalloc((void **)&g_serve_prof, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -3;
            memset(g_serve_prof, 0, 256);
            atexit(serve_prof_print);
        }
        sl.c.prof = g_serve_prof;
    }
    hipLaunchKernelGGL(k_hserve, dim3(kPartG), dim3(kHpThreads), 0, s, sl);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_host_part(const HostPartLaunch &pl, hipStream_t s)
{
    if (pl.n_batches <= 0 || pl.n_batches > kPartMaxB || pl.c.g.entry_size != 64 || pl.c.g.st_value != 31) return -1;
    // HKV_PART_PROF=N: every N-th launch records workgroup 0's phase timestamps and prints the running
    // average (debug; synchronises the stream)
    static const int prof_every = getenv("HKV_PART_PROF") ? atoi(getenv("HKV_PART_PROF")) : 0;
    static unsigned long long *prof = nullptr;
    static long prof_n = 0, k = 0;
    static double sum[4] = {0, 0, 0, 0};
    HostPartLaunch p = pl;
    p.c.prof = nullptr;
    const bool sample = prof_every > 0 && (++prof_n % prof_every) == 0;
    if (sample) {
        if (!prof && hipHostMalloc((void **)&prof, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -3;
        p.c.prof = prof;
    }
    hipLaunchKernelGGL(k_hpart, dim3(kPartG), dim3(kHpThreads), 0, s, p);
    if (sample) {
        hipStreamSynchronize(s);
        ++k;
        for (int i = 0; i < 4; ++i) sum[i] += (double)(prof[i + 1] - prof[i]) * 10.0 / 1000.0;  // 100 MHz ticks -> us
        fprintf(stderr, "[hkv] k_hpart phases (us, avg of %ld): headers %.2f load+lookup %.2f rounds %.2f store %.2f\n", k,
                sum[0] / k, sum[1] / k, sum[2] / k, sum[3] / k);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

__global__ void k_node_suspected(const uint8_t *elems, const int32_t *ns_idx, int32_t *out, int32_t n_batches,
                                 int32_t stride, int32_t esz, const int32_t *offsets)
{
    const int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_batches) return;
    const int32_t i = ns_idx[b];
    const int64_t base = offsets ? (int64_t)offsets[b] : (int64_t)b * stride;
    if (i >= 0) out[b] = elems[(base + i) * esz + kOpValueOff];
}

// ------------------------------------------------------------------ host side
static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t batch_scratch_bytes(int64_t cap, uint32_t entry_size)
{
    return align256(4 * (size_t)cap) * 3 + align256((size_t)cap) + align256(16 * (size_t)cap) * 2 + 256 +
           align256(2 * (size_t)cap) +
           align256((size_t)entry_size * (size_t)cap);
}

void batch_carve(BatchLaunch &bl, uint8_t *base, int64_t cap, uint32_t entry_size)
{
    uint8_t *p = base;
    auto take = [&](size_t bytes) {
        uint8_t *r = p;
        p += align256(bytes);
        return r;
    };
    bl.ent = reinterpret_cast<uint32_t *>(take(4 * (size_t)cap));
    bl.st = take((size_t)cap);
    bl.mem = reinterpret_cast<unsigned long long *>(take(16 * (size_t)cap));
    bl.fbl = reinterpret_cast<uint32_t *>(take(4 * (size_t)cap));
    bl.pf = reinterpret_cast<uint32_t *>(take(4 * (size_t)cap));
    bl.shadow = take((size_t)entry_size * (size_t)cap);
    bl.ctr = reinterpret_cast<uint32_t *>(take(256));
    bl.hx = reinterpret_cast<uint64_t *>(take(16 * (size_t)cap));
    bl.fk = reinterpret_cast<uint16_t *>(take(2 * (size_t)cap));
    bl.cap = (uint32_t)cap;
}

size_t batch_fw_words(uint64_t log_cap) { return (size_t)(log_cap >> 6); }

uint32_t batch_max_epoch() { return (1u << 29) - 1; }

int launch_batch(BatchLaunch &bl, hipStream_t s)
{
    const int64_t n = bl.n;
    if (n <= 0) return 0;
    BatchArgs a;
    a.elems = bl.elems;
    a.counts = bl.counts;
    a.offsets = bl.offsets;
    a.state_out = (bl.type == kLocal || bl.type == kLocalAfterMemb) ? bl.state_out : nullptr;
    a.opc = bl.type == kLocal ? bl.opcode_in : nullptr;
    a.patch = nullptr;
    a.hx = nullptr;
    a.fk = bl.type == kLocal && bl.g.rmw_enabled && bl.esz > 64 ? bl.fk : nullptr;   // (k_resolve0_direct's launches)
    a.ack_out = bl.type == kInvs || (bl.type == kAcks && bl.n_rows > 0) ? bl.ack_out : nullptr;
    a.ack_out_size = bl.ack_out_size;
    a.n_rows = bl.n_rows;
    a.skip_row = bl.skip_row;
    a.row_stride = bl.row_stride;
    a.rws = bl.type == kAcks ? bl.rw_state : nullptr;
    a.rwo = bl.type == kAcks ? bl.opcode_in : nullptr;
#ifdef HKV_DEBUG_MODES
    static const int dbg_env = getenv("HKV_DBG") ? atoi(getenv("HKV_DBG")) : 0;
#else
    constexpr int dbg_env = 0;   // the default build cannot skip work (tools/dbg_modes.sh builds its own)
#endif
    a.dbg = dbg_env;
    static const int check_unique_env = getenv("HKV_CHECK_UNIQUE") ? atoi(getenv("HKV_CHECK_UNIQUE")) : 0;
    a.check_unique = check_unique_env;
    a.index = bl.index;
    a.log = bl.log;
    a.rw = bl.rw;
    a.ns_idx = bl.ns_idx;
    a.fw = bl.fw;
    a.fw_mask = (uint32_t)((bl.g.log_cap >> 6) - 1);
    a.ent = bl.ent;
    a.st = bl.st;
    a.mem = bl.mem;
    a.fbl = bl.fbl;
    a.pf = bl.pf;
    a.shadow = bl.shadow;
    a.ctr = bl.ctr;
    a.error_flags = bl.error_flags;
    a.g = bl.g;
    a.n = n;
    a.rw_stride = bl.rw_stride;
    a.stride = bl.stride;
    a.esz = bl.esz;
    a.type = bl.type;
    a.rtag0 = bl.epoch << 3;
    a.ltag = (uint8_t)(bl.epoch % 255u + 1u);
    a.rounds = rounds_for(bl.type, bl.g.rmw_enabled != 0);
    a.fx = bl.fx;
    a.fy = bl.fy;
    a.inv_direct = bl.type == kInvs && !bl.g.rmw_enabled && n < kInvDirectMax;
    a.ft = bl.ft;
    a.ack_direct = bl.type == kAcks && !bl.g.rmw_enabled && n < (int64_t)kNone;
    a.g_membership = bl.g_membership;
    a.w_ack_init = bl.w_ack_init;
    a.node_suspected = bl.node_suspected;
    a.n_batches = bl.n_batches;
    a.host_src = bl.host_src;
    a.host_dst = bl.host_dst;
    a.dev_region = bl.dev_region;
    a.region_bytes = bl.region_bytes;
    a.done_flag = bl.done_flag;
    a.done_value = bl.done_value;
    a.hdr = bl.hdr;
    const unsigned grid = (unsigned)((n + 255) / 256);
    const unsigned cgrid = (unsigned)((n + 256 * kCandPer - 1) / (256 * kCandPer));
    const bool big = bl.esz > 64;
    // big ops: local and ACK launches resolve round 0 in place (measured at cfg3: local 1.26 ->
    // 1.05 ms, ACK 0.69 -> 0.55 ms); INV launches keep the LDS slab (0.40 vs 0.52 ms in place)
    const bool big_direct = bl.type != kInvs;
    const unsigned rgrid = (unsigned)(big ? (n + 127) / 128 : grid);
    const size_t rlds = (size_t)(big ? 128 : 256) * (size_t)bl.esz;
    const bool small = (bl.path == kPathSmall || (bl.path == kPathAuto && n <= kSmallMax)) && n <= kSmallMax;
    if (bl.region_bytes && !small) return -1;  // host-staged launches are small ones
    // local batches without RMWs in the default layout: the direct path (k_local_pre, k_local_fused)
    const bool local_direct = bl.type == kLocal && !bl.g.rmw_enabled && bl.esz == 56 && bl.g.st_value == 31 &&
                              bl.g.entry_size == 64 && !bl.offsets;
    // big local launches on the rounds engine (configs[2]): k_lookup reads the patches, k_resolve0_direct writes
    // the patched ops (patch_in_resolve, see there): values of at most 320 bytes, the op's pad after its value
    // within its last 8-byte word
    const uint32_t vend = (uint32_t)kOpValueOff + bl.g.st_value;
    const bool patch_in_resolve = bl.patch && !small && !local_direct && bl.type == kLocal && big && big_direct &&
                                  !bl.offsets && bl.g.st_value != 31 && bl.g.st_value <= 320 && bl.esz % 8 == 0 &&
                                  (uint32_t)bl.esz >= vend && (uint32_t)bl.esz <= vend + 8;
    if (patch_in_resolve) {
        a.patch = bl.patch;
        a.hx = bl.hx;
    } else if (bl.patch && (small || !local_direct)) {  // the other paths take the patches as op writes first
        hipLaunchKernelGGL(k_apply_patch, dim3(grid), dim3(256), 0, s, bl.elems, bl.patch, n, bl.esz, bl.g.st_value);
    } else if (bl.patch) {
        a.patch = bl.patch;
    }
    if (small) {
        if (launch_small(a, s)) return -3;
        return 0;                              // node_suspected written by the kernel
    } else if (local_direct) {
        hipLaunchKernelGGL(k_local_pre<kPreHead>, dim3((unsigned)((n + kPreElems - 1) / kPreElems)), dim3(kPreThreads),
                           0, s, a);
        hipLaunchKernelGGL((k_local_fused<2, kLfWaves>), dim3((unsigned)((n + 32 * kLfWaves - 1) / (32 * kLfWaves))),
                           dim3(64 * kLfWaves), 0, s, a);
        // the waiting elements' count is on the device: enough workgroups for the rounds after a
        // membership change (configs[4]: ~100 K elements of keys a failed peer left INVALID), which
        // return at once when there are few
        hipLaunchKernelGGL(k_local_deferred, dim3(128u), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_commit_w, dim3((unsigned)((n + 4 * kCwElems - 1) / (4 * kCwElems))), dim3(256), 0, s, a);
    } else if (bl.n_rows > 0 && bl.unique) {  // HKV_BATCH_ROWS: one pass over positions of all rows
        // two positions per lane group, 32 per wave
        const unsigned lgrid = (unsigned)((n + kLfElems - 1) / kLfElems);
        // elements of 16 B (ACKs without RMWs) keep one chunk each in LDS, others four
        if (bl.type == kInvs) {
            if (bl.n_rows <= 2) hipLaunchKernelGGL((k_unique_rows<kInvs, 2, 4>), dim3(lgrid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_unique_rows<kInvs, 8, 4>), dim3(lgrid), dim3(64), 0, s, a);
        } else if (bl.esz <= 16) {
            if (bl.n_rows <= 2) hipLaunchKernelGGL((k_unique_rows<kAcks, 2, 1>), dim3(lgrid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_unique_rows<kAcks, 8, 1>), dim3(lgrid), dim3(64), 0, s, a);
        } else {
            if (bl.n_rows <= 2) hipLaunchKernelGGL((k_unique_rows<kAcks, 2, 4>), dim3(lgrid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_unique_rows<kAcks, 8, 4>), dim3(lgrid), dim3(64), 0, s, a);
        }
    } else if (bl.unique && (bl.type == kInvs || bl.type == kAcks)) {  // one pass: every key has one element
        // in-place unique pass (big-entry ACKs, other geometries): one element per lane group
        const unsigned ugrid1 = (unsigned)((n + 63) / 64);
#define HKV_UNIQUE(T)                                                                                  \
    do {                                                                                               \
        if (bl.g.st_value == 31) hipLaunchKernelGGL((k_unique<T, 31, 1>), dim3(ugrid1), dim3(256), 0, s, a); \
        else if (bl.g.st_value == 287) hipLaunchKernelGGL((k_unique<T, 287, 1>), dim3(ugrid1), dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((k_unique<T, 0, 1>), dim3(ugrid1), dim3(256), 0, s, a);             \
    } while (0)
        const bool lds64 = bl.g.st_value == 31 && bl.g.entry_size == 64 && bl.esz <= 64;
        const bool lds_big = bl.type == kInvs && bl.g.st_value == 287 && bl.g.entry_size == 320 && bl.esz <= 320;
        if (a.ack_out && !(lds64 || lds_big)) return -1;   // only the LDS-staged passes write the ACKs
        if (lds64) {
            // 64-B entries: the LDS-staged pass, one element per lane group (16 per wave). Same box, INV phase
            // per step (gpurun_out/r04m, r04t): 72-77 us at 1 element per lane group, 78-80 at 2, 91 at 4
            const unsigned g1 = (unsigned)((n + 15) / 16);
            if (bl.type == kInvs) hipLaunchKernelGGL((k_unique_lds<kInvs, 1>), dim3(g1), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_unique_lds<kAcks, 1>), dim3(g1), dim3(64), 0, s, a);
        } else if (lds_big) {
            // big-object INVs, whose raises copy 287-B values: staged through LDS (cfg3: 460 -> 326 us per
            // round). ACKs touch the header and the meta only, so they stay in place (LDS-staged: 110 -> 191 us)
            hipLaunchKernelGGL(k_unique_big<kInvs>, dim3((unsigned)((n + kUbElems - 1) / kUbElems)), dim3(64), 0, s, a);
        } else if (bl.type == kInvs) HKV_UNIQUE(kInvs);
        else HKV_UNIQUE(kAcks);
#undef HKV_UNIQUE
    } else if (bl.type == kVals) {             // one pass (see k_lookup)
        // one element per lane group. Same box, VAL batch per step (gpurun_out/r04m, r04u): 49.6-50.2 us at 1,
        // 52.3-53.9 at 2, 57 at 4
        hipLaunchKernelGGL(k_lookup<1>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, a, (int64_t)0, n);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    } else {
    // The head split pays off where one launch piles many candidates onto a few keys: local
    // batches under Zipf. A replica's INVs and ACKs carry at most one write per key and peer per
    // round, so those launches take one pass (their launch-sized head took ~9 us at cfg2).
    const bool split = bl.type == kLocal || bl.type == kLocalAfterMemb;
    const int64_t head = split && n > kLookupHead ? kLookupHead : n;
    // one element per lane group in the other lookups (configs[2] 0.627-0.635 against 0.620-0.622 G ops/s at
    // two, same box, gpurun_out/r04v)
    hipLaunchKernelGGL(k_lookup<1>, dim3((unsigned)((head + 63) / 64)), dim3(256), 0, s, a, (int64_t)0, head);
    if (n > head) hipLaunchKernelGGL(k_lookup<1>, dim3((unsigned)((n - head + 63) / 64)), dim3(256), 0, s, a, head, n);
    if (a.ack_direct) {
        hipLaunchKernelGGL(k_ack_resolve, dim3(grid), dim3(256), 0, s, a);
    } else if (a.inv_direct) {
        hipLaunchKernelGGL(k_inv_resolve, dim3(grid), dim3(256), 0, s, a, (int64_t)0, n);
        if (bl.g.st_value == 31) hipLaunchKernelGGL((k_inv_commit<31>), dim3(grid), dim3(256), 0, s, a);
        else if (bl.g.st_value == 287) hipLaunchKernelGGL((k_inv_commit<287>), dim3(grid), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_inv_commit<0>), dim3(grid), dim3(256), 0, s, a);
    } else {
#define HKV_ROUNDS(T, V)                                                                          \
    do {                                                                                          \
        if (big && rlds > 64 * 1024 &&                                                            \
            hipFuncSetAttribute((const void *)k_resolve0<T, V, 128>,                              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)rlds) != hipSuccess) \
            return -3;                                                                            \
        if (big && big_direct) hipLaunchKernelGGL((k_resolve0_direct<T, V>), dim3(grid), dim3(256), 0, s, a); \
        else if (big) hipLaunchKernelGGL((k_resolve0<T, V, 128>), dim3(rgrid), dim3(128), rlds, s, a); \
        else hipLaunchKernelGGL((k_resolve0<T, V, 256>), dim3(rgrid), dim3(256), rlds, s, a);     \
        for (int r = 1; r <= a.rounds; ++r) {                                                     \
            hipLaunchKernelGGL((k_cand<T>), dim3(cgrid), dim3(256), 0, s, a, r);                  \
            hipLaunchKernelGGL((k_resolve<T, V>), dim3(grid), dim3(256), V == 31 ? 256 * bl.esz : 0, s, a, r); \
        }                                                                                         \
        hipLaunchKernelGGL((k_commit<V>), dim3(grid), dim3(256), 0, s, a);                         \
        if (a.rounds > 0) hipLaunchKernelGGL((k_fb_exec<T, V>), dim3(256), dim3(kFbThreads), 0, s, a); \
    } while (0)
#define HKV_ROUNDS_SV(T)                                      \
    do {                                                      \
        if (bl.g.st_value == 31) HKV_ROUNDS(T, 31);           \
        else if (bl.g.st_value == 287) HKV_ROUNDS(T, 287);    \
        else HKV_ROUNDS(T, 0);                                \
    } while (0)
    switch (bl.type) {
    case kLocal: HKV_ROUNDS_SV(kLocal); break;
    case kLocalAfterMemb: HKV_ROUNDS_SV(kLocalAfterMemb); break;
    case kInvs: HKV_ROUNDS_SV(kInvs); break;
    case kAcks: HKV_ROUNDS_SV(kAcks); break;
    default: HKV_ROUNDS_SV(kVals); break;
    }
#undef HKV_ROUNDS_SV
#undef HKV_ROUNDS
    }
    }
    if (hipGetLastError() != hipSuccess) return -3;
    if (bl.type == kInvs && bl.ns_idx && bl.node_suspected) {
        hipLaunchKernelGGL(k_node_suspected, dim3((bl.n_batches + 255) / 256), dim3(256), 0, s, bl.elems, bl.ns_idx,
                           bl.node_suspected, bl.n_batches, bl.stride, bl.esz, bl.offsets);
        if (hipGetLastError() != hipSuccess) return -4;
    }
    return 0;
}

}  // namespace hkv
