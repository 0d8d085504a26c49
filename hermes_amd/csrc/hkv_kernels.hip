// hkv_kernels.hip -- CDNA4 (gfx950) kernels of the HermesKV batch path.
//
// One launch of hkv_batch_async runs three device stages over the concatenated batches:
//
//   1. k_lookup        one lane per element, in element order: skip test (hermesKV.c:709-769),
//                      bucket probe over the 8 slots of one 64-B bucket (hermesKV.c:952-975),
//                      wrap test, 8-B key compare against the log entry (hermesKV.c:977-993).
//                      Misses get ST_MISS in byte 9 right here. Hits emit (entry id, element).
//   2. radix sort      stable sort of (entry id, element) pairs: every entry's elements become
//                      one contiguous segment, still in concatenation order.
//   3. k_segment_exec  the first lane of each segment owns that entry: it loads the object meta
//                      once, runs the segment's elements through the Hermes state machine
//                      (hkv_exec.h) in order, and stores the meta once.
//
// The index is immutable after populate (no inserts on the hot path), so stage 1 is
// embarrassingly parallel; stage 3 is exact because elements of one entry never run on two
// lanes. Populate (spacetime.c:32-68 / mica.c:78-146) uses the same shape: hash, sort by
// bucket, one owner lane per bucket replays the MICA slot rules, entries are written in
// parallel.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "hkv_exec.h"
#include "hkv_internal.h"

namespace hkv {

// ------------------------------------------------------------------ CityHash128, 4-byte keys
// city.c:85-400 restricted to the CityMurmur short-string path that mica_gen_keys uses.
__device__ __forceinline__ uint64_t ch_mix16(uint64_t u, uint64_t v)
{
    const uint64_t mul = 0x9ddfea08eb382d69ULL;
    uint64_t a = (u ^ v) * mul;
    a ^= a >> 47;
    uint64_t b = (v ^ a) * mul;
    b ^= b >> 47;
    return b * mul;
}

__device__ __forceinline__ void cityhash128_u32(uint32_t id, uint64_t &first, uint64_t &second)
{
    const uint64_t k0 = 0xc3a5c85c97cb3127ULL, k1 = 0xb492b66fbe98f273ULL;
    uint64_t a = k0 * k1;
    a = (a ^ (a >> 47)) * k1;                                  // ShiftMix(seed.lo * k1) * k1
    uint64_t c = k1 * k1 + ch_mix16(4u + ((uint64_t)id << 3), (uint64_t)id);  // HashLen0to16(len 4)
    uint64_t d = (a + c) ^ ((a + c) >> 47);                    // ShiftMix(a + c), len < 8
    uint64_t aa = ch_mix16(a, c);
    uint64_t bb = ch_mix16(d, k1);
    first = aa ^ bb;
    second = ch_mix16(bb, aa);
}

__global__ void k_hash_ids(const uint32_t *__restrict__ ids, uint64_t *__restrict__ out, int64_t n)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t f, s;
    cityhash128_u32(ids[i], f, s);
    out[i] = s;
}

// ------------------------------------------------------------------ batch stage 1: lookup
struct LookupArgs {
    uint8_t *elems;
    const int32_t *counts;
    const uint8_t *index;
    const uint8_t *log;
    uint32_t *keys;
    uint32_t *vals;
    int32_t *ns_idx;      // per batch: last ST_OP_MEMBERSHIP_CHANGE element (INV batches)
    Geometry g;
    int64_t n;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint32_t skip_key;
};

// Four lanes per element: each lane reads 16 bytes (two slots) of the element's 64-byte
// bucket, so one load instruction covers a whole bucket line per element and the vector
// memory pipeline sees one request per bucket instead of four. Slots are searched in the
// reference's order (first tag match wins, hermesKV.c:954-975).
constexpr int kLookupPerBlock = 64;
__global__ __launch_bounds__(256) void k_lookup(LookupArgs a)
{
    const int q = threadIdx.x & 3;
    const int lane = threadIdx.x & 63;
    const int64_t gi = (int64_t)blockIdx.x * kLookupPerBlock + (threadIdx.x >> 2);
    const bool in = gi < a.n;
    int32_t b = 0, idx = 0;
    uint8_t *x = nullptr;
    uint64_t key = 0;
    int probe = 0;
    if (in && q == 0) {
        b = (int32_t)(gi / a.stride);
        idx = (int32_t)(gi - (int64_t)b * a.stride);
        if (a.counts == nullptr || idx < a.counts[b]) {
            x = a.elems + gi * a.esz;
            key = ld64(x);
            const uint32_t w2 = ld32(x + 8);
            if (skip_elem_os(a.type, (uint8_t)w2, (uint8_t)(w2 >> 8))) {
                if (a.type == kInvs && a.ns_idx) atomicMax(&a.ns_idx[b], idx);
            } else {
                probe = 1;
            }
        }
    }
    probe = __shfl(probe, 0, 4);
    key = __shfl(key, 0, 4);
    uint64_t s0 = 0, s1 = 0;
    if (probe) {
        const uint4 v = reinterpret_cast<const uint4 *>(a.index + ((key & 0xFFFFFFFFFFFFULL) & a.g.bkt_mask) * 64u)[q];
        s0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
        s1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    const uint32_t tag = (uint32_t)(key >> 48);
    const bool m0 = probe && (s0 & 1u) && ((uint32_t)(s0 >> 1) & 0x7FFFFFu) == tag;
    const bool m1 = probe && (s1 & 1u) && ((uint32_t)(s1 >> 1) & 0x7FFFFFu) == tag;
    const int gbase = lane & ~3;
    const uint32_t g0 = (uint32_t)(__ballot(m0) >> gbase) & 0xFu;
    const uint32_t g1 = (uint32_t)(__ballot(m1) >> gbase) & 0xFu;
    uint32_t order = 0;  // bit 2*l + j: slot 2*l + j matches
#pragma unroll
    for (int l = 0; l < 4; ++l) order |= ((g0 >> l) & 1u) << (2 * l) | ((g1 >> l) & 1u) << (2 * l + 1);
    const int first = order ? __ffs(order) - 1 : 0;
    const uint64_t off = __shfl((first & 1) ? (s1 >> 24) : (s0 >> 24), first >> 1, 4);
    if (!in || q != 0) return;
    uint32_t key_out = a.skip_key;
    if (probe) {
        if (order && a.g.log_head - off < a.g.log_cap) {
            const uint64_t phys = off & a.g.log_mask;
            if (ld64(a.log + phys + 8) == key) key_out = (uint32_t)(phys / a.g.entry_unit);
        }
        if (key_out == a.skip_key) x[9] = kMiss;
    }
    a.keys[gi] = key_out;
    a.vals[gi] = (uint32_t)gi;
}

// ------------------------------------------------------------------ batch stage 3: segments
// After the sort every log entry touched by the launch owns one contiguous segment of the
// sorted order, whose elements are in concatenation order. A segment of at most kShortSeg
// elements is applied serially by its first lane (k_segment_exec). Longer ones (hot keys)
// go through chip-wide rounds:
//
//   round r, for every long segment not yet finished: every element after the previous round's
//     mutation asks would_mutate() against the segment's meta S_r; the first such sorted
//     position F_r is found with a wave-segmented min and one atomicMin per wavefront and
//     segment (round 0 inside k_segment_exec, later rounds in k_round_cand); k_round_apply
//     then snapshots the entry (image of S_r), applies element F_r alone with the serial exec
//     function and records S_{r+1}. A segment whose round finds no candidate is finished: S_r
//     is its final meta, stored to the entry.
//   k_round_resolve: every other element of a long segment lies strictly between two
//     consecutive mutations F_{r-1} < pos < F_r and is therefore a non-candidate under S_r:
//     it runs the serial exec function on a private copy of S_r against the snapshot of S_r
//     (so GETs read the value as it was at their point of the order) -- all in parallel.
//   k_long_exec: segments that still mutate after kMaxRounds rounds finish on one workgroup
//     from F_{R-1}+1 with S_R (first-candidate passes, see below).
//
// Exactness only needs would_mutate() to be sound (a false answer guarantees the exec
// function leaves the meta unchanged); every element still runs the reference's exec
// function once, against the meta the sequential order gives it. Checked by bit 0 of
// *error_flags, which a non-candidate that did change its private copy would raise.
//
// F_r lives in a 64-bit word tagged with the launch's epoch ((~epoch << 32) | position), so
// it needs no per-launch initialisation: a newer epoch's tag is smaller, atomicMin replaces
// stale words, and a word whose tag is not this launch's reads as "no candidate".
constexpr int kShortSeg = 4;
constexpr int kMaxRounds = 4;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint8_t kNotDone = 0xFF;

struct SegState {            // per long segment, all in device scratch
    uint32_t *start;         // [cap] first sorted position
    uint32_t *end;           // [cap] one past the last sorted position
    uint32_t *count;         // [2]: [1] = segments left to k_long_exec
    uint32_t *fallback;      // [cap] slots of segments left to k_long_exec
    const uint32_t *lidx;    // [n] long-segment heads at or before each sorted position (scan)
    uint32_t *seg_of;        // [n] long-segment slot of every sorted position (kNone if short/skip)
    uint64_t *hdr;           // [n] header bytes 8..15 of long-segment elements, sorted order
    Meta *meta;              // [cap][kMaxRounds + 1]
    unsigned long long *mut; // [cap][kMaxRounds] epoch-tagged F_r (sorted position)
    uint8_t *done;           // [cap] round whose meta is final, kNotDone while mutating
    uint8_t *snap;           // [cap][kMaxRounds] entry images of S_r
    uint32_t cap;
    uint32_t epoch;          // this launch, >= 1
};

struct SegmentArgs {
    SegState st;
    uint8_t *elems;
    uint8_t *log;
    uint8_t *rw;
    const uint32_t *keys;
    const uint32_t *vals;
    unsigned int *error_flags;
    Geometry g;
    int64_t n;
    int64_t rw_stride;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint32_t skip_key;
    uint8_t g_membership;
    uint8_t w_ack_init;
    int32_t rounds;          // chip-wide rounds before k_long_exec (<= kMaxRounds)
};

// Rounds per batch type: how many mutations a hot key usually sees in one launch. A local
// batch has one write per key (later writes stall on its WRITE state), a VAL batch validates
// once, an ACK batch sets one ack bit and completes; INVs with rising timestamps keep mutating.
__host__ __device__ constexpr int rounds_for(int type)
{
    return type == kLocal || type == kVals ? 2 : type == kAcks ? 3 : kMaxRounds;
}

__device__ __forceinline__ Ctx make_ctx(const SegmentArgs &a)
{
    Ctx c;
    c.g = a.g;
    c.g_membership = a.g_membership;
    c.w_ack_init = a.w_ack_init;
    c.rw = nullptr;
    return c;
}

__device__ __forceinline__ void elem_at(const SegmentArgs &a, uint32_t gi, uint8_t *&x, uint8_t &idx, Ctx &c)
{
    const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
    idx = (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride);
    c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
    x = a.elems + (int64_t)gi * a.esz;
}

__device__ __forceinline__ uint8_t *entry_of(const SegmentArgs &a, uint32_t key)
{
    return a.log + (uint64_t)key * a.g.entry_unit;
}

__device__ __forceinline__ uint64_t mut_tag(const SegmentArgs &a) { return (uint64_t)(~a.st.epoch) << 32; }

__device__ __forceinline__ uint32_t mut_read(const SegmentArgs &a, uint32_t s, int r)
{
    const uint64_t v = a.st.mut[(size_t)s * kMaxRounds + r];
    return (v >> 32) == (uint32_t)~a.st.epoch ? (uint32_t)v : kNone;
}

// Candidates of one segment are consecutive among a wavefront's candidate lanes (sorted
// order): only the first of each run issues the atomicMin, and only if it would lower F_r.
__device__ __forceinline__ void offer_candidate(const SegmentArgs &a, bool cand, uint32_t s, int r, uint32_t p)
{
    const int lane = threadIdx.x & 63;
    const unsigned long long cm = __ballot(cand);
    const unsigned long long below = cm & ((1ull << lane) - 1ull);
    const int prev_lane = below ? 63 - __clzll((long long)below) : -1;
    const uint32_t prev_s = __shfl(s, prev_lane < 0 ? lane : prev_lane, 64);
    if (cand && (prev_lane < 0 || prev_s != s)) {
        unsigned long long *f = &a.st.mut[(size_t)s * kMaxRounds + r];
        const unsigned long long v = mut_tag(a) | p;
        if (v < __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(f, v);
    }
}

// Serial tier, long-segment registration and round 0's candidate search.
//
// Short segments (at most kShortSeg elements) run on LDS copies: the workgroup covers BP sorted
// positions; the head lane of each short segment marks the positions it owns (its segment may
// run up to kShortSeg-1 positions past the range), the ops and the heads' log entries are
// copied in with eight lanes per object (one memory request per object line instead of one
// per field), every head applies its segment with the serial exec functions on LDS, and the
// owned ops and entries are copied back the same way.
//
// A position is in a long segment iff some window of kShortSeg+1 equal sorted keys covers it;
// its slot is its segment's rank among long heads (the scan in lidx), so registration needs
// no atomics. Every long position caches its header for later rounds and offers itself as
// round 0's candidate against the entry's meta as stored (S_0).
template <int TYPE, int SV, int BP>
__global__ __launch_bounds__(256) void k_segment_exec(SegmentArgs a)
{
    extern __shared__ uint64_t smem[];
    constexpr int kSpan = BP + kShortSeg - 1;              // staged positions
    constexpr int kKeys = BP + 2 * kShortSeg;              // sorted keys [P0 - kShortSeg, P0 + BP + kShortSeg)
    uint32_t *ks = reinterpret_cast<uint32_t *>(smem);
    uint8_t *own = reinterpret_cast<uint8_t *>(ks + kKeys); // [kSpan] owned by a short head here
    uint8_t *hflag = own + ((kSpan + 7) & ~7);              // [BP] short head at this position
    uint64_t *ops = reinterpret_cast<uint64_t *>(hflag + BP);
    const uint32_t esz = (uint32_t)a.esz, ew = esz / 8u, entw = a.g.entry_size / 8u;
    uint64_t *ents = ops + (size_t)kSpan * ew;             // [BP] entries of short heads
    const int t = threadIdx.x;
    const int64_t P0 = (int64_t)blockIdx.x * BP;
    if (blockIdx.x == 0 && t == 0) a.st.count[1] = 0;  // fallback list of this launch (read after the rounds)
    for (int i = t; i < kKeys; i += blockDim.x) {
        const int64_t q = P0 - kShortSeg + i;
        ks[i] = (q >= 0 && q < a.n) ? a.keys[q] : a.skip_key;
    }
    for (int i = t; i < kSpan; i += blockDim.x) own[i] = 0;
    __syncthreads();
    const int64_t p = P0 + t;
    const bool valid = p < a.n;
    const uint32_t key = valid ? ks[t + kShortSeg] : a.skip_key;
    const bool live = key != a.skip_key;
    const bool head = live && ks[t + kShortSeg - 1] != key;
    bool in_long = false;
    if (live) {
#pragma unroll
        for (int j = 0; j <= kShortSeg; ++j)  // window [p - j, p - j + kShortSeg]
            in_long |= ks[t + kShortSeg - j] == key && ks[t + 2 * kShortSeg - j] == key;
    }
    const uint32_t s = in_long ? a.st.lidx[p] - 1 : kNone;
    int L = 0;
    bool cand = false;
    if (in_long) {
        uint8_t *entry = entry_of(a, key);
        Meta m0;
        meta_load(entry, m0);
        if (head) {
            a.st.start[s] = (uint32_t)p;
            a.st.meta[(size_t)s * (kMaxRounds + 1)] = m0;
            a.st.done[s] = kNotDone;
        }
        if (ks[t + kShortSeg + 1] != key) a.st.end[s] = (uint32_t)(p + 1);
        const uint64_t h = ld64(a.elems + (int64_t)a.vals[p] * esz + 8);
        a.st.hdr[p] = h;
        uint64_t hdr[2] = {0, h};
        Ctx c = make_ctx(a);
        cand = would_mutate(TYPE, reinterpret_cast<const uint8_t *>(hdr), m0, c);
    } else if (head) {
        L = 1;
        while (L < kShortSeg && ks[t + kShortSeg + L] == key) ++L;
        for (int j = 0; j < L; ++j) own[t + j] = 1;
    }
    if (valid) a.st.seg_of[p] = s;
    offer_candidate(a, cand, s, 0, (uint32_t)p);
    hflag[t] = L ? 1 : 0;
    __syncthreads();
    const int g = t >> 3, l8 = t & 7, ng = BP >> 3;
    for (int i = g; i < kSpan; i += ng) {
        if (!own[i]) continue;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(a.elems + (int64_t)a.vals[P0 + i] * esz);
        for (uint32_t w = l8; w < ew; w += 8) ops[(size_t)i * ew + w] = src[w];
    }
    for (int h = g; h < BP; h += ng) {
        if (!hflag[h]) continue;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(entry_of(a, ks[h + kShortSeg]));
        for (uint32_t w = l8; w < entw; w += 8) ents[(size_t)h * entw + w] = src[w];
    }
    __syncthreads();
    if (L) {
        uint8_t *entry = reinterpret_cast<uint8_t *>(ents + (size_t)t * entw);
        Meta mm;
        meta_load(entry, mm);
        Ctx c = make_ctx(a);
        for (int j = 0; j < L; ++j) {
            const uint32_t gi = a.vals[p + j];
            const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
            const uint8_t idx = (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride);
            c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
            dispatch<SV>(TYPE, reinterpret_cast<uint8_t *>(ops + (size_t)(t + j) * ew), entry, idx, mm, c);
        }
        meta_store(entry, mm);
    }
    __syncthreads();
    for (int i = g; i < kSpan; i += ng) {
        if (!own[i]) continue;
        uint64_t *dst = reinterpret_cast<uint64_t *>(a.elems + (int64_t)a.vals[P0 + i] * esz);
        for (uint32_t w = l8; w < ew; w += 8) dst[w] = ops[(size_t)i * ew + w];
    }
    for (int h = g; h < BP; h += ng) {
        if (!hflag[h]) continue;
        uint64_t *dst = reinterpret_cast<uint64_t *>(entry_of(a, ks[h + kShortSeg]));
        for (uint32_t w = l8; w < entw; w += 8) dst[w] = ents[(size_t)h * entw + w];
    }
}

template <int BP>
static size_t segment_exec_lds(uint32_t esz, uint32_t entry_size)
{
    const int span = BP + kShortSeg - 1;
    return (size_t)4 * (BP + 2 * kShortSeg) + (size_t)((span + 7) & ~7) + BP + (size_t)span * esz +
           (size_t)BP * entry_size;
}

// round r >= 1: candidates after F_{r-1}, against S_r, from the cached headers
template <int TYPE>
__global__ __launch_bounds__(256) void k_round_cand(SegmentArgs a, int r)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s = p < a.n ? a.st.seg_of[p] : kNone;
    bool cand = false;
    if (s != kNone && a.st.done[s] == kNotDone && (uint32_t)p > mut_read(a, s, r - 1)) {
        uint64_t hdr[2] = {0, a.st.hdr[p]};
        const Meta m = a.st.meta[(size_t)s * (kMaxRounds + 1) + r];
        Ctx c = make_ctx(a);
        cand = would_mutate(TYPE, reinterpret_cast<const uint8_t *>(hdr), m, c);
    }
    offer_candidate(a, cand, s, r, (uint32_t)p);
}

template <int TYPE, int SV>
__global__ __launch_bounds__(256) void k_round_apply(SegmentArgs a, int r)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.st.lidx[a.n - 1] || a.st.done[s] != kNotDone) return;
    uint8_t *entry = entry_of(a, a.keys[a.st.start[s]]);
    const uint32_t f = mut_read(a, s, r);
    Meta m = a.st.meta[(size_t)s * (kMaxRounds + 1) + r];
    if (f == kNone) {
        a.st.done[s] = (uint8_t)r;
        meta_store(entry, m);
        return;
    }
    // image of S_r for the elements resolved before F_r (entries are 8-byte aligned)
    const uint64_t *src = reinterpret_cast<const uint64_t *>(entry);
    uint64_t *dst = reinterpret_cast<uint64_t *>(a.st.snap + ((size_t)s * kMaxRounds + r) * a.g.entry_size);
    for (uint32_t w = 0; w < a.g.entry_size / 8; ++w) dst[w] = src[w];
    Ctx c = make_ctx(a);
    uint8_t *x;
    uint8_t idx;
    elem_at(a, a.vals[f], x, idx, c);
    dispatch<SV>(TYPE, x, entry, idx, m, c);
    a.st.meta[(size_t)s * (kMaxRounds + 1) + r + 1] = m;
    if (r == a.rounds - 1) a.st.fallback[atomicAdd(&a.st.count[1], 1u)] = s;
}

template <int TYPE, int SV>
__global__ __launch_bounds__(256) void k_round_resolve(SegmentArgs a)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n) return;
    const uint32_t s = a.st.seg_of[p];
    if (s == kNone) return;
    const uint8_t done = a.st.done[s];
    int r = 0;
    uint32_t f = kNone;
    for (; r < a.rounds; ++r) {
        f = (done != kNotDone && r == done) ? kNone : mut_read(a, s, r);
        if ((uint32_t)p <= f) break;
    }
    if (r == a.rounds || (uint32_t)p == f) return;  // left to k_long_exec, or applied by a round
    const uint8_t *img = f == kNone ? entry_of(a, a.keys[p])
                                    : a.st.snap + ((size_t)s * kMaxRounds + r) * a.g.entry_size;
    const Meta m = a.st.meta[(size_t)s * (kMaxRounds + 1) + r];
    Meta t = m;
    Ctx c = make_ctx(a);
    uint8_t *x;
    uint8_t idx;
    elem_at(a, a.vals[p], x, idx, c);
    // non-candidates only read the entry (the value), so the snapshot stands in for it
    dispatch<SV>(TYPE, x, const_cast<uint8_t *>(img), idx, t, c);
    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
}

template <int NT>
__device__ __forceinline__ int block_min(int v, int *lds)
{
    for (int o = 32; o > 0; o >>= 1) {
        int u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = lds[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) r = lds[w] < r ? lds[w] : r;
    return r;
}

// Fallback for segments still mutating after kMaxRounds rounds: one 1024-thread workgroup per
// segment continues from F_{R-1}+1 with S_R, in chunks of kLongChunk elements: repeat
// {block min of the first candidate f; resolve elements before f on private copies; barrier;
// f applies on the shared meta; barrier} until a chunk has no candidate left.
constexpr int kLongThreads = 1024;
constexpr int kPerThread = 8;
constexpr int kLongChunk = kLongThreads * kPerThread;

template <int TYPE, int SV>
__global__ __launch_bounds__(kLongThreads) void k_long_exec(SegmentArgs a)
{
    __shared__ Meta sm;
    __shared__ int red[kLongThreads / 64];
    const int tid = threadIdx.x;
    const uint32_t nfb = a.st.count[1];
    Ctx c = make_ctx(a);
    for (uint32_t i = blockIdx.x; i < nfb; i += gridDim.x) {
        const uint32_t s = a.st.fallback[i];
        const uint32_t first = mut_read(a, s, a.rounds - 1) + 1, end = a.st.end[s];
        uint8_t *entry = entry_of(a, a.keys[first - 1]);
        if (tid == 0) sm = a.st.meta[(size_t)s * (kMaxRounds + 1) + a.rounds];
        __syncthreads();
        for (uint32_t base = first; base < end; base += kLongChunk) {
            uint32_t pending = 0;
#pragma unroll
            for (int j = 0; j < kPerThread; ++j)
                if (base + j * kLongThreads + tid < end) pending |= 1u << j;
            for (;;) {
                const Meta m = sm;
                int mine = kLongChunk;
#pragma unroll
                for (int j = kPerThread - 1; j >= 0; --j) {
                    if (!(pending >> j & 1u)) continue;
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, a.vals[base + j * kLongThreads + tid], x, idx, c);
                    if (would_mutate(TYPE, x, m, c)) mine = j * kLongThreads + tid;
                }
                const int f = block_min<kLongThreads>(mine, red);
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    const int pos = j * kLongThreads + tid;
                    if (!(pending >> j & 1u) || pos >= f) continue;
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, a.vals[base + pos], x, idx, c);
                    Meta t = m;
                    dispatch<SV>(TYPE, x, entry, idx, t, c);
                    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
                    pending &= ~(1u << j);
                }
                __syncthreads();  // every read of the entry value precedes the mutation
                if (f < kLongChunk && (f % kLongThreads) == tid) {
                    uint8_t *x;
                    uint8_t idx;
                    elem_at(a, a.vals[base + f], x, idx, c);
                    Meta mm = m;
                    dispatch<SV>(TYPE, x, entry, idx, mm, c);
                    pending &= ~(1u << (f / kLongThreads));
                    sm = mm;
                }
                __syncthreads();
                if (f >= kLongChunk) break;
            }
        }
        if (tid == 0) meta_store(entry, sm);
        __syncthreads();
    }
}

__global__ void k_node_suspected(const uint8_t *elems, const int32_t *ns_idx, int32_t *out,
                                 int32_t n_batches, int32_t stride, int32_t esz)
{
    int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_batches) return;
    int32_t i = ns_idx[b];
    if (i >= 0) out[b] = elems[((int64_t)b * stride + i) * esz + kOpValueOff];
}

// ------------------------------------------------------------------ populate
struct PopArgs {
    uint64_t *first;      // [p] CityHash .first of id n-1-p
    uint64_t *second;     // [p] .second
    uint32_t *bkt_keys;   // [p] bucket
    uint32_t *pos;        // [p] = p
    int64_t n;
};

__global__ void k_pop_hash(PopArgs a, uint64_t bkt_mask)
{
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n) return;
    uint32_t id = (uint32_t)(a.n - 1 - p);
    uint64_t f, s;
    cityhash128_u32(id, f, s);
    a.first[p] = f;
    a.second[p] = s;
    a.bkt_keys[p] = (uint32_t)((s & 0xFFFFFFFFu) & bkt_mask);  // mica_insert_one: 32-bit bkt field
    a.pos[p] = (uint32_t)p;
}

struct LogPlan {          // virtual offset of insert p (see hkv_runtime.hip: plan_log)
    uint64_t h0;          // head before the first insert
    uint64_t k;           // inserts before the single wrap
    uint64_t hw;          // head right after the wrap
    uint32_t e;           // entry size
};

__device__ __forceinline__ uint64_t plan_off(const LogPlan &L, uint64_t p)
{
    return p < L.k ? L.h0 + p * L.e : L.hw + (p - L.k) * L.e;
}

// one owner lane per bucket replays mica_insert_one (mica.c:78-146) for that bucket's inserts
__global__ void k_pop_buckets(const uint32_t *__restrict__ sk, const uint32_t *__restrict__ sp,
                              const uint64_t *__restrict__ second, uint8_t *index, int64_t n,
                              LogPlan L, unsigned long long *evictions)
{
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    uint32_t bkt = sk[q];
    if (q > 0 && sk[q - 1] == bkt) return;
    uint64_t *slots = reinterpret_cast<uint64_t *>(index + (uint64_t)bkt * 64u);
    uint64_t s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = slots[j];
    unsigned long long ev = 0;
    for (int64_t r = q; r < n && sk[r] == bkt; ++r) {
        uint32_t p = sp[r];
        uint32_t tag = (uint32_t)(second[p] >> 48);
        int use = -1;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((((uint32_t)(s[j] >> 1)) & 0x7FFFFFu) == tag || (s[j] & 1u) == 0) use = j;
        if (use < 0) {
            use = (int)(tag & 7u);
            ++ev;
        }
        uint64_t v = 1u | ((uint64_t)tag << 1) | (plan_off(L, p) << 24);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j == use) s[j] = v;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) slots[j] = s[j];
    if (ev) atomicAdd(evictions, ev);
}

// entry image of spacetime_populate_fixed_len (spacetime.c:32-68); meta fields the reference
// leaves uninitialised (ack_bv, RMW_flag, last_local_write_ts) are written as zero
__global__ void k_pop_log(const uint64_t *__restrict__ first, const uint64_t *__restrict__ second,
                          uint8_t *log, int64_t p_begin, int64_t p_end, int64_t n, LogPlan L,
                          uint64_t log_mask, uint8_t val_len_byte)
{
    int64_t p = p_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= p_end) return;
    uint64_t id = (uint64_t)(n - 1 - p);
    uint64_t *e = reinterpret_cast<uint64_t *>(log + (plan_off(L, (uint64_t)p) & log_mask));
    uint64_t vv = 0x0101010101010101ULL * (uint8_t)('a' + (id % 20));
    e[0] = first[p];
    e[1] = second[p];
    // bytes 16..23: opcode PUT, val_len, state VALID, ack_bv 0, lwid 127, obi 255, lock 0, cid 255
    e[2] = (uint64_t)kOpPut | ((uint64_t)val_len_byte << 8) | ((uint64_t)kValid << 16) |
           ((uint64_t)(kLwidEmpty << 1) << 32) | ((uint64_t)kObiEmpty << 40) | ((uint64_t)kCidEmpty << 56);
    e[3] = 0;                      // ts.version, llw cid, llw version (low bytes)
    e[4] = vv & ~0xFFULL;          // llw version top byte, value from byte 33
    for (uint32_t w = 5; w < L.e / 8; ++w) e[w] = vv;
}

// ------------------------------------------------------------------ host-side launchers
int launch_hash_ids(const uint32_t *ids, uint64_t *out, int64_t n, hipStream_t s)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_hash_ids, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ids, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Stable LSD radix sort of (entry id, element) pairs. rocPRIM picks a merge sort below 1M
// items by default; a merge_sort_limit of 0 keeps every size on the Onesweep radix passes
// (ceil(key_bits / 8) passes over 8-byte pairs), which is what the key width makes cheapest.
// Onesweep with 10-bit digits (3 passes for the 28-bit entry ids of a 100M-key table) and
// 1024x8 tiles: measured fastest on gfx950 for 0.8M-8M pairs (tools/sort_bench.hip,
// profiles/r01_sort_configs.txt); rocPRIM's default (1024x16, 8-bit) is 20-30% slower here.
using SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<1024, 8>, 10,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// heads of long segments (more than kShortSeg elements) of the sorted keys, 0/1 for the scan
struct LongHeadFlag {
    const uint32_t *keys;
    uint32_t skip_key;
    uint32_t n;
    __device__ uint32_t operator()(uint32_t p) const
    {
        const uint32_t k = keys[p];
        return (k != skip_key && (p == 0 || keys[p - 1] != k) && p + kShortSeg < n && keys[p + kShortSeg] == k) ? 1u
                                                                                                                : 0u;
    }
};
using HeadIter = rocprim::transform_iterator<rocprim::counting_iterator<uint32_t>, LongHeadFlag, uint32_t>;

size_t sort_temp_bytes(int64_t n, int key_bits)
{
    size_t bytes = 0, scan = 0;
    rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                          (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0u,
                                          (unsigned)key_bits);
    HeadIter it(rocprim::counting_iterator<uint32_t>(0), LongHeadFlag{nullptr, 0, 0});
    rocprim::inclusive_scan(nullptr, scan, it, (uint32_t *)nullptr, (size_t)n, rocprim::plus<uint32_t>());
    return bytes > scan ? bytes : scan;
}

int sort_pairs(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
               uint32_t *vout, int64_t n, int key_bits, hipStream_t s)
{
    hipError_t e = rocprim::radix_sort_pairs<SortConfig>(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                         (unsigned)key_bits, s);
    return e == hipSuccess ? 0 : -1;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t seg_scratch_bytes(int64_t n, uint32_t entry_size)
{
    const size_t cap = (size_t)(n / (kShortSeg + 1) + 1);
    return align256(4 * (size_t)n) * 2 + align256(8 * (size_t)n) + align256(4 * cap) * 2 + 256 +
           align256(sizeof(Meta) * cap * (kMaxRounds + 1)) + align256(8 * cap * kMaxRounds) + align256(cap) +
           (size_t)entry_size * cap * kMaxRounds;
}

void seg_carve(BatchLaunch &bl, uint8_t *base, int64_t n, uint32_t entry_size)
{
    (void)entry_size;
    const size_t cap = (size_t)(n / (kShortSeg + 1) + 1);
    uint8_t *p = base;
    auto take = [&](size_t bytes) {
        uint8_t *r = p;
        p += align256(bytes);
        return r;
    };
    bl.seg_fallback = reinterpret_cast<uint32_t *>(take(4 * cap));
    bl.seg_of = reinterpret_cast<uint32_t *>(take(4 * (size_t)n));
    bl.seg_hdr = reinterpret_cast<uint64_t *>(take(8 * (size_t)n));
    bl.seg_start = reinterpret_cast<uint32_t *>(take(4 * cap));
    bl.seg_end = reinterpret_cast<uint32_t *>(take(4 * cap));
    bl.seg_count = reinterpret_cast<uint32_t *>(take(8));
    bl.seg_meta = take(sizeof(Meta) * cap * (kMaxRounds + 1));
    bl.seg_mut = reinterpret_cast<unsigned long long *>(take(8 * cap * kMaxRounds));
    bl.seg_done = take(cap);
    bl.seg_snap = p;
    bl.seg_cap = (uint32_t)cap;
}

int launch_batch(const BatchLaunch &bl, hipStream_t s)
{
    const int64_t n = bl.n;
    if (n <= 0) return 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    LookupArgs la;
    la.elems = bl.elems;
    la.counts = bl.counts;
    la.index = bl.index;
    la.log = bl.log;
    la.keys = bl.keys_a;
    la.vals = bl.vals_a;
    la.ns_idx = bl.ns_idx;
    la.g = bl.g;
    la.n = n;
    la.stride = bl.stride;
    la.esz = bl.esz;
    la.type = bl.type;
    la.skip_key = bl.skip_key;
    hipLaunchKernelGGL(k_lookup, dim3((unsigned)((n + kLookupPerBlock - 1) / kLookupPerBlock)), dim3(256), 0, s, la);
    if (hipGetLastError() != hipSuccess) return -1;
    if (sort_pairs(bl.sort_tmp, bl.sort_tmp_bytes, bl.keys_a, bl.keys_b, bl.vals_a, bl.vals_b, n, bl.key_bits, s))
        return -2;
    SegmentArgs sa;
    sa.st.start = bl.seg_start;
    sa.st.end = bl.seg_end;
    sa.st.count = bl.seg_count;
    sa.st.fallback = bl.seg_fallback;
    sa.st.lidx = bl.keys_a;  // the sort's input keys are free again
    sa.st.seg_of = bl.seg_of;
    sa.st.hdr = bl.seg_hdr;
    sa.st.meta = reinterpret_cast<Meta *>(bl.seg_meta);
    sa.st.mut = bl.seg_mut;
    sa.st.done = bl.seg_done;
    sa.st.snap = bl.seg_snap;
    sa.st.cap = bl.seg_cap;
    sa.st.epoch = bl.epoch;
    sa.elems = bl.elems;
    sa.log = bl.log;
    sa.rw = bl.rw;
    sa.keys = bl.keys_b;
    sa.vals = bl.vals_b;
    sa.error_flags = bl.error_flags;
    sa.g = bl.g;
    sa.n = n;
    sa.rw_stride = bl.rw_stride;
    sa.stride = bl.stride;
    sa.esz = bl.esz;
    sa.type = bl.type;
    sa.skip_key = bl.skip_key;
    sa.g_membership = bl.g_membership;
    sa.w_ack_init = bl.w_ack_init;
    sa.rounds = rounds_for(bl.type);
    {
        HeadIter it(rocprim::counting_iterator<uint32_t>(0), LongHeadFlag{bl.keys_b, bl.skip_key, (uint32_t)n});
        size_t tb = bl.sort_tmp_bytes;
        if (rocprim::inclusive_scan(bl.sort_tmp, tb, it, bl.keys_a, (size_t)n, rocprim::plus<uint32_t>(), s) !=
            hipSuccess)
            return -2;
    }
    const int64_t max_long = n / (kShortSeg + 1) + 1;
    const unsigned sgrid = (unsigned)((max_long + 255) / 256);
#define HKV_LAUNCH_SEG(T, V)                                                                        \
    do {                                                                                            \
        if (V == 287 || bl.esz > 64) {                                                              \
            const size_t lds = segment_exec_lds<128>(bl.esz, bl.g.entry_size);                      \
            if (lds > 64 * 1024)                                                                    \
                hipFuncSetAttribute((const void *)k_segment_exec<T, V, 128>,                        \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);          \
            hipLaunchKernelGGL((k_segment_exec<T, V, 128>), dim3((unsigned)((n + 127) / 128)),     \
                               dim3(128), lds, s, sa);                                              \
        } else {                                                                                    \
            hipLaunchKernelGGL((k_segment_exec<T, V, 256>), dim3(grid), dim3(256),                  \
                               segment_exec_lds<256>(bl.esz, bl.g.entry_size), s, sa);              \
        }                                                                                           \
        for (int r = 0; r < sa.rounds; ++r) {                                                       \
            if (r > 0) hipLaunchKernelGGL((k_round_cand<T>), dim3(grid), dim3(256), 0, s, sa, r);   \
            hipLaunchKernelGGL((k_round_apply<T, V>), dim3(sgrid), dim3(256), 0, s, sa, r);         \
        }                                                                                           \
        hipLaunchKernelGGL((k_round_resolve<T, V>), dim3(grid), dim3(256), 0, s, sa);               \
        hipLaunchKernelGGL((k_long_exec<T, V>), dim3(64), dim3(kLongThreads), 0, s, sa);            \
    } while (0)
#define HKV_LAUNCH_SV(T)                                       \
    do {                                                       \
        if (bl.g.st_value == 31) HKV_LAUNCH_SEG(T, 31);        \
        else if (bl.g.st_value == 287) HKV_LAUNCH_SEG(T, 287); \
        else HKV_LAUNCH_SEG(T, 0);                             \
    } while (0)
    switch (bl.type) {
    case kLocal: HKV_LAUNCH_SV(kLocal); break;
    case kLocalAfterMemb: HKV_LAUNCH_SV(kLocalAfterMemb); break;
    case kInvs: HKV_LAUNCH_SV(kInvs); break;
    case kAcks: HKV_LAUNCH_SV(kAcks); break;
    default: HKV_LAUNCH_SV(kVals); break;
    }
#undef HKV_LAUNCH_SV
#undef HKV_LAUNCH_SEG
    if (hipGetLastError() != hipSuccess) return -3;
    if (bl.type == kInvs && bl.ns_idx && bl.node_suspected) {
        hipLaunchKernelGGL(k_node_suspected, dim3((bl.n_batches + 255) / 256), dim3(256), 0, s, bl.elems,
                           bl.ns_idx, bl.node_suspected, bl.n_batches, bl.stride, bl.esz);
        if (hipGetLastError() != hipSuccess) return -4;
    }
    return 0;
}

int launch_populate(const PopulateLaunch &pl, hipStream_t s)
{
    const int64_t n = pl.n;
    if (n <= 0) return 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    PopArgs a{pl.first, pl.second, pl.keys_a, pl.vals_a, n};
    hipLaunchKernelGGL(k_pop_hash, dim3(grid), dim3(256), 0, s, a, pl.bkt_mask);
    if (hipGetLastError() != hipSuccess) return -1;
    if (sort_pairs(pl.sort_tmp, pl.sort_tmp_bytes, pl.keys_a, pl.keys_b, pl.vals_a, pl.vals_b, n, pl.key_bits, s))
        return -2;
    LogPlan L{pl.h0, pl.k, pl.hw, pl.entry_size};
    hipLaunchKernelGGL(k_pop_buckets, dim3(grid), dim3(256), 0, s, pl.keys_b, pl.vals_b, pl.second, pl.index, n, L,
                       pl.evictions);
    if (hipGetLastError() != hipSuccess) return -3;
    // later inserts overwrite earlier ones when the log wraps: write in chunks no longer than one
    // physical lap, in insertion order
    // (a run of inserts never overlaps itself physically while it stays within one lap of the
    // log and does not cross the single wrap point, so each launch covers such a run)
    int64_t chunk = (int64_t)(pl.log_cap / pl.entry_size);
    if (chunk < 1) chunk = 1;
    const int64_t wrap_at = pl.k < (uint64_t)n ? (int64_t)pl.k : n;
    const int64_t runs[2][2] = {{0, wrap_at}, {wrap_at, n}};
    for (const auto &r : runs) {
        for (int64_t b = r[0]; b < r[1]; b += chunk) {
            int64_t e = b + chunk < r[1] ? b + chunk : r[1];
            hipLaunchKernelGGL(k_pop_log, dim3((unsigned)((e - b + 255) / 256)), dim3(256), 0, s, pl.first,
                               pl.second, pl.log, b, e, n, L, pl.log_mask, pl.val_len_byte);
            if (hipGetLastError() != hipSuccess) return -4;
        }
    }
    return 0;
}

}  // namespace hkv
