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

__global__ __launch_bounds__(256) void k_lookup(LookupArgs a)
{
    int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= a.n) return;
    int32_t b = (int32_t)(gi / a.stride);
    int32_t idx = (int32_t)(gi - (int64_t)b * a.stride);
    uint32_t key_out = a.skip_key;
    a.vals[gi] = (uint32_t)gi;
    if (a.counts == nullptr || idx < a.counts[b]) {
        uint8_t *x = a.elems + gi * a.esz;
        if (skip_elem(a.type, x)) {
            if (a.type == kInvs && a.ns_idx) atomicMax(&a.ns_idx[b], idx);
        } else {
            uint64_t key = ld64(x);
            const uint4 *bkt = reinterpret_cast<const uint4 *>(a.index + ((key & 0xFFFFFFFFFFFFULL) & a.g.bkt_mask) * 64u);
            uint4 q[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = bkt[j];
            const uint64_t *slots = reinterpret_cast<const uint64_t *>(q);
            uint32_t tag = (uint32_t)(key >> 48);
            bool hit = false;
            uint64_t off = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint64_t s = slots[j];
                if (!hit && (s & 1u) && ((uint32_t)(s >> 1) & 0x7FFFFFu) == tag) {
                    hit = true;
                    off = s >> 24;
                }
            }
            if (hit && a.g.log_head - off < a.g.log_cap) {
                uint64_t phys = off & a.g.log_mask;
                if (ld64(a.log + phys + 8) == key) key_out = (uint32_t)(phys / a.g.entry_unit);
            }
            if (key_out == a.skip_key) x[9] = kMiss;
        }
    }
    a.keys[gi] = key_out;
}

// ------------------------------------------------------------------ batch stage 3: segments
struct SegmentArgs {
    uint32_t *long_start;   // hot list: [0, cap)   mid list: [cap, 2*cap)
    uint32_t *long_len;
    uint32_t *long_count;   // [0] hot, [1] mid
    uint32_t list_cap;
    uint8_t *elems;
    uint8_t *log;
    uint8_t *rw;
    const uint32_t *keys;
    const uint32_t *vals;
    Geometry g;
    int64_t n;
    int64_t rw_stride;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint32_t skip_key;
    uint8_t g_membership;
    uint8_t w_ack_init;
};

// Three tiers by segment length: at most kShortSeg elements are applied serially by the
// segment's owner lane (k_segment_exec); up to kMidSeg by one wavefront (k_wave_exec); longer
// ones (the hottest keys) by a 1024-thread workgroup (k_long_exec). The last two receive their
// segments through compact work lists written by k_segment_exec.
constexpr int kShortSeg = 4;
constexpr int kMidSeg = 4096;

// Queue a segment on one of the two work lists with one atomic per wavefront and list
// (a per-lane atomic on a shared counter serialises hundreds of thousands of heads).
__device__ __forceinline__ void enqueue_segment(const SegmentArgs &a, bool want, int tier, uint32_t start,
                                                uint32_t len)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const unsigned long long m = __ballot(want && tier == t);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&a.long_count[t], (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        if (want && tier == t) {
            const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)) + (uint32_t)t * a.list_cap;
            a.long_start[slot] = start;
            a.long_len[slot] = len;
        }
    }
}

template <int TYPE, int SV>
__global__ __launch_bounds__(256) void k_segment_exec(SegmentArgs a)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t key = p < a.n ? a.keys[p] : a.skip_key;
    const bool head = key != a.skip_key && (p == 0 || a.keys[p - 1] != key);
    const bool longseg = head && p + kShortSeg < a.n && a.keys[p + kShortSeg] == key;
    uint32_t len = 0;
    if (longseg) {
        // gallop to the end of the segment on the sorted keys
        int64_t lo = p + kShortSeg, step = 2 * kShortSeg, hi;
        for (;;) {
            hi = lo + step;
            if (hi >= a.n || a.keys[hi] != key) break;
            lo = hi;
            step *= 2;
        }
        if (hi > a.n) hi = a.n;
        while (hi - lo > 1) {  // keys[lo] == key, keys[hi] != key (or hi == n)
            int64_t mid = (lo + hi) / 2;
            if (a.keys[mid] == key) lo = mid;
            else hi = mid;
        }
        len = (uint32_t)(hi - p);
    }
    enqueue_segment(a, longseg, len > (uint32_t)kMidSeg ? 0 : 1, (uint32_t)p, len);
    if (!head || longseg) return;
    uint8_t *entry = a.log + (uint64_t)key * a.g.entry_unit;
    Meta m;
    meta_load(entry, m);
    Ctx c;
    c.g = a.g;
    c.g_membership = a.g_membership;
    c.w_ack_init = a.w_ack_init;
    for (int64_t q = p; q < a.n && a.keys[q] == key; ++q) {
        uint32_t gi = a.vals[q];
        int32_t b = (int32_t)(gi / (uint32_t)a.stride);
        uint32_t idx = gi - (uint32_t)b * (uint32_t)a.stride;
        c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
        dispatch<SV>(TYPE, a.elems + (int64_t)gi * a.esz, entry, (uint8_t)idx, m, c);
    }
    meta_store(entry, m);
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

__device__ __forceinline__ int wave_min(int v)
{
    for (int o = 32; o > 0; o >>= 1) {
        int u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    return v;
}

__device__ __forceinline__ void meta_bcast(Meta &m, int src)
{
    m.w4 = __shfl(m.w4, src, 64);
    m.w5 = __shfl(m.w5, src, 64);
    m.ver = __shfl(m.ver, src, 64);
    m.llw_ver = __shfl(m.llw_ver, src, 64);
    m.llw_cid = (uint8_t)__shfl((int)m.llw_cid, src, 64);
}

// One 1024-thread workgroup per long segment (one hot key), in chunks of kLongChunk elements
// (kPerThread per lane, lane-strided so the sorted element ids are read coalesced).
// Per chunk, repeat: every unresolved element asks would_mutate() against the shared meta;
// the first candidate f is found with a block min; elements before f are resolved in parallel,
// each running the serial exec function on a private copy of the meta (it cannot change it);
// after a barrier, f alone runs the exec function on the shared meta. A chunk without a
// candidate takes one pass, so a hot key costs one pass per kLongChunk elements plus one per
// mutation. A non-candidate that did change its copy sets bit 0 of *error_flags (that would
// mean would_mutate() is unsound).
struct LongArgs {
    uint8_t *elems;
    uint8_t *log;
    uint8_t *rw;
    const uint32_t *keys;
    const uint32_t *vals;
    const uint32_t *long_start;
    const uint32_t *long_len;
    const uint32_t *long_count;
    uint32_t list_cap;
    unsigned int *error_flags;
    Geometry g;
    int64_t rw_stride;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint8_t g_membership;
    uint8_t w_ack_init;
};

constexpr int kLongThreads = 1024;
constexpr int kPerThread = 8;
constexpr int kLongChunk = kLongThreads * kPerThread;

template <int TYPE, int SV>
__global__ __launch_bounds__(kLongThreads) void k_long_exec(LongArgs a)
{
    __shared__ Meta sm;
    __shared__ int red[kLongThreads / 64];
    const int tid = threadIdx.x;
    const uint32_t nseg = a.long_count[0];
    Ctx c;
    c.g = a.g;
    c.g_membership = a.g_membership;
    c.w_ack_init = a.w_ack_init;
    c.rw = nullptr;
    for (uint32_t s = blockIdx.x; s < nseg; s += gridDim.x) {
        const uint32_t start = a.long_start[s], len = a.long_len[s];
        const uint32_t key = a.keys[start];
        uint8_t *entry = a.log + (uint64_t)key * a.g.entry_unit;
        if (tid == 0) {
            Meta m;
            meta_load(entry, m);
            sm = m;
        }
        __syncthreads();
        for (uint32_t base = 0; base < len; base += kLongChunk) {
            uint32_t pending = 0;  // bit j: element base + j*kLongThreads + tid still to apply
#pragma unroll
            for (int j = 0; j < kPerThread; ++j)
                if (base + j * kLongThreads + tid < len) pending |= 1u << j;
            for (;;) {
                const Meta m = sm;
                int mine = kLongChunk;
#pragma unroll
                for (int j = kPerThread - 1; j >= 0; --j) {
                    if (!(pending >> j & 1u)) continue;
                    const uint32_t gi = a.vals[start + base + j * kLongThreads + tid];
                    if (would_mutate(TYPE, a.elems + (int64_t)gi * a.esz, m, c)) mine = j * kLongThreads + tid;
                }
                const int f = block_min<kLongThreads>(mine, red);
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    const int pos = j * kLongThreads + tid;
                    if (!(pending >> j & 1u) || pos >= f) continue;
                    const uint32_t gi = a.vals[start + base + pos];
                    const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
                    Meta t = m;
                    c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
                    dispatch<SV>(TYPE, a.elems + (int64_t)gi * a.esz, entry,
                                 (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride), t, c);
                    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
                    pending &= ~(1u << j);
                }
                __syncthreads();  // every read of the entry value precedes the mutation
                if (f < kLongChunk && (f % kLongThreads) == tid) {
                    const int j = f / kLongThreads;
                    const uint32_t gi = a.vals[start + base + f];
                    const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
                    Meta mm = m;
                    c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
                    dispatch<SV>(TYPE, a.elems + (int64_t)gi * a.esz, entry,
                                 (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride), mm, c);
                    pending &= ~(1u << j);
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

// One wavefront per medium segment: the same first-candidate rounds as k_long_exec, in chunks
// of 64 * kWavePer elements, with the meta replicated in every lane's registers (the owner of
// a mutation broadcasts it by shuffles). Within a wavefront program order separates the
// resolving lanes' entry-value reads from the mutation's writes, so no barrier is needed.
constexpr int kWavePer = 4;

template <int TYPE, int SV>
__global__ __launch_bounds__(256) void k_wave_exec(LongArgs a)
{
    const int lane = threadIdx.x & 63;
    const uint32_t wid = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t nseg = a.long_count[1];
    Ctx c;
    c.g = a.g;
    c.g_membership = a.g_membership;
    c.w_ack_init = a.w_ack_init;
    c.rw = nullptr;
    for (uint32_t s = wid; s < nseg; s += gridDim.x * 4u) {
        const uint32_t start = a.long_start[a.list_cap + s], len = a.long_len[a.list_cap + s];
        const uint32_t key = a.keys[start];
        uint8_t *entry = a.log + (uint64_t)key * a.g.entry_unit;
        Meta m;
        meta_load(entry, m);
        for (uint32_t base = 0; base < len; base += 64 * kWavePer) {
            uint32_t gis[kWavePer];
            uint32_t pending = 0;
#pragma unroll
            for (int j = 0; j < kWavePer; ++j) {
                const uint32_t pos = base + j * 64 + lane;
                gis[j] = pos < len ? a.vals[start + pos] : 0u;
                if (pos < len) pending |= 1u << j;
            }
            for (;;) {
                int mine = 64 * kWavePer;
#pragma unroll
                for (int j = kWavePer - 1; j >= 0; --j)
                    if ((pending >> j & 1u) && would_mutate(TYPE, a.elems + (int64_t)gis[j] * a.esz, m, c))
                        mine = j * 64 + lane;
                const int f = wave_min(mine);
#pragma unroll
                for (int j = 0; j < kWavePer; ++j) {
                    if (!(pending >> j & 1u) || j * 64 + lane >= f) continue;
                    const uint32_t gi = gis[j];
                    const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
                    Meta t = m;
                    c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
                    dispatch<SV>(TYPE, a.elems + (int64_t)gi * a.esz, entry,
                                 (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride), t, c);
                    if (a.error_flags && !meta_equal(t, m)) atomicOr(a.error_flags, 1u);
                    pending &= ~(1u << j);
                }
                if (f >= 64 * kWavePer) break;
                const int owner = f & 63, j = f >> 6;
                if (lane == owner) {
#pragma unroll
                    for (int jj = 0; jj < kWavePer; ++jj) {
                        if (jj != j) continue;
                        const uint32_t gi = gis[jj];
                        const int32_t b = (int32_t)(gi / (uint32_t)a.stride);
                        c.rw = a.rw ? a.rw + (int64_t)b * a.rw_stride : nullptr;
                        dispatch<SV>(TYPE, a.elems + (int64_t)gi * a.esz, entry,
                                     (uint8_t)(gi - (uint32_t)b * (uint32_t)a.stride), m, c);
                        pending &= ~(1u << jj);
                    }
                }
                meta_bcast(m, owner);
            }
        }
        if (lane == 0) meta_store(entry, m);
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
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;

size_t sort_temp_bytes(int64_t n, int key_bits)
{
    size_t bytes = 0;
    rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                          (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0u,
                                          (unsigned)key_bits);
    return bytes;
}

int sort_pairs(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
               uint32_t *vout, int64_t n, int key_bits, hipStream_t s)
{
    hipError_t e = rocprim::radix_sort_pairs<SortConfig>(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                         (unsigned)key_bits, s);
    return e == hipSuccess ? 0 : -1;
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
    hipLaunchKernelGGL(k_lookup, dim3(grid), dim3(256), 0, s, la);
    if (hipGetLastError() != hipSuccess) return -1;
    if (sort_pairs(bl.sort_tmp, bl.sort_tmp_bytes, bl.keys_a, bl.keys_b, bl.vals_a, bl.vals_b, n, bl.key_bits, s))
        return -2;
    SegmentArgs sa;
    sa.elems = bl.elems;
    sa.log = bl.log;
    sa.rw = bl.rw;
    sa.keys = bl.keys_b;
    sa.vals = bl.vals_b;
    sa.g = bl.g;
    sa.n = n;
    sa.rw_stride = bl.rw_stride;
    sa.stride = bl.stride;
    sa.esz = bl.esz;
    sa.type = bl.type;
    sa.skip_key = bl.skip_key;
    sa.g_membership = bl.g_membership;
    sa.w_ack_init = bl.w_ack_init;
    sa.long_start = bl.long_start;
    sa.long_len = bl.long_len;
    sa.long_count = bl.long_count;
    sa.list_cap = bl.list_cap;
    if (hipMemsetAsync(bl.long_count, 0, 2 * sizeof(uint32_t), s) != hipSuccess) return -3;
    LongArgs la2;
    la2.elems = bl.elems;
    la2.log = bl.log;
    la2.rw = bl.rw;
    la2.keys = bl.keys_b;
    la2.vals = bl.vals_b;
    la2.long_start = bl.long_start;
    la2.long_len = bl.long_len;
    la2.long_count = bl.long_count;
    la2.list_cap = bl.list_cap;
    la2.error_flags = bl.error_flags;
    la2.g = bl.g;
    la2.rw_stride = bl.rw_stride;
    la2.stride = bl.stride;
    la2.esz = bl.esz;
    la2.type = bl.type;
    la2.g_membership = bl.g_membership;
    la2.w_ack_init = bl.w_ack_init;
    // grids sized by how many segments each tier can hold at most
    int64_t max_hot = n / (kMidSeg + 1) + 1, max_mid = n / (kShortSeg + 1) + 1;
    const unsigned lgrid = (unsigned)(max_hot < 256 ? max_hot : 256);
    const unsigned wgrid = (unsigned)((max_mid + 3) / 4 < 2048 ? (max_mid + 3) / 4 : 2048);
#define HKV_LAUNCH_SEG(T, V)                                                                       \
    do {                                                                                           \
        hipLaunchKernelGGL((k_segment_exec<T, V>), dim3(grid), dim3(256), 0, s, sa);               \
        hipLaunchKernelGGL((k_wave_exec<T, V>), dim3(wgrid), dim3(256), 0, s, la2);               \
        hipLaunchKernelGGL((k_long_exec<T, V>), dim3(lgrid), dim3(kLongThreads), 0, s, la2);      \
    } while (0)
#define HKV_LAUNCH_SV(T)                                      \
    do {                                                      \
        if (bl.g.st_value == 31) HKV_LAUNCH_SEG(T, 31);       \
        else if (bl.g.st_value == 287) HKV_LAUNCH_SEG(T, 287); \
        else HKV_LAUNCH_SEG(T, 0);                            \
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
