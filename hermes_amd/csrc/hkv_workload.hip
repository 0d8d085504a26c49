// hkv_workload.hip -- device kernels around the batch path (include/hermeskv_workload.h):
// seeded traces, refill + commit counting, and the worker loop's message marshalling, so a
// protocol round never leaves HBM. One 256-thread workgroup per virtual worker where the
// reference walks a worker's op buffer in order (refill, INV marshalling): the slot order
// is kept with a wave-ballot prefix count instead of a serial loop.
#include <hip/hip_runtime.h>

#include "../../include/hermeskv.h"
#include "../../include/hermeskv_workload.h"
#include "hkv_codes.h"
#include "hkv_internal.h"

namespace hkv {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

__device__ __forceinline__ double unit_double(uint64_t r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

// Gray et al. "Quickly generating billion-record synthetic databases" (the YCSB Zipfian
// generator); rank == key id, so id 0 is the hottest key as in parse_trace (util.c:337-343)
__device__ __forceinline__ uint64_t zipf_draw(const hkv_zipf &z, double u)
{
    if (z.theta <= 0.0) {
        uint64_t id = (uint64_t)(u * (double)z.n);
        return id < z.n ? id : z.n - 1;
    }
    double uz = u * z.zetan;
    if (uz < 1.0) return 0;
    if (uz < z.half_pow) return 1;
    uint64_t id = (uint64_t)((double)z.n * pow(z.eta * u - z.eta + 1.0, z.alpha));
    return id < z.n ? id : z.n - 1;
}

__device__ __forceinline__ uint64_t ch_mix16(uint64_t u, uint64_t v)
{
    const uint64_t mul = 0x9ddfea08eb382d69ULL;
    uint64_t a = (u ^ v) * mul;
    a ^= a >> 47;
    uint64_t b = (v ^ a) * mul;
    b ^= b >> 47;
    return b * mul;
}

// CityHash128(&id, 4).second (city.c:276-308 short path; see hkv_kernels.hip)
__device__ __forceinline__ uint64_t key_of_id(uint32_t id)
{
    const uint64_t k0 = 0xc3a5c85c97cb3127ULL, k1 = 0xb492b66fbe98f273ULL;
    uint64_t a = k0 * k1;
    a = (a ^ (a >> 47)) * k1;
    uint64_t c = k1 * k1 + ch_mix16(4u + ((uint64_t)id << 3), (uint64_t)id);
    uint64_t d = (a + c) ^ ((a + c) >> 47);
    uint64_t aa = ch_mix16(a, c);
    uint64_t bb = ch_mix16(d, k1);
    return ch_mix16(bb, aa);
}

// exclusive prefix count of `flag` over a 256-thread workgroup, in thread order
__device__ __forceinline__ int block_rank(bool flag, int &total)
{
    __shared__ int wave_tot[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long m = __ballot(flag);
    int in_wave = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wave] = __popcll(m);
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (w < wave) before += wave_tot[w];
        total += wave_tot[w];
    }
    __syncthreads();
    return before + in_wave;
}

__device__ __forceinline__ int block_sum(int v)
{
    __shared__ int part[4];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    int s = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    return s;
}

__global__ void k_gen_trace(uint64_t *tkey, uint8_t *top, uint32_t *tid, int32_t n_workers, int32_t len,
                            hkv_zipf z, uint32_t write_pm, uint32_t rmw_pm, uint64_t seed)
{
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (int64_t)n_workers * len) return;
    uint64_t r1 = splitmix64(seed ^ (0x1000003ull * (uint64_t)g));
    uint64_t r2 = splitmix64(r1 ^ 0x5EEDull);
    uint32_t id = (uint32_t)zipf_draw(z, unit_double(r1));
    uint32_t coin = (uint32_t)(r2 % 1000u);
    uint8_t op = kOpGet;
    if (coin < write_pm) {  // create_uni_trace, util.c:236-240
        op = kOpPut;
        if (rmw_pm && (uint32_t)((r2 >> 32) % 1000u) < rmw_pm) op = kOpRmw;
    }
    tkey[g] = key_of_id(id);
    top[g] = op;
    if (tid) tid[g] = id;
}

// refill_ops, inline-util.h:149-303 (hot-key coalescing and latency probes off)
constexpr int kStripes = (HKV_WL_COUNTER_WORDS - HKV_WL_STRIPE_BASE) / 16;
constexpr int kCounters = 5;  // committed, misses, completed writes, dropped (refill_all), RMW aborts

// Ops a fresh-batch refill (refill_all) must keep: writes and replays between their local
// success and their completion (waiting for INV credits, ACKs or the VALs of a membership
// change), and membership-change ops. Overwriting one would leave its key in WRITE/REPLAY with
// an op buffer index that points at an unrelated op.
// val_skip_or_get_sender_id (hermes_worker.c:122-136, assertions off as configured, config.h:83):
// an ACK element answers with a VAL unless it is ST_ACK_SUCCESS, a membership change or empty;
// afterwards every one of them is empty (the skipped ones by the skip, the sent ones by
// val_modify_elem_after_send)
__device__ __forceinline__ bool val_sends(uint8_t oc) { return oc != kAckSuccess && oc != kOpMembChange && oc != kEmpty; }

__device__ __forceinline__ bool in_flight(uint8_t st)
{
    return st == kPutSuccess || st == kRmwSuccess || st == kReplaySuccess || st == kInProgressPut ||
           st == kInProgressRmw || st == kInProgressReplay || st == kPutCompleteSendVals ||
           st == kRmwCompleteSendVals || st == kReplayCompleteSendVals || st == kOpMembChange;
}

__device__ __forceinline__ bool is_complete(uint8_t st)  // refill_ops, inline-util.h:189-195
{
    return st == kMiss || st == kPutComplete || st == kRmwAbort || st == kRmwComplete || st == kOpMembComplete ||
           st == kGetComplete;
}

// folds the refill stripes into counters[0..4] and clears them
__global__ __launch_bounds__(256) void k_fold_counters(unsigned long long *counters)
{
    __shared__ unsigned long long part[4][kCounters];
    unsigned long long v[kCounters] = {0, 0, 0, 0, 0};
    for (int s = threadIdx.x; s < kStripes; s += 256) {
        unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + s * 16;
#pragma unroll
        for (int k = 0; k < kCounters; ++k) {
            v[k] += stripe[k];
            stripe[k] = 0;
        }
    }
#pragma unroll
    for (int k = 0; k < kCounters; ++k) {
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_down(v[k], o, 64);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < kCounters) counters[threadIdx.x] += part[0][threadIdx.x] + part[1][threadIdx.x] +
                                                         part[2][threadIdx.x] + part[3][threadIdx.x];
}

// The worker's op slab (stride * op_size contiguous bytes) is staged through LDS so HBM sees
// full-width coalesced reads and writes; the per-op byte edits then happen in LDS.
__global__ __launch_bounds__(256) void k_refill(uint8_t *ops, int32_t stride, uint32_t op_size, uint32_t st_value,
                                                uint32_t shift, const uint64_t *tkey, const uint8_t *top,
                                                int32_t tlen, uint32_t *cursor, uint32_t machine_id,
                                                int32_t first_iter, uint32_t flags, unsigned long long *counters,
                                                uint8_t *opc_out)
{
    const bool refill_all = (flags & HKV_WL_REFILL_ALL) != 0;
    extern __shared__ uint64_t slab[];
    const int w = blockIdx.x, i = threadIdx.x;
    const bool live = i < stride;
    uint64_t *gslab = reinterpret_cast<uint64_t *>(ops + (int64_t)w * stride * op_size);
    const int words = (int)((uint32_t)stride * op_size / 8u);
    // 16-B accesses when the slab allows (250 x 56 B does): half the memory instructions
    const bool wide = (words & 1) == 0 && (reinterpret_cast<uintptr_t>(gslab) & 15) == 0;
    if (wide) {
        const uint4 *g4 = reinterpret_cast<const uint4 *>(gslab);
        uint4 *s4 = reinterpret_cast<uint4 *>(slab);
        for (int k = i; k < words / 2; k += 256) s4[k] = g4[k];
    } else {
        for (int k = i; k < words; k += 256) slab[k] = gslab[k];
    }
    __syncthreads();
    uint8_t *op = reinterpret_cast<uint8_t *>(slab) + (uint32_t)i * op_size;
    uint8_t st = live ? op[9] : 0;
    const bool complete = is_complete(st);
    // refill_all: stalled ops are dropped (and counted), ops in flight keep their slot
    const bool drop = live && !first_iter && refill_all && !complete && !in_flight(st);
    bool done = live && (first_iter || complete || drop);
    int commits = (live && complete && !first_iter && st != kMiss && st != kRmwAbort) ? 1 : 0;
    int misses = (live && !first_iter && st == kMiss) ? 1 : 0;
    int writes = (live && !first_iter && st == kPutComplete) ? 1 : 0;
    int total;
    int rank = block_rank(done, total);
    uint32_t base = cursor[w];
    int c = block_sum(commits), m = block_sum(misses), wr = block_sum(writes), dr = block_sum(drop ? 1 : 0);
    int ab = block_sum((live && !first_iter && st == kRmwAbort) ? 1 : 0);
    if (i == 0) {
        cursor[w] = (uint32_t)((base + (uint32_t)total) % (uint32_t)tlen);
        unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + (w % kStripes) * 16;
        if (c) atomicAdd(&stripe[0], (unsigned long long)c);
        if (m) atomicAdd(&stripe[1], (unsigned long long)m);
        if (wr) atomicAdd(&stripe[2], (unsigned long long)wr);
        if (dr) atomicAdd(&stripe[3], (unsigned long long)dr);
        if (ab) atomicAdd(&stripe[4], (unsigned long long)ab);
    }
    if (done) {
        int64_t t = (int64_t)w * tlen + (int64_t)((base + (uint32_t)rank) % (uint32_t)tlen);
        uint8_t oc = top[t];
        *reinterpret_cast<uint64_t *>(op) = tkey[t];
        op[8] = oc;
        op[9] = kNew;
        op[10] = oc == kOpGet ? 0 : (uint8_t)(st_value >> shift);
        if (oc == kOpGet && (flags & HKV_WL_READ_TS_RESET)) {  // inline-util.h:268-272
            op[11] = 0;
            *reinterpret_cast<uint32_t *>(op + 12) = 0;
        }
        const uint16_t fl = (uint16_t)((oc == kOpRmw ? 1u : 0u) | (first_iter ? 0u : 2u));  // RMW_flag, no_coales = 1
        *reinterpret_cast<uint16_t *>(op + 16) = fl;
        if (oc != kOpGet) {
            uint8_t v = (uint8_t)('a' + machine_id);
            for (uint32_t k = 0; k < st_value; ++k) op[kOpValueOff + k] = v;
        }
    }
    if (opc_out && live) opc_out[(int64_t)w * stride + i] = op[8];  // the opcode mirror
    __syncthreads();
    if (wide) {
        uint4 *g4 = reinterpret_cast<uint4 *>(gslab);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(slab);
        for (int k = i; k < words / 2; k += 256) g4[k] = s4[k];
    } else {
        for (int k = i; k < words; k += 256) gslab[k] = slab[k];
    }
}

// refill_ops with ENABLE_COALESCE_OF_HOT_REQS (inline-util.h:237-257, config.h:77-78): a trace
// command on one of the COALESCE_N_HOTTEST_KEYS hottest ids (GET or PUT) whose worker's last op
// inserted for that id and opcode class (n_hottest_keys_in_ops_get/_put, hermes_worker.c:394-399:
// per worker, kept across refills, never cleared) currently has the same opcode is absorbed into
// it (no_coales + 1) instead of taking a slot; the pointer names a slot, not an op, so as in the
// reference the slot may hold another key by then. A completed op counts no_coales commits. The
// walk is sequential by nature (each command's fate depends on the pointers the previous ones
// left), so one lane runs it over LDS copies of the slab, the pointers and a window of the trace;
// the slab edits that do not feed the walk (key, value, timestamp) then go in parallel.
constexpr int kHotKeys = 100;         // COALESCE_N_HOTTEST_KEYS, config.h:78
constexpr int kHotWindow = 2048;      // trace commands staged in LDS (the walk reads on from memory)
__global__ __launch_bounds__(256) void k_refill_hot(uint8_t *ops, int32_t stride, uint32_t op_size, uint32_t st_value,
                                                    uint32_t shift, const uint64_t *tkey, const uint8_t *top,
                                                    const uint32_t *tid, int32_t tlen, uint32_t *cursor,
                                                    uint32_t machine_id, int32_t first_iter, uint32_t flags,
                                                    unsigned long long *counters, uint8_t *opc_out, uint8_t *hot)
{
    extern __shared__ uint64_t slab[];
    __shared__ uint32_t wid[kHotWindow];
    __shared__ uint8_t wop[kHotWindow];
    __shared__ uint8_t hp[2 * kHotKeys];     // [0, 100): GET pointers, [100, 200): PUT/RMW; 0xFF = NULL
    __shared__ int32_t tpos[256];            // trace position a refilled slot takes, -1: kept
    __shared__ unsigned long long tot[kCounters];
    const int w = blockIdx.x, i = threadIdx.x;
    const bool refill_all = (flags & HKV_WL_REFILL_ALL) != 0;
    uint64_t *gslab = reinterpret_cast<uint64_t *>(ops + (int64_t)w * stride * op_size);
    const int words = (int)((uint32_t)stride * op_size / 8u);
    for (int k = i; k < words; k += 256) slab[k] = gslab[k];
    const uint32_t base = cursor[w];
    for (int k = i; k < kHotWindow; k += 256) {
        const int64_t t = (int64_t)w * tlen + (int64_t)((base + (uint32_t)k) % (uint32_t)tlen);
        wid[k] = tid[t];
        wop[k] = top[t];
    }
    for (int k = i; k < 2 * kHotKeys; k += 256) hp[k] = hot[(int64_t)w * 2 * kHotKeys + k];
    __syncthreads();
    uint8_t *sb = reinterpret_cast<uint8_t *>(slab);
    if (i == 0) {
        unsigned long long c = 0, m = 0, wr = 0, dr = 0, ab = 0;
        uint32_t it = 0;   // commands consumed (window position)
        auto cmd = [&](uint32_t k, uint32_t &id, uint8_t &oc) {
            if (k < (uint32_t)kHotWindow) {
                id = wid[k];
                oc = wop[k];
            } else {
                const int64_t t = (int64_t)w * tlen + (int64_t)((base + k) % (uint32_t)tlen);
                id = tid[t];
                oc = top[t];
            }
        };
        for (int s = 0; s < stride; ++s) {
            uint8_t *op = sb + (uint32_t)s * op_size;
            const uint8_t st = op[9];
            const bool complete = is_complete(st);
            const bool drop = !first_iter && refill_all && !complete && !in_flight(st);
            if (!(first_iter || complete || drop)) {
                tpos[s] = -1;
                continue;
            }
            if (!first_iter) {
                if (complete) {
                    if (st == kMiss) ++m;
                    else if (st != kRmwAbort) c += (unsigned long long)(*reinterpret_cast<uint16_t *>(op + 16) >> 1);
                    if (st == kPutComplete) ++wr;
                    if (st == kRmwAbort) ++ab;
                }
                if (drop) ++dr;
                op[8] = kEmpty;   // reset op bucket: no_coales = 1, state = opcode = ST_EMPTY
                op[9] = kEmpty;
            }
            uint32_t id;
            uint8_t oc;
            cmd(it, id, oc);
            if (oc != kOpRmw) {   // coalesce while the command's hot id has a live op of its opcode
                for (;;) {
                    cmd(it, id, oc);
                    const int arr = oc == kOpGet ? 0 : kHotKeys;
                    if (id < (uint32_t)kHotKeys && hp[arr + id] != 0xFF &&
                        sb[(uint32_t)hp[arr + id] * op_size + 8] == oc) {
                        uint16_t *nc = reinterpret_cast<uint16_t *>(sb + (uint32_t)hp[arr + id] * op_size + 16);
                        *nc = (uint16_t)((*nc & 1u) | ((((*nc >> 1) + 1u) & 0x7FFFu) << 1));
                        ++it;
                    } else {
                        break;
                    }
                }
                if (id < (uint32_t)kHotKeys) hp[(oc == kOpGet ? 0 : kHotKeys) + id] = (uint8_t)s;
            }
            tpos[s] = (int32_t)it;
            op[8] = oc;
            op[9] = kNew;
            op[10] = oc == kOpGet ? 0 : (uint8_t)(st_value >> shift);
            // no_coales := 1 (0 on the first pass, where refill_ops does not reset it), RMW_flag
            *reinterpret_cast<uint16_t *>(op + 16) = (uint16_t)((oc == kOpRmw ? 1u : 0u) | (first_iter ? 0u : 2u));
            ++it;
        }
        cursor[w] = (uint32_t)((base + it) % (uint32_t)tlen);
        tot[0] = c;
        tot[1] = m;
        tot[2] = wr;
        tot[3] = dr;
        tot[4] = ab;
    }
    __syncthreads();
    if (i < stride && tpos[i] >= 0) {   // key, timestamp, value of the refilled slots
        uint8_t *op = sb + (uint32_t)i * op_size;
        const uint32_t k = (uint32_t)tpos[i];
        const int64_t t = (int64_t)w * tlen + (int64_t)((base + k) % (uint32_t)tlen);
        *reinterpret_cast<uint64_t *>(op) = tkey[t];
        const uint8_t oc = op[8];
        if (oc == kOpGet && (flags & HKV_WL_READ_TS_RESET)) {
            op[11] = 0;
            *reinterpret_cast<uint32_t *>(op + 12) = 0;
        }
        if (oc != kOpGet) {
            const uint8_t v = (uint8_t)('a' + machine_id);
            for (uint32_t q = 0; q < st_value; ++q) op[kOpValueOff + q] = v;
        }
    }
    if (opc_out && i < stride) opc_out[(int64_t)w * stride + i] = sb[(uint32_t)i * op_size + 8];
    if (i < kCounters && tot[i]) {
        unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + (w % kStripes) * 16;
        atomicAdd(&stripe[i], tot[i]);
    }
    for (int k = i; k < 2 * kHotKeys; k += 256) hot[(int64_t)w * 2 * kHotKeys + k] = hp[k];
    __syncthreads();
    for (int k = i; k < words; k += 256) gslab[k] = slab[k];
}

// k_refill for big ops (312 B): staging a 78-KB slab per workgroup caps occupancy at two
// workgroups per CU, so each thread edits its own op in place instead -- the same bytes as
// k_refill (key, opcode, state, val_len, flags, and the value of a write), 8-B stores.
__global__ __launch_bounds__(256) void k_refill_direct(uint8_t *ops, int32_t stride, uint32_t op_size,
                                                       uint32_t st_value, uint32_t shift, const uint64_t *tkey,
                                                       const uint8_t *top, int32_t tlen, uint32_t *cursor,
                                                       uint32_t machine_id, int32_t first_iter, uint32_t rflags,
                                                       unsigned long long *counters, uint8_t *opc_out,
                                                       uint8_t *states)
{
    const bool refill_all = (rflags & HKV_WL_REFILL_ALL) != 0;
    const int w = blockIdx.x, i = threadIdx.x;
    const bool live = i < stride;
    const int64_t e = (int64_t)w * stride + (live ? i : 0);
    uint8_t *op = ops + e * op_size;
    // states: the caller's state mirror (every op's state byte, kept by the batches and marshals),
    // read instead of the op, so a slot that is not refilled is not touched at all (312-B ops: one
    // line each), and the refilled ones are only written
    const uint8_t st = live ? (states ? states[e] : op[9]) : 0;
    const bool complete = is_complete(st);
    const bool drop = live && !first_iter && refill_all && !complete && !in_flight(st);
    const bool done = live && (first_iter || complete || drop);
    const int commits = (live && complete && !first_iter && st != kMiss && st != kRmwAbort) ? 1 : 0;
    const int misses = (live && !first_iter && st == kMiss) ? 1 : 0;
    const int writes = (live && !first_iter && st == kPutComplete) ? 1 : 0;
    int total;
    const int rank = block_rank(done, total);
    const uint32_t base = cursor[w];
    const int c = block_sum(commits), m = block_sum(misses), wr = block_sum(writes), dr = block_sum(drop ? 1 : 0);
    const int ab = block_sum((live && !first_iter && st == kRmwAbort) ? 1 : 0);
    if (i == 0) {
        cursor[w] = (uint32_t)((base + (uint32_t)total) % (uint32_t)tlen);
        unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + (w % kStripes) * 16;
        if (c) atomicAdd(&stripe[0], (unsigned long long)c);
        if (m) atomicAdd(&stripe[1], (unsigned long long)m);
        if (wr) atomicAdd(&stripe[2], (unsigned long long)wr);
        if (dr) atomicAdd(&stripe[3], (unsigned long long)dr);
        if (ab) atomicAdd(&stripe[4], (unsigned long long)ab);
    }
    const int64_t t = (int64_t)w * tlen + (int64_t)((base + (uint32_t)rank) % (uint32_t)tlen);
    const uint8_t oc = done ? top[t] : (uint8_t)kOpGet;
    const uint16_t flags = (uint16_t)((oc == kOpRmw ? 1u : 0u) | (first_iter ? 0u : 2u));  // RMW_flag, no_coales
    if (done) {
        *reinterpret_cast<uint64_t *>(op) = tkey[t];
        // bytes 8..10 (opcode, state, val_len) of the second header word; 11..15 keep their bytes
        uint64_t *h1 = reinterpret_cast<uint64_t *>(op + 8);
        const uint64_t vl = oc == kOpGet ? 0 : (uint8_t)(st_value >> shift);
        // a GET's timestamp (bytes 11..15) is reset under HKV_WL_READ_TS_RESET (inline-util.h:268-272)
        const bool reset = oc == kOpGet && (rflags & HKV_WL_READ_TS_RESET);
        if (states) {   // stores only (no read of the op's line)
            op[8] = oc;
            op[9] = kNew;
            op[10] = (uint8_t)vl;
            if (reset) {
                op[11] = 0;
                *reinterpret_cast<uint32_t *>(op + 12) = 0;
            }
            states[e] = kNew;
        } else {
            const uint64_t keep = reset ? 0ull : ~0xFFFFFFull;
            *h1 = (*h1 & keep) | oc | ((uint64_t)kNew << 8) | (vl << 16);
        }
        if (oc == kOpGet) *reinterpret_cast<uint16_t *>(op + 16) = flags;
    }
    // the opcode mirror (with the state mirror, a slot that is not refilled keeps its mirror byte)
    if (opc_out && live && (done || !states)) opc_out[(int64_t)w * stride + i] = done ? oc : op[8];
    // the values of the writes, one op at a time per wave: lane k stores 8-B word k of bytes
    // 16 .. 18 + st_value (word 0 carries the flags), the tail bytes go to the lanes after them
    const uint64_t vv = 0x0101010101010101ull * (uint8_t)('a' + machine_id);
    const uint32_t span = kOpValueOff - 16 + st_value;
    const int nfull = (int)(span / 8), tail = (int)(span % 8);
    const int lane = threadIdx.x & 63;
    uint8_t *wave_ops = ops + ((int64_t)w * stride + (threadIdx.x & ~63)) * op_size;
    unsigned long long todo = __ballot(done && oc != kOpGet);
    while (todo) {
        const int j = __ffsll((long long)todo) - 1;
        todo &= todo - 1;
        const uint16_t fj = (uint16_t)__shfl((int)flags, j, 64);
        uint8_t *oj = wave_ops + (int64_t)j * op_size + 16;
        if (lane < nfull)
            *reinterpret_cast<uint64_t *>(oj + 8 * lane) = lane == 0 ? ((uint64_t)fj | (vv << 16)) : vv;
        else if (lane < nfull + tail)
            oj[8 * nfull + (lane - nfull)] = (uint8_t)vv;
    }
}

// 16 bytes at an 8-byte aligned address: one dwordx4 access (op headers, 16-B messages)
struct __attribute__((aligned(8))) W16 {
    uint64_t a, b;
};
// header word (bytes 8..15) with opcode (byte 8) and state/sender (byte 9) replaced
__device__ __forceinline__ uint64_t with_op_state(uint64_t h, uint8_t op, uint8_t st)
{
    return (h & ~0xFFFFull) | op | ((uint64_t)st << 8);
}

// ---- one wave per worker (stride <= 256: slot r * 64 + lane, four rows): ranks and counts come
// from ballots, with no block barrier, so a CU holds 32 workers in flight instead of 8 -- these
// kernels are a few dependent loads per worker, bound by latency, not bytes.
__device__ __forceinline__ void wave_ranks(const unsigned long long *b, int lane, int *rank, int &total)
{
    const unsigned long long lower = (1ull << lane) - 1ull;
    int before = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        rank[r] = before + __popcll(b[r] & lower);
        before += __popcll(b[r]);
    }
    total = before;
}

// refill_ops as a plan (hkv_wl_refill_plan): the same decisions, cursors and counts as k_refill,
// made from the state mirror (one byte per op instead of every op's line); each refilled
// slot gets a patch (hkv_batch_desc.d_patch) that the next local launch applies as it reads the op,
// so the op slab is read and written once per round (by that launch) instead of twice.
// One wave per WPW workers: all their state loads, then all their trace loads, are in flight
// together (a wave's work is two dependent loads; with WPW = 2 the 16384 workers of configs[1] fit
// the chip's 8192 wave slots in one pass instead of two).
#ifdef HKV_PLAN_NUM_SGPR
#define HKV_PLAN_SGPR_ATTR __attribute__((amdgpu_num_sgpr(HKV_PLAN_NUM_SGPR)))
#else
#define HKV_PLAN_SGPR_ATTR
#endif
struct PlanArgs {   // hkv_wl_refill_plan's arguments
    uint8_t *states;
    int32_t n_workers, stride;
    uint32_t st_value, shift;
    const uint64_t *tkey;
    const uint8_t *top;
    int32_t tlen;
    uint32_t *cursor;
    uint32_t machine_id, flags;
    unsigned long long *counters;
    uint8_t *opc, *patch;
};
// (block bx of the plan's grid; every lane of a wave calls it)
template <int WPW>
__device__ __forceinline__ void refill_plan_body(const PlanArgs &pa, int bx)
{
    uint8_t *states = pa.states;
    const int32_t n_workers = pa.n_workers, stride = pa.stride, tlen = pa.tlen;
    const uint32_t st_value = pa.st_value, shift = pa.shift, machine_id = pa.machine_id, flags = pa.flags;
    const uint64_t *tkey = pa.tkey;
    const uint8_t *top = pa.top;
    uint32_t *cursor = pa.cursor;
    unsigned long long *counters = pa.counters;
    uint8_t *opc = pa.opc, *patch = pa.patch;
    const int lane = threadIdx.x & 63;
    const int wb = (bx * 4 + (int)(threadIdx.x >> 6)) * WPW;
    if (wb >= n_workers) return;
    uint8_t st[WPW][4];
    uint32_t base[WPW];
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        const bool wl = wb + v < n_workers;
        const int64_t e0 = (int64_t)(wb + v) * stride;
#pragma unroll
        for (int r = 0; r < 4; ++r) st[v][r] = wl && r * 64 + lane < stride ? states[e0 + r * 64 + lane] : 0;
        base[v] = wl ? cursor[wb + v] : 0;
    }
    unsigned long long bd[WPW][4];
    int rank[WPW][4];
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        const int w = wb + v;
        const bool wl = w < n_workers;
        int c = 0, m = 0, wr = 0, dr = 0, ab = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const bool live = wl && r * 64 + lane < stride;
            const uint8_t x = st[v][r];
            const bool complete = is_complete(x);
            const bool drop = live && (flags & HKV_WL_REFILL_ALL) && !complete && !in_flight(x);
            bd[v][r] = __ballot(live && (complete || drop));
            c += __popcll(__ballot(live && complete && x != kMiss && x != kRmwAbort));
            m += __popcll(__ballot(live && x == kMiss));
            wr += __popcll(__ballot(live && x == kPutComplete));
            dr += __popcll(__ballot(drop));
            ab += __popcll(__ballot(live && x == kRmwAbort));
        }
        int total;
        wave_ranks(bd[v], lane, rank[v], total);
        if (lane == 0 && wl) {
            cursor[w] = (uint32_t)((base[v] + (uint32_t)total) % (uint32_t)tlen);
            unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + (w % kStripes) * 16;
            if (c) atomicAdd(&stripe[0], (unsigned long long)c);
            if (m) atomicAdd(&stripe[1], (unsigned long long)m);
            if (wr) atomicAdd(&stripe[2], (unsigned long long)wr);
            if (dr) atomicAdd(&stripe[3], (unsigned long long)dr);
            if (ab) atomicAdd(&stripe[4], (unsigned long long)ab);
        }
    }
    uint8_t oc[WPW][4];
    uint64_t key[WPW][4];
#pragma unroll
    for (int v = 0; v < WPW; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const bool rf = (bd[v][r] >> lane) & 1ull;
            const int64_t t = (int64_t)(wb + v) * tlen + (int64_t)((base[v] + (uint32_t)rank[v][r]) % (uint32_t)tlen);
            oc[v][r] = rf ? top[t] : (uint8_t)0;
            key[v][r] = rf ? tkey[t] : 0ull;
        }
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        if (wb + v >= n_workers) break;
        const int64_t e0 = (int64_t)(wb + v) * stride;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = r * 64 + lane;
            if (i >= stride) continue;
            const int64_t e = e0 + i;
            W16 p{0, 0};
            if ((bd[v][r] >> lane) & 1ull) {
                const uint8_t o = oc[v][r];
                const bool get = o == kOpGet;
                p.a = key[v][r];
                p.b = (uint64_t)o | ((uint64_t)(get ? 0u : (uint8_t)(st_value >> shift)) << 8) |
                      ((uint64_t)((o == kOpRmw ? 1u : 0u) | 2u) << 16) |
                      ((uint64_t)(get ? 0u : (uint8_t)('a' + machine_id)) << 32) |
                      ((uint64_t)(get && (flags & HKV_WL_READ_TS_RESET) ? 1u : 0u) << 40) | (1ull << 48);
                opc[e] = o;
            }
            *reinterpret_cast<W16 *>(patch + e * 16) = p;
        }
    }
}

template <int WPW>
__global__ __launch_bounds__(256) HKV_PLAN_SGPR_ATTR void k_refill_plan_w(PlanArgs pa)
{
    refill_plan_body<WPW>(pa, blockIdx.x);
}

// k_refill_direct from the state mirror (hkv_wl_refill_st: big ops refilled in place), one wave per
// worker as k_refill_plan_w: ranks and counts from ballots instead of six block reductions, every
// trace load of the worker in flight together, then the stores -- key, opcode, ST_NEW, val_len,
// a GET's flags and timestamp reset, the state and opcode mirrors, and a write's value, one op at
// a time per wave (lane k stores 8-B word k of bytes 16 .. 18 + st_value, word 0 the flags).
__global__ __launch_bounds__(256) void k_refill_st_w(uint8_t *ops, int32_t n_workers, int32_t stride,
                                                     uint32_t op_size, uint32_t st_value, uint32_t shift,
                                                     const uint64_t *tkey, const uint8_t *top, int32_t tlen,
                                                     uint32_t *cursor, uint32_t machine_id, uint32_t rflags,
                                                     unsigned long long *counters, uint8_t *opc_out, uint8_t *states)
{
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (w >= n_workers) return;
    const int64_t e0 = (int64_t)w * stride;
    uint8_t st[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) st[r] = r * 64 + lane < stride ? states[e0 + r * 64 + lane] : 0;
    const uint32_t base = cursor[w];
    unsigned long long bd[4];
    int c = 0, m = 0, wr = 0, dr = 0, ab = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const bool live = r * 64 + lane < stride;
        const bool complete = is_complete(st[r]);
        const bool drop = live && (rflags & HKV_WL_REFILL_ALL) && !complete && !in_flight(st[r]);
        bd[r] = __ballot(live && (complete || drop));
        c += __popcll(__ballot(live && complete && st[r] != kMiss && st[r] != kRmwAbort));
        m += __popcll(__ballot(live && st[r] == kMiss));
        wr += __popcll(__ballot(live && st[r] == kPutComplete));
        dr += __popcll(__ballot(drop));
        ab += __popcll(__ballot(live && st[r] == kRmwAbort));
    }
    int rank[4], total;
    wave_ranks(bd, lane, rank, total);
    if (lane == 0) {
        cursor[w] = (uint32_t)((base + (uint32_t)total) % (uint32_t)tlen);
        unsigned long long *stripe = counters + HKV_WL_STRIPE_BASE + (w % kStripes) * 16;
        if (c) atomicAdd(&stripe[0], (unsigned long long)c);
        if (m) atomicAdd(&stripe[1], (unsigned long long)m);
        if (wr) atomicAdd(&stripe[2], (unsigned long long)wr);
        if (dr) atomicAdd(&stripe[3], (unsigned long long)dr);
        if (ab) atomicAdd(&stripe[4], (unsigned long long)ab);
    }
    uint8_t oc[4];
    uint64_t key[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const bool rf = (bd[r] >> lane) & 1ull;
        const int64_t t = (int64_t)w * tlen + (int64_t)((base + (uint32_t)rank[r]) % (uint32_t)tlen);
        oc[r] = rf ? top[t] : (uint8_t)kOpGet;
        key[r] = rf ? tkey[t] : 0ull;
    }
    const uint64_t vv = 0x0101010101010101ull * (uint8_t)('a' + machine_id);
    const uint32_t span = kOpValueOff - 16 + st_value;
    const int nfull = (int)(span / 8), tail = (int)(span % 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const bool rf = (bd[r] >> lane) & 1ull;
        const int64_t e = e0 + r * 64 + lane;
        const uint16_t flags = (uint16_t)((oc[r] == kOpRmw ? 1u : 0u) | 2u);   // RMW_flag, no_coales
        if (rf) {
            uint8_t *op = ops + e * op_size;
            *reinterpret_cast<uint64_t *>(op) = key[r];
            const bool get = oc[r] == kOpGet;
            op[8] = oc[r];
            op[9] = kNew;
            op[10] = get ? (uint8_t)0 : (uint8_t)(st_value >> shift);
            if (get && (rflags & HKV_WL_READ_TS_RESET)) {   // inline-util.h:268-272
                op[11] = 0;
                *reinterpret_cast<uint32_t *>(op + 12) = 0;
            }
            if (get) *reinterpret_cast<uint16_t *>(op + 16) = flags;
            states[e] = kNew;
            opc_out[e] = oc[r];
        }
        unsigned long long todo = __ballot(rf && oc[r] != kOpGet);
        uint8_t *row = ops + (e0 + r * 64) * op_size;
        while (todo) {
            const int j = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const uint16_t fj = (uint16_t)__shfl((int)flags, j, 64);
            uint8_t *oj = row + (int64_t)j * op_size + 16;
            if (lane < nfull)
                *reinterpret_cast<uint64_t *>(oj + 8 * lane) = lane == 0 ? ((uint64_t)fj | (vv << 16)) : vv;
            else if (lane < nfull + tail)
                oj[8 * nfull + (lane - nfull)] = (uint8_t)vv;
        }
    }
}

// The sent ops of one worker (bit set in bs, rank below cap; e0: the worker's first op) copied as INVs to
// out_w + rank * op_size, four lanes per op (16 bytes a lane; op_size <= 64) from a list in LDS (lst, 256
// words for the wave), then marked in flight in the op and the state mirror. The whole wave calls it.
__device__ __forceinline__ void wave_copy_invs(uint8_t *ops, int64_t e0, const unsigned long long *bs, const int *rank,
                                               int cap, int total, const uint8_t *st, uint32_t op_size, uint8_t *out_w,
                                               uint32_t machine_id, uint8_t *states, uint32_t *lst, int lane)
{
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (((bs[r] >> lane) & 1ull) && rank[r] < cap) lst[rank[r]] = (uint32_t)(r * 64 + lane) | ((uint32_t)st[r] << 16);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nsend = total < cap ? total : cap, q = lane & 3;
    const uint32_t b0 = 16u * (uint32_t)q;
    for (int j = lane >> 2; j < nsend; j += 16) {
        const uint32_t li = lst[j];
        const int64_t e = e0 + (int64_t)(li & 0xFFFFu);
        uint8_t *op = ops + e * op_size;
        uint8_t *dst = out_w + (int64_t)j * op_size;
        if (b0 + 16 <= op_size) {
            W16 h = *reinterpret_cast<const W16 *>(op + b0);
            if (q == 0) h.b = with_op_state(h.b, kOpInv, (uint8_t)machine_id);
            *reinterpret_cast<W16 *>(dst + b0) = h;
        } else if (b0 + 8 <= op_size) {
            *reinterpret_cast<uint64_t *>(dst + b0) = *reinterpret_cast<const uint64_t *>(op + b0);
        }
        if (q == 0) {
            const uint8_t x = (uint8_t)(li >> 16);
            const uint8_t ns = x == kPutSuccess ? kInProgressPut : x == kRmwSuccess ? kInProgressRmw
                             : x == kReplaySuccess ? kInProgressReplay : kOpMembComplete;
            op[9] = ns;
            if (states) states[e] = ns;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();   // the list is rewritten for the next worker
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// k_marshal_invs for ops of at most 64 bytes, one wave per WPW workers (their state loads all in
// flight together, see k_refill_plan_w)
template <int WPW, bool WAVE = false>
__global__ __launch_bounds__(256) void k_marshal_invs_w(uint8_t *ops, int32_t n_workers, int32_t stride,
                                                        uint32_t op_size, uint8_t *out, int32_t out_stride,
                                                        int32_t *count, uint32_t machine_id,
                                                        unsigned long long *held, const int32_t *aq_n,
                                                        int32_t r_alive, uint8_t *states)
{
    __shared__ uint32_t s_list[4][256];   // WAVE: each wave's sent ops (index in the worker | state << 16)
    const int lane = threadIdx.x & 63;
    const int wb = (blockIdx.x * 4 + (int)(threadIdx.x >> 6)) * WPW;
    if (wb >= n_workers) return;
    uint8_t st[WPW][4];
    int aqn[WPW];
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        const bool wl = wb + v < n_workers;
        const int64_t e0 = (int64_t)(wb + v) * stride;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = r * 64 + lane;
            st[v][r] = wl && i < stride ? (states ? states[e0 + i] : ops[(e0 + i) * op_size + 9]) : 0;
        }
        aqn[v] = aq_n && wl ? aq_n[wb + v] : 0;
    }
#pragma unroll
    for (int v = 0; v < WPW; ++v) {
        const int w = wb + v;
        if (w >= n_workers) break;
        const int64_t e0 = (int64_t)w * stride;
        unsigned long long bs[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint8_t x = st[v][r];
            bs[r] = __ballot(r * 64 + lane < stride &&
                             (x == kPutSuccess || x == kRmwSuccess || x == kReplaySuccess || x == kOpMembChange));
        }
        int rank[4], total;
        wave_ranks(bs, lane, rank, total);
        const int cap = aq_n ? max(0, out_stride - aqn[v] / max(1, r_alive)) : out_stride;
        if (lane == 0) {
            count[w] = total < cap ? total : cap;
            if (total > cap && held) atomicAdd(held, (unsigned long long)(total - cap));
        }
        if (WAVE) {   // the sent ops listed in LDS, then copied four lanes per op, 16 bytes per lane
            wave_copy_invs(ops, e0, bs, rank, cap, total, st[v], op_size, out + (int64_t)w * out_stride * op_size,
                           machine_id, states, s_list[threadIdx.x >> 6], lane);
            continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (!((bs[r] >> lane) & 1ull) || rank[r] >= cap) continue;
            const int64_t e = e0 + r * 64 + lane;
            uint8_t *op = ops + e * op_size;
            uint8_t *dst = out + ((int64_t)w * out_stride + rank[r]) * op_size;
            const W16 h = *reinterpret_cast<const W16 *>(op);
            *reinterpret_cast<W16 *>(dst) = W16{h.a, with_op_state(h.b, kOpInv, (uint8_t)machine_id)};
            uint32_t k = 16;
            for (; k + 16 <= op_size; k += 16) *reinterpret_cast<W16 *>(dst + k) = *reinterpret_cast<const W16 *>(op + k);
            if (k < op_size) *reinterpret_cast<uint64_t *>(dst + k) = *reinterpret_cast<const uint64_t *>(op + k);
            const uint8_t x = st[v][r];
            const uint8_t ns = x == kPutSuccess ? kInProgressPut : x == kRmwSuccess ? kInProgressRmw
                             : x == kReplaySuccess ? kInProgressReplay : kOpMembComplete;
            op[9] = ns;
            if (states) states[e] = ns;
        }
    }
}

// The INV marshals copy the sent ops four lanes per op from a list in LDS (round 4: 4.18 -> 4.23 G ops/s
// against one lane per op), and the wave-per-worker workload kernels take two workers per wave (round 4:
// refill plan 34 -> 31 us, marshal 34 -> 33 us against one)
static bool marshal_wave() { return true; }
static int wl_wpw() { return 2; }

// wings_issue_pkts(inv) with the INV callbacks of hermes_worker.c:12-65. At most out_stride
// INVs per worker go out per round (the send credits); the rest keep their state and are
// sent by a later round, as with the reference's credit-limited wings sends.
__global__ __launch_bounds__(256) void k_marshal_invs(uint8_t *ops, int32_t stride, uint32_t op_size, uint8_t *out,
                                                      int32_t out_stride, int32_t *count, uint32_t machine_id,
                                                      unsigned long long *held, const int32_t *aq_n, int32_t r_alive,
                                                      uint8_t *states)
{
    const int w = blockIdx.x, i = threadIdx.x;
    const bool live = i < stride;
    uint8_t *op = ops + ((int64_t)w * stride + i) * op_size;
    // the local batch's state mirror, when it kept one, instead of every op's line
    uint8_t st = live ? (states ? states[(int64_t)w * stride + i] : op[9]) : 0;
    bool send = live && (st == kPutSuccess || st == kRmwSuccess || st == kReplaySuccess || st == kOpMembChange);
    int total;
    int rank = block_rank(send, total);
    // INV credits: ACK packets return them (wings.h:426-540), so INVs whose ACKs this worker has not
    // applied yet (aq_n / r_alive of them: held while VALs were outstanding) still hold theirs
    const int cap = aq_n ? max(0, out_stride - aq_n[w] / max(1, r_alive)) : out_stride;
    if (i == 0) {
        count[w] = total < cap ? total : cap;
        if (total > cap && held) atomicAdd(held, (unsigned long long)(total - cap));
    }
    out_stride = cap > 0 ? out_stride : 0;  // row stride unchanged; rank < cap below
    const int send_cap = cap;
    if (op_size > 64) {  // big ops: one op at a time per wave, 8-B word k by lane k
        const int lane = i & 63;
        const int words = (int)(op_size / 8);
        uint8_t *wave_ops = ops + ((int64_t)w * stride + (i & ~63)) * op_size;
        unsigned long long todo = __ballot(send && rank < send_cap);
        while (todo) {
            const int j = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const int rj = __shfl(rank, j, 64);
            const uint64_t *src = reinterpret_cast<const uint64_t *>(wave_ops + (int64_t)j * op_size);
            uint64_t *dst = reinterpret_cast<uint64_t *>(out + ((int64_t)w * out_stride + rj) * op_size);
            for (int k = lane; k < words; k += 64) {
                const uint64_t v = src[k];
                dst[k] = k == 1 ? with_op_state(v, kOpInv, (uint8_t)machine_id) : v;
            }
        }
        if (send && rank < send_cap) {
            const uint8_t ns = st == kPutSuccess ? kInProgressPut : st == kRmwSuccess ? kInProgressRmw
                             : st == kReplaySuccess ? kInProgressReplay : kOpMembComplete;
            op[9] = ns;
            if (states) states[(int64_t)w * stride + i] = ns;
        }
        return;
    }
    if (!send || rank >= send_cap) return;
    uint8_t *dst = out + ((int64_t)w * out_stride + rank) * op_size;
    // 16-B words; the header word is rewritten in registers
    const W16 h = *reinterpret_cast<const W16 *>(op);
    *reinterpret_cast<W16 *>(dst) = W16{h.a, with_op_state(h.b, kOpInv, (uint8_t)machine_id)};
    uint32_t k = 16;
    for (; k + 16 <= op_size; k += 16) *reinterpret_cast<W16 *>(dst + k) = *reinterpret_cast<const W16 *>(op + k);
    if (k < op_size) *reinterpret_cast<uint64_t *>(dst + k) = *reinterpret_cast<const uint64_t *>(op + k);
    const uint8_t ns = st == kPutSuccess ? kInProgressPut : st == kRmwSuccess ? kInProgressRmw
                     : st == kReplaySuccess ? kInProgressReplay : kOpMembComplete;
    op[9] = ns;
    if (states) states[(int64_t)w * stride + i] = ns;   // the mirror stays the ops' state bytes
}

// VALs of the writes and replays a membership change completed: wings_issue_pkts(val) over the
// ops with memb_change_skip_or_get_sender_id / memb_change_copy_and_modify_elem /
// memb_change_modify_elem_after_send (hermes_worker.c:163-203). The callback sets opcode, sender
// and ts of the message; the key is the op's (the 16-B op_meta with opcode and sender replaced).
// *_COMPLETE_SEND_VALS -> PUT_COMPLETE / RMW_COMPLETE / NEW (a replayed GET is issued again).
__global__ __launch_bounds__(256) void k_marshal_memb_vals(uint8_t *ops, int32_t stride, uint32_t op_size,
                                                           uint8_t *out, int32_t out_stride, int32_t *count,
                                                           uint32_t machine_id, uint8_t *states)
{
    const int w = blockIdx.x, i = threadIdx.x;
    const bool live = i < stride;
    uint8_t *op = ops + ((int64_t)w * stride + i) * op_size;
    const uint8_t st = live ? op[9] : 0;
    const bool send = live && (st == kPutCompleteSendVals || st == kRmwCompleteSendVals || st == kReplayCompleteSendVals);
    int total;
    const int rank = block_rank(send, total);
    if (i == 0) count[w] = total < out_stride ? total : out_stride;
    if (!send) return;
    if (rank < out_stride) {
        const W16 h = *reinterpret_cast<const W16 *>(op);
        *reinterpret_cast<W16 *>(out + ((int64_t)w * out_stride + rank) * kOpMetaSize) =
            W16{h.a, with_op_state(h.b, kOpVal, (uint8_t)machine_id)};
    }
    const uint8_t ns = st == kPutCompleteSendVals ? kPutComplete : st == kRmwCompleteSendVals ? kRmwComplete : kNew;
    op[9] = ns;
    if (states) states[(int64_t)w * stride + i] = ns;
}

// The largest of n counts, stored straight into pinned host memory (one workgroup): the host
// reads a round's ACK width without a reduction kernel and a copy.
__global__ __launch_bounds__(1024) void k_max_to_host(const int32_t *counts, int32_t n, int32_t *out)
{
    __shared__ int32_t part[16];
    int32_t m = 0;
    for (int32_t i = threadIdx.x; i < n; i += 1024) m = counts[i] > m ? counts[i] : m;
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t u = __shfl_down(m, o, 64);
        m = u > m ? u : m;
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 16; ++k) m = part[k] > m ? part[k] : m;
        *out = m;
    }
}

// ACKs for received INV rows: row r holds in_count[r] INVs (row stride C); its ACKs are
// compacted to the front of output row r (ack_skip_or_get_sender_id + ack_copy_and_modify_elem
// + ack_modify_elem_after_send, hermes_worker.c:67-110)
__global__ __launch_bounds__(256) void k_marshal_acks_rows(uint8_t *invs, const int32_t *in_count, int32_t C,
                                                           uint32_t op_size, uint8_t *out, uint32_t ack_size,
                                                           int32_t *out_count, uint32_t machine_id)
{
    const int64_t r = blockIdx.x;
    const int n = in_count[r];
    int base = 0;
    for (int j0 = 0; j0 < n; j0 += 256) {
        const int j = j0 + (int)threadIdx.x;
        uint8_t *x = invs + (r * C + j) * (int64_t)op_size;
        const uint8_t oc = j < n ? x[8] : 0;
        const bool send = j < n && (oc == kInvSuccess || (oc == kOpInvAbort && ack_size >= op_size));
        int total;
        const int rank = block_rank(send, total);
        if (send) {
            uint8_t *y = out + (r * C + base + rank) * (int64_t)ack_size;
            const uint32_t words = (oc == kInvSuccess ? kOpMetaSize : op_size) / 8;
            for (uint32_t k = 0; k < words; ++k)
                reinterpret_cast<uint64_t *>(y)[k] = reinterpret_cast<const uint64_t *>(x)[k];
            y[9] = (uint8_t)machine_id;
            y[8] = oc == kInvSuccess ? kOpAck : kOpInvAbort;
        }
        if (j < n && (oc == kInvSuccess || oc == kOpInvAbort || oc == kOpMembChange)) x[8] = kEmpty;
        base += total;
    }
    if (threadIdx.x == 0) out_count[r] = base;
}

// [P][W][C] rows with counts[P][W] -> per-worker batches [W][out_stride], peers' elements
// back to back (one worker's receive poll over all peers)
__global__ __launch_bounds__(256) void k_regroup(const uint8_t *in, const int32_t *counts, int32_t P, int32_t W,
                                                 int32_t C, uint32_t esz, uint8_t *out, int32_t out_stride,
                                                 int32_t *out_count)
{
    const int w = blockIdx.x;
    int off = 0;
    for (int p = 0; p < P; ++p) {
        const int n = counts[(int64_t)p * W + w];
        const uint64_t *src = reinterpret_cast<const uint64_t *>(in + ((int64_t)p * W + w) * C * esz);
        uint64_t *dst = reinterpret_cast<uint64_t *>(out + ((int64_t)w * out_stride + off) * esz);
        const int words = (int)((uint32_t)n * esz / 8u);
        for (int k = threadIdx.x; k < words; k += 256) dst[k] = src[k];
        off += n;
    }
    if (threadIdx.x == 0) out_count[w] = off;
}

// VALs of the writes an ACK batch completed (ST_LAST_ACK_SUCCESS), compacted per worker into
// [W][C]; the ACK elements become ST_EMPTY (hermes_worker.c:112-160)
__global__ __launch_bounds__(64) void k_collect_vals(uint8_t *acks, const int32_t *count, int32_t stride,
                                                     uint32_t ack_size, uint8_t *out, int32_t C, int32_t *out_count,
                                                     uint32_t machine_id, unsigned long long *held,
                                                     const int32_t *offsets, int32_t n_blocks, int64_t block_stride)
{
    // one wave per worker (a worker's round has a few dozen ACKs)
    const int64_t w = blockIdx.x;
    const int lane = (int)threadIdx.x;
    // rows: worker w's ACKs at w * stride, count[w] of them; packed: [offsets[w], offsets[w+1]);
    // n_blocks > 1: peer-major blocks of block_stride elements (0: offsets[gridDim.x], back to back),
    // worker w's part in each
    const int n = offsets ? offsets[w + 1] - offsets[w] : count[w];
    const int64_t block = n_blocks > 1 ? (block_stride > 0 ? block_stride : (int64_t)offsets[gridDim.x]) : 0;
    int base = 0;
    for (int blk = 0; blk < n_blocks; ++blk)
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int64_t row = (offsets ? (int64_t)offsets[w] : w * stride) + blk * block;
        const int j = j0 + lane;
        uint8_t *x = acks + (row + j) * (int64_t)ack_size;
        const uint8_t oc = j < n ? x[8] : 0;
        const bool send = j < n && val_sends(oc);
        const unsigned long long m = __ballot(send);
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        if (send && base + rank < C) {
            uint64_t *y = reinterpret_cast<uint64_t *>(out + (w * C + base + rank) * (int64_t)kOpMetaSize);
            y[0] = reinterpret_cast<const uint64_t *>(x)[0];
            uint64_t h = reinterpret_cast<const uint64_t *>(x)[1];
            y[1] = (h & ~0xFFFFull) | kOpVal | ((uint64_t)(machine_id & 0xFF) << 8);
        }
        if (j < n && oc != kEmpty) x[8] = kEmpty;
        base += __popcll(m);
    }
    if (lane == 0) {
        out_count[w] = base < C ? base : C;
        if (base > C && held) atomicAdd(held, (unsigned long long)(base - C));
    }
}

// ack_skip_or_get_sender_id + ack_copy_and_modify_elem + ack_modify_elem_after_send
__global__ void k_marshal_acks(uint8_t *invs, int64_t n, uint32_t op_size, uint8_t *out, uint32_t ack_size,
                               uint32_t machine_id)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *x = invs + i * op_size;
    uint8_t *y = out + i * ack_size;
    const W16 h = *reinterpret_cast<const W16 *>(x);
    const uint8_t oc = (uint8_t)h.b;
    if (oc == kInvSuccess || (oc == kOpInvAbort && ack_size >= op_size)) {
        *reinterpret_cast<W16 *>(y) =
            W16{h.a, with_op_state(h.b, oc == kInvSuccess ? kOpAck : kOpInvAbort, (uint8_t)machine_id)};
        if (oc != kInvSuccess)
            for (uint32_t k = 16; k < op_size; k += 8)
                *reinterpret_cast<uint64_t *>(y + k) = *reinterpret_cast<const uint64_t *>(x + k);
    } else {
        y[8] = kEmpty;
    }
    if (oc == kInvSuccess || oc == kOpInvAbort || oc == kOpMembChange) x[8] = kEmpty;
}

// val_skip_or_get_sender_id + val_copy_and_modify_elem + val_modify_elem_after_send
__global__ void k_marshal_vals(uint8_t *acks, int64_t n, uint32_t ack_size, uint8_t *out, uint32_t machine_id)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *x = acks + i * ack_size;
    uint8_t *y = out + i * kOpMetaSize;
    const W16 h = *reinterpret_cast<const W16 *>(x);
    const uint8_t oc = (uint8_t)h.b;
    if (val_sends(oc)) *reinterpret_cast<W16 *>(y) = W16{h.a, with_op_state(h.b, kOpVal, (uint8_t)machine_id)};
    else y[8] = kEmpty;
    x[8] = kEmpty;
}

// ---- packed slabs (replica groups): one contiguous slab per rank instead of [W][C] rows
// exclusive prefix of counts[0..n) into off[0..n], off[n] = the total (one workgroup)
__global__ __launch_bounds__(1024) void k_scan_counts(const int32_t *counts, int32_t n, int32_t *off)
{
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int lo = t * per, hi = min(n, lo + per);
    int32_t sum = 0;
    for (int k = lo; k < hi; ++k) sum += counts[k];
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the per-thread sums
        const int32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = part[t] - sum;
    for (int k = lo; k < hi; ++k) {
        off[k] = run;
        run += counts[k];
    }
    if (t == 1023) off[n] = part[1023];
}

// ---- a rank's INVs straight into its packed slab, at most `cap` of them (replica groups without a
// host read per round): k_count_invs counts each worker's sendable ops (at most C, the INV credits),
// k_scan_cap turns the counts into slab offsets and how many each worker sends within cap, and
// k_marshal_invs_packed copies them to their offsets. INVs past the cap keep their PUT_SUCCESS (or
// RMW/REPLAY_SUCCESS, MEMBERSHIP_CHANGE) state and go out in a later round, as the credit-held ones do.
__device__ __forceinline__ bool inv_sendable(uint8_t st)
{
    return st == kPutSuccess || st == kRmwSuccess || st == kReplaySuccess || st == kOpMembChange;
}

__global__ __launch_bounds__(256) void k_count_invs(const uint8_t *states, int32_t n_workers, int32_t stride,
                                                    int32_t *count)
{
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (w >= n_workers) return;
    int c = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = r * 64 + lane;
        c += __popcll(__ballot(i < stride && inv_sendable(states[(int64_t)w * stride + i])));
    }
    if (lane == 0) count[w] = c;
}

// counts[W] (sendable) -> off[0..W] (off[W] = the slab's total) and sent[W]: worker w sends
// min(count, C, what is left of cap after the workers before it); the rest is added to *held
__global__ __launch_bounds__(1024) void k_scan_cap(const int32_t *counts, int32_t n, int32_t C, int32_t cap,
                                                   int32_t *off, int32_t *sent, unsigned long long *held)
{
    __shared__ int32_t part[1024];
    __shared__ unsigned long long held_s[16];
    const int t = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int lo = t * per, hi = min(n, lo + per);
    int32_t sum = 0;
    for (int k = lo; k < hi; ++k) sum += min(counts[k], C);
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = part[t] - sum;   // uncapped offset of worker lo
    int32_t h = 0;
    for (int k = lo; k < hi; ++k) {
        const int32_t c = counts[k], want = min(c, C);
        const int32_t start = min(run, cap);
        const int32_t s = max(0, min(want, cap - run));
        off[k] = start;
        sent[k] = s;
        h += c - s;
        run += want;
    }
    // the held total: a wave sum, then the 16 waves' (a serial walk over 1024 LDS words took ~20 us)
    unsigned long long hw = (unsigned long long)h;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hw += __shfl_down(hw, o, 64);
    if ((t & 63) == 0) held_s[t >> 6] = hw;
    __syncthreads();
    if (t == 0) {
        unsigned long long tot = 0;
        for (int k = 0; k < 16; ++k) tot += held_s[k];
        if (tot && held) atomicAdd(held, tot);
        off[n] = min(part[1023], cap);
    }
}

// k_marshal_invs_w writing worker w's first sent[w] INVs at out[off[w] ..]
__global__ __launch_bounds__(256) void k_marshal_invs_packed(uint8_t *ops, int32_t n_workers, int32_t stride,
                                                             uint32_t op_size, uint8_t *out, const int32_t *off,
                                                             const int32_t *sent, uint32_t machine_id,
                                                             uint8_t *states, int32_t wave)
{
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (w >= n_workers) return;
    const int64_t e0 = (int64_t)w * stride;
    uint8_t st[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = r * 64 + lane;
        st[r] = i < stride ? states[e0 + i] : 0;
    }
    unsigned long long bs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[r] = __ballot(r * 64 + lane < stride && inv_sendable(st[r]));
    int rank[4], total;
    wave_ranks(bs, lane, rank, total);
    const int cap = sent[w];
    const int64_t base = off[w];
    if (op_size <= 64 && wave) {   // four lanes per op from a list in LDS (HKV_MARSHAL_WAVE)
        __shared__ uint32_t s_list[4][256];
        wave_copy_invs(ops, e0, bs, rank, cap, total, st, op_size, out + base * op_size, machine_id, states,
                       s_list[threadIdx.x >> 6], lane);
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (!((bs[r] >> lane) & 1ull) || rank[r] >= cap) continue;
        const int64_t e = e0 + r * 64 + lane;
        uint8_t *op = ops + e * op_size;
        uint8_t *dst = out + (base + rank[r]) * op_size;
        const W16 h = *reinterpret_cast<const W16 *>(op);
        *reinterpret_cast<W16 *>(dst) = W16{h.a, with_op_state(h.b, kOpInv, (uint8_t)machine_id)};
        uint32_t k = 16;
        for (; k + 16 <= op_size; k += 16) *reinterpret_cast<W16 *>(dst + k) = *reinterpret_cast<const W16 *>(op + k);
        if (k < op_size) *reinterpret_cast<uint64_t *>(dst + k) = *reinterpret_cast<const uint64_t *>(op + k);
        const uint8_t s = st[r];
        const uint8_t ns = s == kPutSuccess ? kInProgressPut : s == kRmwSuccess ? kInProgressRmw
                         : s == kReplaySuccess ? kInProgressReplay : kOpMembComplete;
        op[9] = ns;
        states[e] = ns;
    }
}

// rows [W][C] x esz with counts[W] -> packed[off[w] ..], one workgroup per row
__global__ __launch_bounds__(256) void k_pack_rows(const uint8_t *rows, const int32_t *counts, const int32_t *off,
                                                   int32_t C, uint32_t esz, uint8_t *packed)
{
    const int w = blockIdx.x;
    const int words = (int)((uint32_t)counts[w] * esz / 8u);
    const uint64_t *src = reinterpret_cast<const uint64_t *>(rows + (int64_t)w * C * esz);
    uint64_t *dst = reinterpret_cast<uint64_t *>(packed + (int64_t)off[w] * esz);
    for (int k = threadIdx.x; k < words; k += 256) dst[k] = src[k];
}

// ACKs in the positions of the received INVs ([rows][width], counts[rows]): an ACK (or, with
// RMWs, an INV-abort) where the INV applied, ST_EMPTY elsewhere (also past the row's count),
// so row r of the output lines up with the packed INV slab its coordinator sent
__global__ void k_marshal_acks_aligned(uint8_t *invs, const int32_t *counts, int32_t width, int64_t n,
                                       uint32_t op_size, uint8_t *out, uint32_t ack_size, uint32_t machine_id)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *y = out + i * ack_size;
    // a slot that carries no ACK: ST_EMPTY, with ST_OP_MEMBERSHIP_CHANGE in byte 9, which
    // hermes_skip_ack skips (hermesKV.c:746-750), so a coordinator may apply a whole row as it
    // arrives (ReplicaRound.acks); regrouping drops these slots by their opcode
    if ((int32_t)(i % width) >= counts[i / width]) {
        y[8] = kEmpty;
        y[9] = kOpMembChange;
        return;
    }
    uint8_t *x = invs + i * op_size;
    const W16 h = *reinterpret_cast<const W16 *>(x);
    const uint8_t oc = (uint8_t)h.b;
    if (oc == kInvSuccess || (oc == kOpInvAbort && ack_size >= op_size)) {
        *reinterpret_cast<W16 *>(y) =
            W16{h.a, with_op_state(h.b, oc == kInvSuccess ? kOpAck : kOpInvAbort, (uint8_t)machine_id)};
        if (oc != kInvSuccess)
            for (uint32_t k = 16; k < op_size; k += 8)
                *reinterpret_cast<uint64_t *>(y + k) = *reinterpret_cast<const uint64_t *>(x + k);
    } else {
        y[8] = kEmpty;
        y[9] = kOpMembChange;
    }
    if (oc == kInvSuccess || oc == kOpInvAbort || oc == kOpMembChange) x[8] = kEmpty;
}

// The ACKs returned to this coordinator ([n_peers][width], row p from peer p, lined up with the
// packed INV slab it sent: worker w's INVs at off[w] .. off[w] + count[w]) -> per-worker ACK
// batches [W][out_stride]: the peers' ACKs back to back in peer order, ST_EMPTY slots dropped
__global__ __launch_bounds__(256) void k_regroup_aligned(const uint8_t *in, int32_t n_peers, int32_t width,
                                                         const int32_t *off, const int32_t *count, uint32_t esz,
                                                         uint8_t *out, int32_t out_stride, int32_t *out_count)
{
    const int w = blockIdx.x;
    const int n = count[w];
    int base = 0;
    for (int p = 0; p < n_peers; ++p) {
        for (int j0 = 0; j0 < n; j0 += 256) {
            const int j = j0 + (int)threadIdx.x;
            const uint8_t *x = in + ((int64_t)p * width + off[w] + j) * esz;
            const bool keep = j < n && x[8] != kEmpty;
            int total;
            const int rank = block_rank(keep, total);
            if (keep && base + rank < out_stride) {
                uint8_t *y = out + ((int64_t)w * out_stride + base + rank) * esz;
                for (uint32_t k = 0; k < esz; k += 8)
                    *reinterpret_cast<uint64_t *>(y + k) = *reinterpret_cast<const uint64_t *>(x + k);
            }
            base += total;
        }
    }
    if (threadIdx.x == 0) out_count[w] = base < out_stride ? base : out_stride;
}

// ---- virtual peer replicas
// A virtual peer stands for a replica that runs the same workload as this one. Its INVs of a
// round are its successful writes: at most one per key and round (a second local write of the
// key stalls on op_buffer_index, hermesKV.c:314-356), each with the timestamp its
// update_actions_n_unlock gives (hermesKV.c:100-141): the key's current version + 2 (+4 for a
// plain write in an RMW build) and the peer's id as cid. Keys, values and the dedup are drawn
// once per round index (hkv_wl_gen_peer_round); the timestamps are taken from the table at the
// start of each round (hkv_wl_peer_ts), when every replica holds the same converged state.

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    return x ^ (x >> 33);
}

// open-addressed (peer, id) -> smallest order index, for the first-occurrence dedup
__device__ __forceinline__ uint32_t dedup_slot(const unsigned long long *hk, uint64_t key, uint32_t mask, bool insert)
{
    uint32_t h = (uint32_t)mix64(key) & mask;
    for (;;) {
        unsigned long long cur = hk[h];
        if (cur == key) return h;
        if (cur == 0ull) {
            if (!insert) return 0xFFFFFFFFu;
            cur = atomicCAS(const_cast<unsigned long long *>(hk) + h, 0ull, (unsigned long long)key);
            if (cur == 0ull || cur == key) return h;
        }
        h = (h + 1) & mask;
    }
}

__global__ void k_peer_draw(uint32_t *ids, uint8_t *rmw, unsigned long long *hk, uint32_t *hmin, uint32_t mask,
                            int32_t per_peer, int32_t n_peers, hkv_zipf z, uint32_t rmw_pm, uint32_t round,
                            uint64_t seed, int64_t total)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total) return;
    const int64_t row = (int64_t)per_peer * n_peers;
    const int32_t w = (int32_t)(g / row);
    const int32_t rem = (int32_t)(g - (int64_t)w * row);
    const int32_t r = rem / per_peer, j = rem - r * per_peer;
    const uint64_t r1 = splitmix64(seed ^ ((uint64_t)round << 40) ^ (0x9E37ull * (uint64_t)g));
    const uint32_t id = (uint32_t)zipf_draw(z, unit_double(r1));
    ids[g] = id;
    rmw[g] = rmw_pm && (uint32_t)((r1 >> 3) % 1000u) < rmw_pm;
    const uint64_t key = (((uint64_t)r << 32) | id) + 1;
    const uint32_t h = dedup_slot(hk, key, mask, true);
    atomicMin(&hmin[h], (uint32_t)w * (uint32_t)per_peer + (uint32_t)j);  // the peer's own op order
}

// one workgroup per worker: each peer's first occurrences, compacted in peer order
__global__ __launch_bounds__(256) void k_peer_compact(const uint32_t *ids, const uint8_t *rmw,
                                                      const unsigned long long *hk, const uint32_t *hmin, uint32_t mask,
                                                      uint8_t *invs, uint8_t *vals, int32_t *peer_counts,
                                                      int32_t per_peer, const uint8_t *peers, int32_t n_peers,
                                                      uint32_t op_size, uint32_t st_value, uint32_t shift)
{
    const int w = blockIdx.x;
    const int32_t row = per_peer * n_peers;
    int base = 0;
    for (int r = 0; r < n_peers; ++r) {
        const uint8_t peer = peers[r];
        int cnt = 0;
        for (int j0 = 0; j0 < per_peer; j0 += 256) {
            const int j = j0 + (int)threadIdx.x;
            const int64_t g = (int64_t)w * row + (int64_t)r * per_peer + j;
            bool keep = false;
            uint32_t id = 0;
            if (j < per_peer) {
                id = ids[g];
                const uint32_t h = dedup_slot(hk, (((uint64_t)r << 32) | id) + 1, mask, false);
                keep = h != 0xFFFFFFFFu && hmin[h] == (uint32_t)w * (uint32_t)per_peer + (uint32_t)j;
            }
            int total;
            const int rank = block_rank(keep, total);
            if (keep) {
                const int64_t o = (int64_t)w * row + base + cnt + rank;
                const uint64_t key = key_of_id(id);
                const uint8_t f = rmw[g];
                // inv_copy_and_modify_elem of the peer's op: version filled in per round
                const uint64_t h1 = (uint64_t)kOpInv | ((uint64_t)peer << 8) | ((uint64_t)(st_value >> shift) << 16) |
                                    ((uint64_t)peer << 24);
                uint64_t *x = reinterpret_cast<uint64_t *>(invs + o * op_size);
                x[0] = key;
                x[1] = h1;
                const uint64_t vv = 0x0101010101010101ULL * (uint8_t)('a' + peer);
                x[2] = (vv << 16) | f;  // bytes 16..17: RMW_flag, no_coales 0; value from byte 18
                for (uint32_t k = 3; k < op_size / 8; ++k) x[k] = vv;
                uint64_t *v = reinterpret_cast<uint64_t *>(vals + o * kOpMetaSize);
                v[0] = key;
                v[1] = (h1 & ~0xFFull) | kOpVal;
            }
            cnt += total;
        }
        if (threadIdx.x == 0) peer_counts[(int64_t)w * n_peers + r] = cnt;
        base += cnt;
    }
}

// the MICA lookup of hermesKV.c:952-993 (first tag match, wrap test, 8-B key compare): the
// entry's physical offset, or ~0 for a miss
__device__ __forceinline__ uint64_t find_entry(const TableView &t, uint64_t key)
{
    const uint64_t *b = reinterpret_cast<const uint64_t *>(t.index + ((key & 0xFFFFFFFFFFFFULL) & t.g.bkt_mask) * 64u);
    const uint32_t tag = (uint32_t)(key >> 48);
    for (int s = 0; s < 8; ++s) {
        const uint64_t slot = b[s];
        if ((slot & 1u) && ((uint32_t)(slot >> 1) & 0x7FFFFFu) == tag) {
            const uint64_t off = slot >> 24;
            if (t.g.log_head - off >= t.g.log_cap) return ~0ull;
            const uint64_t phys = off & t.g.log_mask;
            return *reinterpret_cast<const uint64_t *>(t.log + phys + 8) == key ? phys : ~0ull;
        }
    }
    return ~0ull;
}

// The virtual peers' per-entry words: live entries never overlap and are entry_size long, so
// phys / entry_size is distinct for every entry (one slot per possible entry, not per 8 bytes)
__device__ __forceinline__ uint64_t peer_slot(const TableView &t, uint64_t phys) { return phys / t.g.entry_size; }

// peer_ts words: round tag (23 bits) << 41 | the write's RMW flag << 40 | its 40-bit timestamp
__device__ __forceinline__ uint32_t peer_round_tag(uint32_t round) { return (round + 1u) & 0x7FFFFFu; }

// per round: every live peer INV (and its VAL) takes its key's current timestamp + the write's
// step, cid = the peer; peer_ts (RMW builds) records the peer's write per [entry][peer id].
// Four lanes per INV, as in the batch lookup (hkv_batch.hip k_lookup): each lane reads 16 B of
// the bucket, so one load instruction covers the 64-B bucket line, then lanes 0 and 1 read the
// entry's key and timestamp.
struct __attribute__((aligned(8))) U64x2w {
    uint64_t a, b;
};
constexpr int kPeerTsPair = 2;  // elements in flight per 4-lane group
__global__ __launch_bounds__(256) void k_peer_ts(TableView t, uint8_t *invs, uint8_t *vals, const int32_t *counts,
                                                 int32_t stride, uint32_t op_size, unsigned long long *peer_ts,
                                                 uint32_t round, int64_t total)
{
    const int q = threadIdx.x & 3;
    const int gbase = (threadIdx.x & 63) & ~3;
    int64_t g[kPeerTsPair];
    int live[kPeerTsPair];
    uint64_t key[kPeerTsPair], flags[kPeerTsPair];
#pragma unroll
    for (int k = 0; k < kPeerTsPair; ++k) {
        g[k] = ((int64_t)blockIdx.x * kPeerTsPair + k) * 64 + (threadIdx.x >> 2);
        live[k] = 0;
        key[k] = flags[k] = 0;
        if (g[k] < total && q == 0) {
            const int32_t w = (int32_t)(g[k] / stride);
            if ((int32_t)(g[k] - (int64_t)w * stride) < counts[w]) {
                live[k] = 1;
                const uint8_t *x = invs + g[k] * op_size;
                key[k] = *reinterpret_cast<const uint64_t *>(x);
                flags[k] = *reinterpret_cast<const uint64_t *>(x + 8) >> 8 & 0xFFu;  // byte 9: the peer
                flags[k] |= (uint64_t)(x[16] & 1u) << 8;                               // RMW_flag
            }
        }
    }
    uint4 v[kPeerTsPair];
#pragma unroll
    for (int k = 0; k < kPeerTsPair; ++k) {
        live[k] = __shfl(live[k], 0, 4);
        key[k] = __shfl(key[k], 0, 4);
        v[k] = live[k] ? reinterpret_cast<const uint4 *>(t.index + ((key[k] & 0xFFFFFFFFFFFFULL) & t.g.bkt_mask) * 64u)[q]
                       : make_uint4(0u, 0u, 0u, 0u);
    }
    bool ok[kPeerTsPair];
    uint64_t phys[kPeerTsPair];
    U64x2w ln[kPeerTsPair];
#pragma unroll
    for (int k = 0; k < kPeerTsPair; ++k) {
        const uint64_t s0 = (uint64_t)v[k].x | ((uint64_t)v[k].y << 32), s1 = (uint64_t)v[k].z | ((uint64_t)v[k].w << 32);
        const uint32_t tag = (uint32_t)(key[k] >> 48);
        const bool mt0 = live[k] && (s0 & 1u) && ((uint32_t)(s0 >> 1) & 0x7FFFFFu) == tag;
        const bool mt1 = live[k] && (s1 & 1u) && ((uint32_t)(s1 >> 1) & 0x7FFFFFu) == tag;
        const uint32_t g0 = (uint32_t)(__ballot(mt0) >> gbase) & 0xFu, g1 = (uint32_t)(__ballot(mt1) >> gbase) & 0xFu;
        uint32_t o = 0;  // bit 2*l + j: slot 2*l + j matches (the reference's slot order)
#pragma unroll
        for (int l = 0; l < 4; ++l) o |= ((g0 >> l) & 1u) << (2 * l) | ((g1 >> l) & 1u) << (2 * l + 1);
        const int first = o ? __ffs(o) - 1 : 0;
        const uint64_t off = __shfl((first & 1) ? (s1 >> 24) : (s0 >> 24), first >> 1, 4);
        ok[k] = live[k] && o && t.g.log_head - off < t.g.log_cap;
        phys[k] = off & t.g.log_mask;
        // lane 0: entry bytes 0..15 (key at 8), lane 1: bytes 16..31 (version at 24)
        ln[k] = ok[k] && q < 2 ? reinterpret_cast<const U64x2w *>(t.log + phys[k])[q] : U64x2w{0, 0};
    }
#pragma unroll
    for (int k = 0; k < kPeerTsPair; ++k) {
        const uint64_t ekey = __shfl(ln[k].b, 0, 4);
        const uint32_t cur = (uint32_t)__shfl(ln[k].b, 1, 4);
        if (q != 0 || !live[k]) continue;
        uint8_t *x = invs + g[k] * op_size;
        const uint8_t peer = (uint8_t)flags[k];
        const bool rmw = (flags[k] >> 8) & 1u;
        uint32_t ver = 2;
        if (ok[k] && ekey == key[k]) {
            ver = cur + ((!t.g.rmw_enabled || rmw) ? 2u : 4u);
            if (peer_ts && peer < 8)
                atomicMax(peer_ts + peer_slot(t, phys[k]) * 8 + peer,
                          ((unsigned long long)peer_round_tag(round) << 41) | ((unsigned long long)rmw << 40) |
                              ((unsigned long long)ver << 8) | peer);
        }
        // a fresh message each round: the batches of a previous use of the slab rewrote the opcodes
        x[8] = kOpInv;
        *reinterpret_cast<uint32_t *>(x + 12) = ver;
        uint8_t *vv = vals + g[k] * kOpMetaSize;
        vv[8] = kOpVal;
        *reinterpret_cast<uint32_t *>(vv + 12) = ver;
    }
}

// The virtual peers' answers to this round's INVs: an ACK (ack_copy_and_modify_elem,
// hermes_worker.c:100-118) -- or, for an RMW INV whose timestamp is below the peer's own write of
// the key this round (peer_ts, RMW builds), the INV-abort hermes_exec_inv makes at the peer
// (hermesKV.c:566-576): the peer's local state (local_state_to_op, hermesKV.c:143-153: its RMW
// flag, timestamp, val_len and value 'a' + peer) with opcode ST_OP_INV_ABORT and sender = peer.
__device__ __forceinline__ void peer_answer(const uint8_t *x, uint8_t *y, uint32_t op_size, uint32_t ack_size,
                                            uint8_t peer, const TableView &t, const unsigned long long *peer_ts,
                                            uint32_t round)
{
    const W16 h = *reinterpret_cast<const W16 *>(x);
    if (peer_ts && (x[16] & 1u) && peer < 8 && ack_size >= op_size) {
        const uint64_t phys = find_entry(t, h.a);
        if (phys != ~0ull) {
            const unsigned long long pw = peer_ts[peer_slot(t, phys) * 8 + peer];
            const uint64_t ours = ((uint64_t)(uint32_t)(h.b >> 32) << 8) | (uint8_t)(h.b >> 24);
            if ((uint32_t)(pw >> 41) == peer_round_tag(round) && (pw & 0xFFFFFFFFFFull) > ours) {
                const uint64_t pts = pw & 0xFFFFFFFFFFull;
                uint64_t *d = reinterpret_cast<uint64_t *>(y);
                d[0] = h.a;
                d[1] = (uint64_t)kOpInvAbort | ((uint64_t)peer << 8) | ((uint64_t)(uint8_t)x[10] << 16) |
                       ((pts & 0xFFull) << 24) | ((pts >> 8) << 32);
                // the peer key's RMW flag is its write's (update_actions, hermesKV.c:100-141)
                const uint64_t vv = 0x0101010101010101ULL * (uint8_t)('a' + peer);
                d[2] = (vv << 16) | ((uint64_t)x[17] << 8) | ((pw >> 40) & 1u);
                for (uint32_t k = 3; k < op_size / 8; ++k) d[k] = vv;
                return;
            }
        }
    }
    *reinterpret_cast<W16 *>(y) = W16{h.a, with_op_state(h.b, kOpAck, peer)};  // ack_copy_and_modify_elem
}

// rows: worker w's answers at w * out_stride; out_off (packed ACK batches): at out_off[w]
__global__ void k_peer_acks(const uint8_t *invs, const int32_t *inv_count, int32_t inv_stride, uint32_t op_size,
                            uint8_t *acks, uint32_t ack_size, int32_t out_stride, int32_t *ack_count,
                            const uint8_t *peers, int32_t n_peers, int64_t total, TableView t,
                            const unsigned long long *peer_ts, uint32_t round, const int32_t *out_off,
                            int32_t pm_workers)
{
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total) return;
    int64_t per_w = out_stride;     // slots x n_peers ACK positions per worker (host checks)
    int32_t w = (int32_t)(g / per_w);
    int32_t rem = (int32_t)(g - (int64_t)w * per_w);
    int32_t j = rem / n_peers, r = rem - j * n_peers;
    int32_t n = inv_count[w];
    if (rem == 0 && ack_count) ack_count[w] = n * n_peers;
    if (j >= n) return;
    const uint8_t *x = invs + ((int64_t)w * inv_stride + j) * op_size;
    // peer-major (pm_workers > 0): peer r's answers to every INV of the round as one block of
    // T = out_off[pm_workers] elements, worker w's at out_off[w] in it
    const int64_t pos = pm_workers > 0 ? (int64_t)r * out_off[pm_workers] + out_off[w] + j
                      : out_off ? (int64_t)out_off[w] + rem : (int64_t)w * out_stride + rem;
    peer_answer(x, acks + pos * ack_size, op_size, ack_size, peers[r], t, peer_ts, round);
}

// Packed ACK batches: off[w] = n_peers x (INVs of workers before w), off[n] = the total; the total
// and the largest per-worker INV count land in pinned host memory (h[0], h[1]) for the host to size
// the round's launches while the GPU runs the INV batch
__global__ __launch_bounds__(1024) void k_ack_offsets(const int32_t *counts, int32_t n, int32_t n_peers, int32_t *off,
                                                      int32_t *h, int32_t seq)
{
    // each thread owns 16 consecutive counts (one pass up to 16384 workers, loads issued together)
    __shared__ int32_t part[16], pmax[16];
    __shared__ int32_t carry;
    if (threadIdx.x == 0) carry = 0;
    int32_t mx = 0;
    const bool vec = (((uintptr_t)counts | (uintptr_t)off) & 15u) == 0;
    for (int32_t i0 = 0; i0 < n; i0 += 16384) {
        __syncthreads();
        const int32_t b = i0 + (int32_t)threadIdx.x * 16;
        int32_t c[16], sum = 0;
        if (vec && b + 16 <= n) {
            const int4 *p = reinterpret_cast<const int4 *>(counts + b);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int4 v = p[k];
                c[4 * k] = v.x;
                c[4 * k + 1] = v.y;
                c[4 * k + 2] = v.z;
                c[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = b + k < n ? counts[b + k] : 0;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            mx = c[k] > mx ? c[k] : mx;
            sum += c[k] * n_peers;
        }
        int32_t v = sum;  // inclusive scan of the thread sums within the wave, then across waves
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t u = __shfl_up(v, o, 64);
            if ((threadIdx.x & 63) >= (unsigned)o) v += u;
        }
        if ((threadIdx.x & 63) == 63) part[threadIdx.x >> 6] = v;
        __syncthreads();
        int32_t run = carry;
        for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) run += part[k];
        run += v - sum;
        if (vec && b + 16 <= n) {
            int4 *q = reinterpret_cast<int4 *>(off + b);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int4 o4;
                o4.x = run;
                run += c[4 * k] * n_peers;
                o4.y = run;
                run += c[4 * k + 1] * n_peers;
                o4.z = run;
                run += c[4 * k + 2] * n_peers;
                o4.w = run;
                run += c[4 * k + 3] * n_peers;
                q[k] = o4;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (b + k < n) off[b + k] = run;
                run += c[k] * n_peers;
            }
        }
        __syncthreads();
        if (threadIdx.x == 1023) carry = run;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t u = __shfl_down(mx, o, 64);
        mx = u > mx ? u : mx;
    }
    if ((threadIdx.x & 63) == 0) pmax[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 16; ++k) mx = pmax[k] > mx ? pmax[k] : mx;
        off[n] = carry;
        if (seq == 0) {  // the host waits on an event recorded after this kernel
            h[0] = carry;
            h[1] = mx;
        } else {
            // the host spins on h[2]: system-scope stores write through to host memory, the wait
            // orders the flag after the values, and no release fence (an L2 write-back of
            // everything dirty, ~6 us before the next kernel could start) is needed
            __hip_atomic_store(h, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(h + 1, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(h + 2, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The virtual peers' answers appended to each worker's ACK queue (aq: [W][q_stride] elements of
// ack_size bytes, aq_n[w] queued): one workgroup per worker. A worker with outstanding VALs
// (vq_n[w] > 0) does not poll its ACKs this round (hermes_worker.c:479): acnt[w] = 0 and the
// queue keeps growing; otherwise acnt[w] = the whole queue, applied by this round's ACK batch.
__global__ __launch_bounds__(256) void k_peer_acks_q(const uint8_t *invs, const int32_t *inv_count, int32_t inv_stride,
                                                     uint32_t op_size, uint8_t *aq, uint32_t ack_size, int32_t q_stride,
                                                     int32_t *aq_n, const int32_t *vq_n, int32_t *acnt,
                                                     const uint8_t *peers, int32_t n_peers, TableView t,
                                                     const unsigned long long *peer_ts, uint32_t round)
{
    const int w = blockIdx.x;
    const int n = inv_count[w], base = aq_n[w];
    const int total = n * n_peers;
    for (int g = threadIdx.x; g < total; g += 256) {
        const int j = g / n_peers, r = g - j * n_peers;
        if (base + g >= q_stride) break;  // the host sizes q_stride for C INVs x n_peers
        const uint8_t *x = invs + ((int64_t)w * inv_stride + j) * op_size;
        peer_answer(x, aq + ((int64_t)w * q_stride + base + g) * ack_size, op_size, ack_size, peers[r], t, peer_ts,
                    round);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int q = min(base + total, q_stride);
        aq_n[w] = q;
        acnt[w] = vq_n[w] > 0 ? 0 : q;
    }
}

// VALs under credits: the worker's carried VALs (vq, from rounds whose VALs did not all fit) and
// then the VALs of the writes this round's ACK batch completed (ST_LAST_ACK_SUCCESS in its ACK
// queue, when it applied one: acnt[w] > 0) go out in that order, at most v_credits per round
// (the VAL channel's credits, returned by the peers' CRD messages once they apply them:
// hermes_worker.c:513, wings.h:862-916); the rest is carried to the next round, when the worker
// sends them before polling ACKs again (has_outstanding_vals, hermes_worker.c:479, 500-503). An
// applied queue empties (val_skip_or_get_sender_id / val_modify_elem_after_send set its elements
// ST_EMPTY). One workgroup per worker.
constexpr int kMaxVq = 1024;
__global__ __launch_bounds__(256) void k_vals_credit(uint8_t *aq, int32_t *aq_n, const int32_t *acnt, int32_t q_stride,
                                                     uint32_t ack_size, uint8_t *vq, int32_t *vq_n, int32_t vq_stride,
                                                     uint8_t *out, int32_t *out_count, int32_t out_stride,
                                                     int32_t v_credits, uint32_t machine_id,
                                                     unsigned long long *overflow)
{
    __shared__ W16 buf[kMaxVq];
    const int w = blockIdx.x;
    const int carried = vq_n[w], applied = acnt[w];
    W16 *vrow = reinterpret_cast<W16 *>(vq + (int64_t)w * vq_stride * kOpMetaSize);
    for (int j = threadIdx.x; j < carried && j < kMaxVq; j += 256) buf[j] = vrow[j];
    int total = min(carried, kMaxVq);
    for (int j0 = 0; j0 < applied; j0 += 256) {
        const int j = j0 + (int)threadIdx.x;
        uint8_t *x = aq + ((int64_t)w * q_stride + j) * ack_size;
        const uint8_t oc = j < applied ? x[8] : 0;
        const bool send = j < applied && val_sends(oc);
        int cnt;
        const int rank = block_rank(send, cnt);
        if (send && total + rank < kMaxVq) {
            const W16 h = *reinterpret_cast<const W16 *>(x);
            buf[total + rank] = W16{h.a, (h.b & ~0xFFFFull) | kOpVal | ((uint64_t)(machine_id & 0xFF) << 8)};
        } else if (send && overflow) {
            atomicAdd(overflow, 1ull);
        }
        if (j < applied && oc != kEmpty) x[8] = kEmpty;
        total = min(total + cnt, kMaxVq);
    }
    __syncthreads();
    const int send = min(total, min(v_credits, out_stride));
    W16 *orow = reinterpret_cast<W16 *>(out + (int64_t)w * out_stride * kOpMetaSize);
    for (int j = threadIdx.x; j < send; j += 256) orow[j] = buf[j];
    const int keep = min(total - send, vq_stride);
    for (int j = threadIdx.x; j < keep; j += 256) vrow[j] = buf[send + j];
    if (threadIdx.x == 0) {
        out_count[w] = send;
        vq_n[w] = keep;
        if (applied) aq_n[w] = 0;
        if (total - send > keep && overflow) atomicAdd(overflow, (unsigned long long)(total - send - keep));
    }
}

// The entry of every peer INV of a pre-drawn round index, located once when the index is drawn
// (the index never changes under the rounds: writes update entries in place and nothing is
// inserted), so the per-round timestamps need one entry line per INV instead of bucket + line.
__global__ __launch_bounds__(256) void k_peer_locate(TableView t, const uint8_t *invs, uint32_t op_size,
                                                     int64_t total, uint64_t *phys_out)
{
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    phys_out[g] = find_entry(t, *reinterpret_cast<const uint64_t *>(invs + g * op_size));
}

// k_peer_ts for located INVs (one thread each): the key is checked at the entry, and an INV
// whose entry does not hold its key any more takes the full lookup
struct PeerTsArgs {   // hkv_wl_peer_ts_at's arguments
    TableView t;
    uint8_t *invs, *vals;
    const uint64_t *phys_in;
    int64_t total;
    uint32_t op_size;
    unsigned long long *peer_ts;
    uint32_t round;
};
__device__ __forceinline__ void peer_ts_at_body(const PeerTsArgs &pt, int bx)
{
    const TableView &t = pt.t;
    uint8_t *invs = pt.invs, *vals = pt.vals;
    const uint64_t *phys_in = pt.phys_in;
    const int64_t total = pt.total;
    const uint32_t op_size = pt.op_size, round = pt.round;
    unsigned long long *peer_ts = pt.peer_ts;
    const int64_t g = (int64_t)bx * 256 + threadIdx.x;
    if (g >= total) return;
    uint8_t *x = invs + g * op_size;
    // every load that does not need the entry first: INV header, flags, location and the VAL's header
    uint8_t *vv = vals + g * kOpMetaSize;
    const uint64_t key = *reinterpret_cast<const uint64_t *>(x);
    const uint64_t h8 = *reinterpret_cast<const uint64_t *>(x + 8);
    const uint64_t vh = *reinterpret_cast<const uint64_t *>(vv + 8);
    const uint8_t peer = (uint8_t)(h8 >> 8);
    const bool rmw = x[16] & 1u;
    uint64_t phys = phys_in[g];
    uint32_t cur = 0;
    bool ok = false;
    if (phys != ~0ull) {
        const U64x2w *e = reinterpret_cast<const U64x2w *>(t.log + phys);
        const U64x2w l0 = e[0], l1 = e[1];  // key at 8, timestamp version at 24
        if (l0.b == key) {
            ok = true;
            cur = (uint32_t)l1.b;
        }
    }
    if (!ok) {
        phys = find_entry(t, key);
        if (phys != ~0ull) {
            ok = true;
            cur = *reinterpret_cast<const uint32_t *>(t.log + phys + 24);
        }
    }
    uint32_t ver = 2;
    if (ok) {
        ver = cur + ((!t.g.rmw_enabled || rmw) ? 2u : 4u);
        if (peer_ts && peer < 8)
            atomicMax(peer_ts + peer_slot(t, phys) * 8 + peer,
                      ((unsigned long long)peer_round_tag(round) << 41) | ((unsigned long long)rmw << 40) |
                          ((unsigned long long)ver << 8) | peer);
    }
    // bytes 8..15 rewritten whole (opcode, sender, val_len, cid, version): one 8-B store
    const uint64_t nh = (h8 & 0xFFFFFF00ull & 0xFFFFFFFFull) | kOpInv | ((uint64_t)ver << 32);
    *reinterpret_cast<uint64_t *>(x + 8) = nh;
    *reinterpret_cast<uint64_t *>(vv + 8) = (vh & 0xFFFFFF00ull & 0xFFFFFFFFull) | kOpVal | ((uint64_t)ver << 32);
}

__global__ __launch_bounds__(256) void k_peer_ts_at(PeerTsArgs pt) { peer_ts_at_body(pt, blockIdx.x); }

// The refill plan of this round and the virtual peers' timestamps of the next, in one launch (round 6): both
// run between a round's VAL batch and the next local launch, touch disjoint data (op mirrors and patches; the
// peers' slabs, reading the table) and are bound by dependent loads, so side by side in one grid they overlap
// and the launch boundary between them goes. Blocks [0, plan_blocks) plan, the rest take timestamps.
__global__ __launch_bounds__(256) HKV_PLAN_SGPR_ATTR void k_plan_peer_ts(PlanArgs pa, PeerTsArgs pt, int plan_blocks)
{
    if ((int)blockIdx.x < plan_blocks) refill_plan_body<2>(pa, blockIdx.x);
    else peer_ts_at_body(pt, (int)blockIdx.x - plan_blocks);
}

}  // namespace hkv

using namespace hkv;

static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }
static inline int ok() { return hipGetLastError() == hipSuccess ? 0 : -5; }

extern "C" {

int hkv_wl_gen_trace(uint64_t *tkey, uint8_t *top, uint32_t *tid, int32_t n_workers, int32_t len, const hkv_zipf *z,
                     uint32_t write_pm, uint32_t rmw_pm, uint64_t seed, void *stream)
{
    int64_t n = (int64_t)n_workers * len;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_gen_trace, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, tkey, top, tid, n_workers,
                       len, *z, write_pm, rmw_pm, seed);
    return ok();
}

int hkv_wl_refill(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint32_t st_value, uint32_t shift,
                  const uint64_t *tkey, const uint8_t *top, const uint32_t *tid, int32_t tlen, uint32_t *cursor,
                  uint32_t machine_id, int32_t first_iter, uint32_t flags, unsigned long long *counters,
                  uint8_t *opc_out, uint8_t *hot, void *stream)
{
    if (stride > 256 || n_workers <= 0 || op_size % 8 || tlen <= 0) return -1;
    if (flags & ~(uint32_t)(HKV_WL_REFILL_ALL | HKV_WL_READ_TS_RESET | HKV_WL_COALESCE_HOT)) return -1;
    const size_t lds = (size_t)stride * op_size;
    if (flags & HKV_WL_COALESCE_HOT) {
        // one 256-thread workgroup per worker, the slab and a slot index per pointer in LDS
        if (!tid || !hot || stride > 255 || lds > 56 * 1024) return -1;
        hipLaunchKernelGGL(k_refill_hot, dim3(n_workers), dim3(256), lds, (hipStream_t)stream, ops, stride, op_size,
                           st_value, shift, tkey, top, tid, tlen, cursor, machine_id, first_iter, flags, counters,
                           opc_out, hot);
        return ok();
    }
    if (op_size > 64 && st_value >= 6 && (kOpValueOff - 16 + st_value) / 8 + 7 <= 64) {  // big ops: in place
        hipLaunchKernelGGL(k_refill_direct, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size,
                           st_value, shift, tkey, top, tlen, cursor, machine_id, first_iter, flags, counters,
                           opc_out, (uint8_t *)nullptr);
        return ok();
    }
    if (lds > 160 * 1024 - 64) return -1;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)k_refill, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_refill, dim3(n_workers), dim3(256), lds, (hipStream_t)stream, ops, stride, op_size, st_value,
                       shift, tkey, top, tlen, cursor, machine_id, first_iter, flags, counters, opc_out);
    return ok();
}

int hkv_wl_refill_st(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint32_t st_value,
                     uint32_t shift, const uint64_t *tkey, const uint8_t *top, int32_t tlen, uint32_t *cursor,
                     uint32_t machine_id, uint32_t flags, unsigned long long *counters, uint8_t *opc,
                     uint8_t *states, void *stream)
{
    if (stride > 256 || n_workers <= 0 || tlen <= 0 || !states || !opc) return -1;
    if (flags & ~(uint32_t)(HKV_WL_REFILL_ALL | HKV_WL_READ_TS_RESET)) return -1;   // no hot-request coalescing
    if (!(op_size > 64 && op_size % 8 == 0 && st_value >= 6 && (kOpValueOff - 16 + st_value) / 8 + 7 <= 64)) return -1;
    // one wave per worker (round 4: level with the workgroup-per-worker k_refill_direct, kept for its
    // ballot-only ranks)
    constexpr bool st_w = true;
    if (st_w)
        hipLaunchKernelGGL(k_refill_st_w, dim3((unsigned)((n_workers + 3) / 4)), dim3(256), 0, (hipStream_t)stream, ops,
                           n_workers, stride, op_size, st_value, shift, tkey, top, tlen, cursor, machine_id, flags,
                           counters, opc, states);
    else
        hipLaunchKernelGGL(k_refill_direct, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size,
                           st_value, shift, tkey, top, tlen, cursor, machine_id, 0, flags, counters, opc, states);
    return ok();
}

int hkv_wl_refill_plan(uint8_t *states, int32_t n_workers, int32_t stride, uint32_t st_value, uint32_t shift,
                       const uint64_t *tkey, const uint8_t *top, int32_t tlen, uint32_t *cursor, uint32_t machine_id,
                       uint32_t flags, unsigned long long *counters, uint8_t *opc, uint8_t *patch, void *stream)
{
    if (stride > 256 || n_workers <= 0 || tlen <= 0 || !states || !opc || !patch) return -1;
    if (flags & ~(uint32_t)(HKV_WL_REFILL_ALL | HKV_WL_READ_TS_RESET)) return -1;   // no hot-request coalescing
    if (((uintptr_t)patch & 15) || (st_value >> shift) > 255) return -1;   // val_len: a byte
    const PlanArgs pa{states, n_workers, stride, st_value, shift, tkey, top, tlen, cursor, machine_id, flags, counters, opc,
                      patch};
    hipLaunchKernelGGL(k_refill_plan_w<2>, dim3((unsigned)((n_workers + 7) / 8)), dim3(256), 0, (hipStream_t)stream, pa);
    return ok();
}

int hkv_wl_fold_counters(unsigned long long *counters, void *stream)
{
    hipLaunchKernelGGL(k_fold_counters, dim3(1), dim3(256), 0, (hipStream_t)stream, counters);
    return ok();
}

int hkv_wl_marshal_invs(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *out,
                        int32_t *count, uint32_t machine_id, void *stream)
{
    if (stride > 256 || n_workers <= 0) return -1;
    hipLaunchKernelGGL(k_marshal_invs, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size, out,
                       stride, count, machine_id, (unsigned long long *)nullptr, (const int32_t *)nullptr, 1,
                       (uint8_t *)nullptr);
    return ok();
}

int hkv_wl_marshal_acks(uint8_t *invs, int64_t n, uint32_t op_size, uint8_t *out, uint32_t ack_size,
                        uint32_t machine_id, void *stream)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_marshal_acks, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, invs, n, op_size, out,
                       ack_size, machine_id);
    return ok();
}

int hkv_wl_marshal_vals(uint8_t *acks, int64_t n, uint32_t ack_size, uint8_t *out, uint32_t machine_id, void *stream)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_marshal_vals, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, acks, n, ack_size, out,
                       machine_id);
    return ok();
}

int hkv_wl_peer_acks_pm(hkv_table *t, const uint8_t *inv_out, const int32_t *inv_count, int32_t n_workers,
                        int32_t inv_stride, uint32_t op_size, uint8_t *acks, uint32_t ack_size, int32_t max_invs,
                        int32_t *ack_count, const uint8_t *peer_ids, int32_t n_peers,
                        const unsigned long long *peer_ts, uint32_t round, const int32_t *inv_off, void *stream)
{
    if (n_peers <= 0 || n_workers <= 0 || ack_size < kOpMetaSize || ack_size % 8 || !inv_off) return -1;
    if (max_invs <= 0 || max_invs > inv_stride) return -1;
    TableView tv{};
    if (peer_ts && table_view(t, &tv)) return -1;
    const int32_t out_stride = max_invs * n_peers;
    int64_t total = (int64_t)n_workers * out_stride;
    hipLaunchKernelGGL(k_peer_acks, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, inv_out, inv_count,
                       inv_stride, op_size, acks, ack_size, out_stride, ack_count, peer_ids, n_peers, total, tv,
                       peer_ts, round, inv_off, n_workers);
    return ok();
}

int hkv_wl_peer_acks(hkv_table *t, const uint8_t *inv_out, const int32_t *inv_count, int32_t n_workers,
                     int32_t inv_stride, uint32_t op_size, uint8_t *acks, uint32_t ack_size, int32_t out_stride,
                     int32_t *ack_count, const uint8_t *peer_ids, int32_t n_peers,
                     const unsigned long long *peer_ts, uint32_t round, const int32_t *out_off, void *stream)
{
    if (n_peers <= 0 || n_workers <= 0 || ack_size < kOpMetaSize || ack_size % 8) return -1;
    if (out_stride % n_peers || out_stride > inv_stride * n_peers || out_stride <= 0) return -1;
    TableView tv{};
    if (peer_ts && table_view(t, &tv)) return -1;
    int64_t total = (int64_t)n_workers * out_stride;
    hipLaunchKernelGGL(k_peer_acks, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, inv_out, inv_count,
                       inv_stride, op_size, acks, ack_size, out_stride, ack_count, peer_ids, n_peers, total, tv,
                       peer_ts, round, out_off, 0);
    return ok();
}

static size_t peer_slots(int64_t total)
{
    size_t s = 1024;
    while (s < 2 * (size_t)total) s <<= 1;
    return s;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t hkv_wl_peer_round_scratch(int32_t n_workers, int32_t per_peer, int32_t n_peers)
{
    const int64_t total = (int64_t)n_workers * per_peer * n_peers;
    const size_t slots = peer_slots(total);
    return align_up(8 * slots) + align_up(4 * slots) + align_up(4 * (size_t)total) + align_up((size_t)total);
}

int hkv_wl_gen_peer_round(uint8_t *invs, uint8_t *vals, int32_t *peer_counts, int32_t n_workers, int32_t per_peer,
                          const uint8_t *peer_ids, int32_t n_peers, uint32_t op_size, uint32_t st_value,
                          uint32_t shift, const hkv_zipf *z, uint32_t rmw_pm, uint32_t round, uint64_t seed,
                          void *scratch, void *stream)
{
    const int64_t total = (int64_t)n_workers * per_peer * n_peers;
    if (total <= 0) return 0;
    if (op_size % 8 || op_size < kOpValueOff + st_value || total > 0x7FFFFFFFll) return -1;
    hipStream_t s = (hipStream_t)stream;
    const size_t slots = peer_slots(total);
    uint8_t *p = static_cast<uint8_t *>(scratch);
    unsigned long long *hk = reinterpret_cast<unsigned long long *>(p);
    p += align_up(8 * slots);
    uint32_t *hmin = reinterpret_cast<uint32_t *>(p);
    p += align_up(4 * slots);
    uint32_t *ids = reinterpret_cast<uint32_t *>(p);
    p += align_up(4 * (size_t)total);
    uint8_t *rmw = p;
    if (hipMemsetAsync(hk, 0, 8 * slots, s) != hipSuccess || hipMemsetAsync(hmin, 0xFF, 4 * slots, s) != hipSuccess)
        return -5;
    hipLaunchKernelGGL(k_peer_draw, dim3(blocks_for(total)), dim3(256), 0, s, ids, rmw, hk, hmin,
                       (uint32_t)(slots - 1), per_peer, n_peers, *z, rmw_pm, round, seed, total);
    hipLaunchKernelGGL(k_peer_compact, dim3(n_workers), dim3(256), 0, s, ids, rmw, hk, hmin, (uint32_t)(slots - 1), invs,
                       vals, peer_counts, per_peer, peer_ids, n_peers, op_size, st_value, shift);
    return ok();
}

int hkv_wl_peer_ts(hkv_table *t, uint8_t *invs, uint8_t *vals, const int32_t *counts, int32_t n_workers,
                   int32_t stride, uint32_t op_size, unsigned long long *peer_ts, uint32_t round, void *stream)
{
    TableView tv;
    if (table_view(t, &tv) || n_workers <= 0 || stride <= 0 || op_size % 8) return -1;
    const int64_t total = (int64_t)n_workers * stride;
    const int64_t per_block = 64 * kPeerTsPair;  // 4 lanes per element, kPeerTsPair elements per group
    hipLaunchKernelGGL(k_peer_ts, dim3((unsigned)((total + per_block - 1) / per_block)), dim3(256), 0,
                       (hipStream_t)stream, tv, invs, vals, counts, stride, op_size, peer_ts, round, total);
    return ok();
}

uint64_t hkv_wl_peer_ts_words(const hkv_table *t)
{
    TableView tv;
    if (table_view(t, &tv)) return 0;
    return (tv.g.log_cap / tv.g.entry_size + 1) * 8;
}

int hkv_wl_marshal_invs_cap(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *out,
                            int32_t out_stride, int32_t *count, uint32_t machine_id, unsigned long long *held,
                            uint8_t *states, void *stream)
{
    if (stride > 256 || n_workers <= 0 || out_stride <= 0 || op_size % 8) return -1;
    const bool mwave = marshal_wave();
    if (op_size <= 64)
        if (wl_wpw() == 2 && mwave)
            hipLaunchKernelGGL((k_marshal_invs_w<2, true>), dim3((unsigned)((n_workers + 7) / 8)), dim3(256), 0,
                               (hipStream_t)stream, ops, n_workers, stride, op_size, out, out_stride, count, machine_id,
                               held, (const int32_t *)nullptr, 1, states);
        else if (wl_wpw() == 2)
            hipLaunchKernelGGL(k_marshal_invs_w<2>, dim3((unsigned)((n_workers + 7) / 8)), dim3(256), 0, (hipStream_t)stream,
                               ops, n_workers, stride, op_size, out, out_stride, count, machine_id, held,
                               (const int32_t *)nullptr, 1, states);
        else
            hipLaunchKernelGGL(k_marshal_invs_w<1>, dim3((unsigned)((n_workers + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                               ops, n_workers, stride, op_size, out, out_stride, count, machine_id, held,
                               (const int32_t *)nullptr, 1, states);
    else
        hipLaunchKernelGGL(k_marshal_invs, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size,
                           out, out_stride, count, machine_id, held, (const int32_t *)nullptr, 1, states);
    return ok();
}

int hkv_wl_marshal_invs_credits(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *out,
                                int32_t out_stride, int32_t *count, uint32_t machine_id, unsigned long long *held,
                                const int32_t *aq_n, int32_t r_alive, void *stream)
{
    if (stride > 256 || n_workers <= 0 || out_stride <= 0 || op_size % 8) return -1;
    if (op_size <= 64)
        hipLaunchKernelGGL(k_marshal_invs_w<1>, dim3((unsigned)((n_workers + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                           ops, n_workers, stride, op_size, out, out_stride, count, machine_id, held, aq_n, r_alive,
                           (uint8_t *)nullptr);
    else
        hipLaunchKernelGGL(k_marshal_invs, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size,
                           out, out_stride, count, machine_id, held, aq_n, r_alive, (uint8_t *)nullptr);
    return ok();
}

int hkv_wl_marshal_memb_vals(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *out,
                             int32_t out_stride, int32_t *count, uint32_t machine_id, uint8_t *states, void *stream)
{
    if (stride > 256 || n_workers <= 0 || out_stride <= 0 || op_size % 8) return -1;
    hipLaunchKernelGGL(k_marshal_memb_vals, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, ops, stride, op_size,
                       out, out_stride, count, machine_id, states);
    return ok();
}

int hkv_wl_max_to_host(const int32_t *counts, int32_t n, int32_t *h_out, void *stream)
{
    if (n <= 0) return -1;
    int32_t *d_out = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d_out), h_out, 0) != hipSuccess || !d_out) return -1;
    hipLaunchKernelGGL(k_max_to_host, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, n, d_out);
    return ok();
}

int hkv_wl_marshal_acks_rows(uint8_t *invs, const int32_t *in_count, int32_t rows, int32_t C, uint32_t op_size,
                             uint8_t *out, uint32_t ack_size, int32_t *out_count, uint32_t machine_id, void *stream)
{
    if (rows <= 0) return 0;
    if (C <= 0 || op_size % 8 || ack_size % 8) return -1;
    hipLaunchKernelGGL(k_marshal_acks_rows, dim3(rows), dim3(256), 0, (hipStream_t)stream, invs, in_count, C, op_size,
                       out, ack_size, out_count, machine_id);
    return ok();
}

int hkv_wl_regroup(const uint8_t *in, const int32_t *counts, int32_t n_peers, int32_t n_workers, int32_t C,
                   uint32_t elem_size, uint8_t *out, int32_t out_stride, int32_t *out_count, void *stream)
{
    if (n_workers <= 0) return 0;
    if (n_peers <= 0 || C <= 0 || elem_size % 8 || out_stride < n_peers * C) return -1;
    hipLaunchKernelGGL(k_regroup, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, in, counts, n_peers, n_workers,
                       C, elem_size, out, out_stride, out_count);
    return ok();
}

int hkv_wl_collect_vals(uint8_t *acks, const int32_t *count, int32_t n_workers, int32_t stride, uint32_t ack_size,
                        uint8_t *out, int32_t C, int32_t *out_count, uint32_t machine_id, unsigned long long *held,
                        const int32_t *offsets, void *stream)
{
    return hkv_wl_collect_vals_blocks(acks, count, n_workers, stride, ack_size, out, C, out_count, machine_id, held,
                                      offsets, 1, stream);
}

int hkv_wl_collect_vals_blocks(uint8_t *acks, const int32_t *count, int32_t n_workers, int32_t stride,
                               uint32_t ack_size, uint8_t *out, int32_t C, int32_t *out_count, uint32_t machine_id,
                               unsigned long long *held, const int32_t *offsets, int32_t n_blocks, void *stream)
{
    if (n_workers <= 0) return 0;
    if (C <= 0 || ack_size % 8 || n_blocks < 1 || (n_blocks > 1 && !offsets)) return -1;
    hipLaunchKernelGGL(k_collect_vals, dim3(n_workers), dim3(64), 0, (hipStream_t)stream, acks, count, stride,
                       ack_size, out, C, out_count, machine_id, held, offsets, n_blocks, (int64_t)0);
    return ok();
}

int hkv_wl_collect_vals_rows(uint8_t *acks, int32_t n_workers, int32_t n_rows, int64_t row_stride, uint32_t ack_size,
                             uint8_t *out, int32_t C, int32_t *out_count, uint32_t machine_id,
                             unsigned long long *held, const int32_t *offsets, void *stream)
{
    if (n_workers <= 0) return 0;
    if (C <= 0 || ack_size % 8 || n_rows < 1 || row_stride <= 0 || !offsets) return -1;
    hipLaunchKernelGGL(k_collect_vals, dim3(n_workers), dim3(64), 0, (hipStream_t)stream, acks, nullptr, 0, ack_size,
                       out, C, out_count, machine_id, held, offsets, n_rows, row_stride);
    return ok();
}

int hkv_wl_ack_offsets(const int32_t *inv_count, int32_t n_workers, int32_t n_peers, int32_t *offsets, int32_t *h_out,
                       int32_t seq, void *stream)
{
    if (n_workers <= 0 || n_peers <= 0 || seq < 0) return -1;
    int32_t *d_out = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d_out), h_out, 0) != hipSuccess || !d_out) return -1;
    hipLaunchKernelGGL(k_ack_offsets, dim3(1), dim3(1024), 0, (hipStream_t)stream, inv_count, n_workers, n_peers,
                       offsets, d_out, seq);
    return ok();
}

int hkv_wl_marshal_invs_packed(uint8_t *ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *states,
                               int32_t C, int32_t cap, uint8_t *out, int32_t *offsets, int32_t *count, int32_t *sent,
                               uint32_t machine_id, unsigned long long *held, void *stream)
{
    if (stride > 256 || n_workers <= 0 || C <= 0 || cap < 0 || op_size % 8 || !states) return -1;
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = (unsigned)((n_workers + 3) / 4);
    hipLaunchKernelGGL(k_count_invs, dim3(g), dim3(256), 0, s, states, n_workers, stride, count);
    hipLaunchKernelGGL(k_scan_cap, dim3(1), dim3(1024), 0, s, count, n_workers, C, cap, offsets, sent, held);
    hipLaunchKernelGGL(k_marshal_invs_packed, dim3(g), dim3(256), 0, s, ops, n_workers, stride, op_size, out, offsets,
                       sent, machine_id, states, (int32_t)marshal_wave());
    return ok();
}

int hkv_wl_pack_rows(const uint8_t *rows, const int32_t *counts, int32_t n_rows, int32_t C, uint32_t elem_size,
                     uint8_t *packed, int32_t *offsets, void *stream)
{
    if (n_rows <= 0) return 0;
    if (C <= 0 || elem_size % 8) return -1;
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, n_rows, offsets);
    hipLaunchKernelGGL(k_pack_rows, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, rows, counts, offsets, C,
                       elem_size, packed);
    return ok();
}

int hkv_wl_marshal_acks_aligned(uint8_t *invs, const int32_t *counts, int32_t rows, int32_t width, uint32_t op_size,
                                uint8_t *out, uint32_t ack_size, uint32_t machine_id, void *stream)
{
    const int64_t n = (int64_t)rows * width;
    if (n <= 0) return 0;
    if (op_size % 8 || ack_size % 8) return -1;
    hipLaunchKernelGGL(k_marshal_acks_aligned, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, invs, counts,
                       width, n, op_size, out, ack_size, machine_id);
    return ok();
}

int hkv_wl_regroup_aligned(const uint8_t *in, int32_t n_peers, int32_t width, const int32_t *offsets,
                           const int32_t *counts, int32_t n_workers, uint32_t elem_size, uint8_t *out,
                           int32_t out_stride, int32_t *out_count, void *stream)
{
    if (n_workers <= 0) return 0;
    if (n_peers <= 0 || width <= 0 || elem_size % 8) return -1;
    hipLaunchKernelGGL(k_regroup_aligned, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, in, n_peers, width,
                       offsets, counts, elem_size, out, out_stride, out_count);
    return ok();
}

}  // extern "C"

extern "C" {

int hkv_wl_peer_acks_queue(hkv_table *t, const uint8_t *inv_out, const int32_t *inv_count, int32_t n_workers,
                           int32_t inv_stride, uint32_t op_size, uint8_t *aq, uint32_t ack_size, int32_t q_stride,
                           int32_t *aq_n, const int32_t *vq_n, int32_t *acnt, const uint8_t *peer_ids, int32_t n_peers,
                           const unsigned long long *peer_ts, uint32_t round, void *stream)
{
    if (n_peers <= 0 || n_workers <= 0 || ack_size < kOpMetaSize || ack_size % 8 || q_stride <= 0) return -1;
    TableView tv{};
    if (peer_ts && table_view(t, &tv)) return -1;
    hipLaunchKernelGGL(k_peer_acks_q, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, inv_out, inv_count, inv_stride,
                       op_size, aq, ack_size, q_stride, aq_n, vq_n, acnt, peer_ids, n_peers, tv, peer_ts, round);
    return ok();
}

int hkv_wl_vals_credit(uint8_t *aq, int32_t *aq_n, const int32_t *acnt, int32_t n_workers, int32_t q_stride,
                       uint32_t ack_size, uint8_t *vq, int32_t *vq_n, int32_t vq_stride, uint8_t *out,
                       int32_t *out_count, int32_t out_stride, int32_t v_credits, uint32_t machine_id,
                       unsigned long long *overflow, void *stream)
{
    if (n_workers <= 0 || ack_size % 8 || vq_stride <= 0 || out_stride <= 0 || v_credits < 0) return -1;
    hipLaunchKernelGGL(k_vals_credit, dim3(n_workers), dim3(256), 0, (hipStream_t)stream, aq, aq_n, acnt, q_stride,
                       ack_size, vq, vq_n, vq_stride, out, out_count, out_stride, v_credits, machine_id, overflow);
    return ok();
}

}  // extern "C"

extern "C" {

int hkv_wl_peer_locate(hkv_table *t, const uint8_t *invs, int64_t n, uint32_t op_size, uint64_t *phys_out, void *stream)
{
    TableView tv;
    if (table_view(t, &tv) || n < 0 || op_size % 8) return -1;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_peer_locate, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, tv, invs, op_size, n,
                       phys_out);
    return ok();
}

int hkv_wl_peer_ts_at(hkv_table *t, uint8_t *invs, uint8_t *vals, const uint64_t *phys, int64_t n, uint32_t op_size,
                      unsigned long long *peer_ts, uint32_t round, void *stream)
{
    TableView tv;
    if (table_view(t, &tv) || n < 0 || op_size % 8) return -1;
    if (n == 0) return 0;
    const PeerTsArgs pt{tv, invs, vals, phys, n, op_size, peer_ts, round};
    hipLaunchKernelGGL(k_peer_ts_at, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, pt);
    return ok();
}

int hkv_wl_refill_plan_peer_ts(uint8_t *states, int32_t n_workers, int32_t stride, uint32_t st_value, uint32_t shift,
                               const uint64_t *tkey, const uint8_t *top, int32_t tlen, uint32_t *cursor,
                               uint32_t machine_id, uint32_t flags, unsigned long long *counters, uint8_t *opc,
                               uint8_t *patch, hkv_table *t, uint8_t *invs, uint8_t *vals, const uint64_t *phys, int64_t n,
                               uint32_t op_size, unsigned long long *peer_ts, uint32_t round, void *stream)
{
    if (stride > 256 || n_workers <= 0 || tlen <= 0 || !states || !opc || !patch) return -1;
    if (flags & ~(uint32_t)(HKV_WL_REFILL_ALL | HKV_WL_READ_TS_RESET)) return -1;
    if (((uintptr_t)patch & 15) || (st_value >> shift) > 255) return -1;
    TableView tv;
    if (table_view(t, &tv) || n < 0 || op_size % 8) return -1;
    const PlanArgs pa{states, n_workers, stride, st_value, shift, tkey, top, tlen, cursor, machine_id, flags, counters, opc,
                      patch};
    const PeerTsArgs pt{tv, invs, vals, phys, n, op_size, peer_ts, round};
    const int plan_blocks = (n_workers + 7) / 8;
#ifdef HKV_PLAN_PTS_SPLIT   // (a build macro for A/B: the two launches of before)
    hipLaunchKernelGGL(k_refill_plan_w<2>, dim3((unsigned)plan_blocks), dim3(256), 0, (hipStream_t)stream, pa);
    if (n) hipLaunchKernelGGL(k_peer_ts_at, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, pt);
#else
    hipLaunchKernelGGL(k_plan_peer_ts, dim3((unsigned)plan_blocks + blocks_for(n)), dim3(256), 0, (hipStream_t)stream, pa,
                       pt, plan_blocks);
#endif
    return ok();
}

}  // extern "C"
