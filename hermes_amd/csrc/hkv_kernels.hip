// hkv_kernels.hip -- CDNA4 (gfx950) kernels of table setup: CityHash128 of key ids and populate.
//
// Populate (spacetime.c:32-68 / mica.c:78-146): hash every id, sort the inserts by bucket (stable,
// so each bucket sees its inserts in insertion order), one owner lane per bucket replays the MICA
// slot rules, and the log entries are written in parallel. The batch path is in hkv_batch.hip.
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

// Stable LSD radix sort of (bucket, insert) pairs. rocPRIM picks a merge sort below 1M
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
