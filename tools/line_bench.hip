// Microbenchmark for where a key's F word lives: the shape of
// k_local_fused's lookup chain, four lanes per element, two elements per lane group, 4M elements:
//   A  bucket 64 B -> entry line 64 B, plus the F word (8 B) at a scrambled index beside the line
//      (the F array: one word per log line, the round-5 layout);
//   B  bucket 128 B (the bucket and its slots' F words side by side, 32 B per lane) -> entry line
//      64 B: the F word comes with the bucket;
//   C  bucket 64 B -> entry line 64 B, no F word (the floor of the chain).
// and the prepass's offer after a lookup: an atomicMin on the scrambled F array (D) or on the
// bucket's side half the lookup just read (E). The entry address depends on the bucket's bytes, as a
// real lookup's does. Index 2 GiB (buckets at 64 or 128 B), log 4 GiB, F array 512 MiB.
//   hipcc -O3 --offload-arch=gfx950 tools/line_bench.hip -o tools/line_bench && tools/line_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x)
{
    x ^= x >> 31; x *= 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    return x;
}

// MODE 0: A, 1: B, 2: C, 3: D (offer to the F array), 4: E (offer to the bucket's side half)
template <int MODE>
__global__ __launch_bounds__(64) void k_chain(const uint8_t *index, uint64_t nb, const uint8_t *log, uint64_t nl,
                                              unsigned long long *fw, uint64_t nf, uint32_t n, uint32_t salt,
                                              uint32_t *sink)
{
    const int tid = threadIdx.x, q = tid & 3;
    const uint32_t e0 = blockIdx.x * 32 + (tid >> 2);
    const int stride = MODE == 1 || MODE == 4 ? 128 : 64;
    uint4 b[2], s[2], l[2];
    uint64_t bk[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t e = e0 + 16 * k;
        bk[k] = mix(e ^ ((uint64_t)salt << 32)) & (nb - 1);
        const uint8_t *bp = index + bk[k] * stride;
        b[k] = e < n ? reinterpret_cast<const uint4 *>(bp)[q] : make_uint4(0, 0, 0, 0);
        s[k] = (MODE == 1) && e < n ? reinterpret_cast<const uint4 *>(bp + 64)[q] : make_uint4(0, 0, 0, 0);
    }
    uint64_t ln[2];
    unsigned long long f[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t v = (uint32_t)__shfl((int)(b[k].x ^ b[k].y ^ b[k].z ^ b[k].w), 0, 4);
        ln[k] = mix(bk[k] * 7 + v) & (nl - 1);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t e = e0 + 16 * k;
        l[k] = e < n ? reinterpret_cast<const uint4 *>(log + ln[k] * 64)[q] : make_uint4(0, 0, 0, 0);
        if (MODE == 0 && e < n && q == 0) f[k] = fw[(ln[k] * 0x9E3779B1ull) & (nf - 1)];
        if (MODE == 1) f[k] = (unsigned long long)s[k].x | ((unsigned long long)s[k].y << 32);
    }
    if (MODE == 3 || MODE == 4) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t e = e0 + 16 * k;
            const uint32_t v = (uint32_t)__shfl((int)(l[k].x ^ l[k].y), 0, 4);
            if (e < n && q == 0 && v != 0x12345678u) {
                unsigned long long *w = MODE == 3 ? fw + ((ln[k] * 0x9E3779B1ull) & (nf - 1))
                                                  : reinterpret_cast<unsigned long long *>(const_cast<uint8_t *>(index) + bk[k] * 128 + 64) + (e & 7);
                atomicMin(w, (unsigned long long)e);
            }
        }
        return;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) acc ^= l[k].x ^ l[k].y ^ l[k].z ^ l[k].w ^ (uint32_t)f[k] ^ s[k].z;
    if (acc == 0x12345678u) sink[0] = acc;
}

int main()
{
    const uint64_t index_bytes = 4ull << 30, log_bytes = 4ull << 30, fw_bytes = 512ull << 20;
    uint8_t *index, *log;
    unsigned long long *fw;
    uint32_t *sink;
    CK(hipMalloc(&index, index_bytes));
    CK(hipMalloc(&log, log_bytes));
    CK(hipMalloc(&fw, fw_bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(index, 0x11, index_bytes));
    CK(hipMemset(log, 0x22, log_bytes));
    CK(hipMemset(fw, 0xFF, fw_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t n = 4u << 20;
    const dim3 g((n + 31) / 32);
    printf("{\"what\": \"lookup chain per element, 4M elements, 4 lanes each (MI355X)\", \"rows\": [\n");
    static const char *names[] = {"A bucket64+entry+F(array)", "B bucket128(F side)+entry", "C bucket64+entry (no F)",
                                  "D lookup + atomicMin F array", "E lookup + atomicMin bucket side",
                                  "B' bucket128 as many buckets as A (2x footprint)", "E' atomicMin bucket side, 2x footprint"};
    for (int mode = 0; mode < 7; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 7; ++rep) {
            // A, C, D: 2 GiB of 64-B buckets; B, E: the same 2 GiB at 128 B (half the buckets); B', E': as
            // many buckets as A at 128 B (4 GiB)
            const uint64_t nb = mode >= 5 ? index_bytes / 128 : (mode == 1 || mode == 4 ? index_bytes / 256 : index_bytes / 128);
            CK(hipEventRecord(e0));
            if (mode == 0) hipLaunchKernelGGL(k_chain<0>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 1) hipLaunchKernelGGL(k_chain<1>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 2) hipLaunchKernelGGL(k_chain<2>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 3) hipLaunchKernelGGL(k_chain<3>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 5) hipLaunchKernelGGL(k_chain<1>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 6) hipLaunchKernelGGL(k_chain<4>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            if (mode == 4) hipLaunchKernelGGL(k_chain<4>, g, dim3(64), 0, 0, index, nb, log, log_bytes / 64, fw, fw_bytes / 8, n, rep, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;
        }
        printf("%s{\"mode\": \"%s\", \"us\": %.2f, \"g_elems_per_s\": %.2f}", mode ? ",\n" : "", names[mode], best * 1e3,
               n / (best * 1e-3) / 1e9);
    }
    printf("\n]}\n");
    return 0;
}
