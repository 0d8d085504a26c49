// Microbenchmark behind the local launch's PUT-prepass redesign: what random
// accesses cost on MI355X by the size of the region they land in.
//   * random 16-B loads (one per thread, the shape of a key-table probe);
//   * random 8-B atomicMin / atomicCAS (one per thread, the shape of a first-PUT offer / slot claim);
//   * random 1-B stores (the shape of a seqlock-byte tag).
// Regions: 4 MiB (XCD L2), 32 MiB and 128 MiB (MALL), 1 GiB and 8 GiB (HBM). Indices come from a
// multiplicative hash of the thread id, masked to the region: every access is in bounds.
//   hipcc -O3 --offload-arch=gfx950 tools/table_bench.hip -o tools/table_bench && tools/table_bench
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

__global__ void k_load16(const uint4 *t, uint64_t mask16, uint32_t n, uint32_t salt, uint32_t *sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 v = t[mix(i ^ ((uint64_t)salt << 32)) & mask16];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = 1;
}

__global__ void k_amin(unsigned long long *t, uint64_t mask8, uint32_t n, uint32_t salt)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    atomicMin(t + (mix(i ^ ((uint64_t)salt << 32)) & mask8), (unsigned long long)i);
}

__global__ void k_cas(unsigned long long *t, uint64_t mask8, uint32_t n, uint32_t salt)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    atomicCAS(t + (mix(i ^ ((uint64_t)salt << 32)) & mask8), 0ull, (unsigned long long)i + 1);
}

__global__ void k_byte(uint8_t *t, uint64_t mask, uint32_t n, uint32_t salt)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    t[(mix(i ^ ((uint64_t)salt << 32)) & mask) | 4] = (uint8_t)i;
}

int main()
{
    const size_t big = 8ull << 30;
    uint8_t *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, big));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t regions[] = {4ull << 20, 32ull << 20, 128ull << 20, 1ull << 30, 8ull << 30};
    const uint32_t counts[] = {500000, 1000000, 4000000};
    printf("{\"what\": \"random accesses per second by region size (MI355X)\", \"rows\": [\n");
    bool first = true;
    for (size_t r : regions) {
        for (uint32_t n : counts) {
            for (int kind = 0; kind < 4; ++kind) {
                float best = 1e30f;
                for (int rep = 0; rep < 5; ++rep) {
                    const dim3 g((n + 255) / 256);
                    CK(hipEventRecord(e0));
                    if (kind == 0) hipLaunchKernelGGL(k_load16, g, dim3(256), 0, 0, (const uint4 *)buf, r / 16 - 1, n, rep, sink);
                    if (kind == 1) hipLaunchKernelGGL(k_amin, g, dim3(256), 0, 0, (unsigned long long *)buf, r / 8 - 1, n, rep);
                    if (kind == 2) hipLaunchKernelGGL(k_cas, g, dim3(256), 0, 0, (unsigned long long *)buf, r / 8 - 1, n, rep);
                    if (kind == 3) hipLaunchKernelGGL(k_byte, g, dim3(256), 0, 0, buf, (r - 1) & ~63ull, n, rep);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (ms < best) best = ms;
                }
                static const char *names[] = {"load16", "atomicMin64", "atomicCAS64", "store8"};
                printf("%s{\"region_mib\": %zu, \"n\": %u, \"kind\": \"%s\", \"us\": %.2f, \"g_per_s\": %.2f}", first ? "" : ",\n",
                       r >> 20, n, names[kind], best * 1e3, n / (best * 1e-3) / 1e9);
                first = false;
            }
        }
    }
    printf("\n]}\n");
    CK(hipFree(buf));
    return 0;
}
