// Random 64-B reads (four lanes x 16 B, one 64-B aligned record per lane group) from an 8-GiB
// buffer: coarse-grained hipMalloc vs hipDeviceMallocFinegrained vs hipDeviceMallocUncached.
// Prints useful GB/s and the time per pass. tools/uc_bench [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__global__ __launch_bounds__(256) void k_rand64(const uint4 *buf, uint64_t nrec, uint32_t iters, uint64_t seed,
                                                unsigned long long *sink)
{
    const int q = threadIdx.x & 3;
    uint64_t g = (uint64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
    uint64_t x = seed ^ (g * 0x9E3779B97F4A7C15ull);
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint64_t r = x % nrec;
        const uint4 v = buf[r * 4 + q];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main(int argc, char **argv)
{
    const size_t gib = argc > 1 ? atoi(argv[1]) : 8;
    const size_t bytes = gib << 30;
    const uint64_t nrec = bytes / 64;
    const unsigned flags[3] = {0xFFFFFFFFu, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    const char *names[3] = {"hipMalloc", "fine-grained", "uncached"};
    unsigned long long *sink;
    hipMalloc(&sink, 8);
    for (int m = 0; m < 3; ++m) {
        void *p = nullptr;
        hipError_t e = flags[m] == 0xFFFFFFFFu ? hipMalloc(&p, bytes) : hipExtMallocWithFlags(&p, bytes, flags[m]);
        if (e != hipSuccess) { printf("%s: alloc failed %s\n", names[m], hipGetErrorString(e)); continue; }
        hipMemset(p, 1, bytes);
        hipDeviceSynchronize();
        const uint32_t blocks = 256 * 32, iters = 64;
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(k_rand64, dim3(blocks), dim3(256), 0, 0, (const uint4 *)p, nrec, iters, 1ull, sink);
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r)
            hipLaunchKernelGGL(k_rand64, dim3(blocks), dim3(256), 0, 0, (const uint4 *)p, nrec, iters, 2ull + r, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double recs = 5.0 * blocks * 64.0 * iters;
        printf("%-13s random 64-B records: %.1f M rec/s, %.0f GB/s useful (%.3f ms per pass)\n", names[m],
               recs / ms / 1e3, recs * 64 / ms / 1e6, ms / 5);
        hipFree(p);
    }
    return 0;
}
