// Microbenchmark: HBM cost of writes that leave holes in the lines they touch (partial-line writes)
// against whole-line writes, over an op slab of 4M 312-byte ops (configs[2]'s layout).
//   hipcc -O3 --offload-arch=gfx950 -o tools/write_bench tools/write_bench.hip && tools/write_bench
// Each wave owns 64 consecutive ops; lane l stores 8-byte words l, l + 64, ... of that region.
// mode 0  every word (whole lines)
// mode 1  every word but each op's first (an 8-byte hole every 312 bytes: the key a GET's result
//         does not rewrite)
// mode 2  only each op's words 1 and 2 (bytes 8..23: what a refill writes of a GET)
// mode 3  mode 1 after loading each op's first word (the holes' lines read first)
// mode 4  every word after loading each op's first word
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kOpWords = 39;   // 312 bytes

__global__ __launch_bounds__(256) void k_write(uint64_t *slab, int64_t n_ops, int mode, uint64_t *sink)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t op0 = wave * 64;
    if (op0 >= n_ops) return;
    uint64_t *base = slab + op0 * kOpWords;
    uint64_t acc = 0;
    if (mode >= 3) acc = base[(int64_t)lane * kOpWords];
    const uint64_t v = 0x6161616161616161ull + (acc & 1);
    for (int w = lane; w < 64 * kOpWords; w += 64) {
        const int wi = w % kOpWords;
        bool st = true;
        if (mode == 1 || mode == 3) st = wi != 0;
        else if (mode == 2) st = wi == 1 || wi == 2;
        if (st) base[w] = v;
    }
    if (acc == 0x123456789ull) sink[0] = acc;
}

int main()
{
    const int64_t n_ops = 4 << 20;
    uint64_t *slab, *sink;
    hipMalloc(&slab, n_ops * kOpWords * 8);
    hipMalloc(&sink, 64);
    hipMemset(slab, 0, n_ops * kOpWords * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned grid = (unsigned)((n_ops / 64 * 64 + 255) / 256);
    const double algo[5] = {312.0, 304.0, 16.0, 312.0, 312.0};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 5; ++mode) {
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, slab, n_ops, mode, sink);
            hipEventRecord(e0);
            const int it = 5;
            for (int k = 0; k < it; ++k) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, slab, n_ops, mode, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1000.0 / it;
            printf("rep %d mode %d: %8.1f us per launch, %6.2f TB/s of bytes stored, %6.2f TB/s of slab\n", rep, mode, us,
                   n_ops * algo[mode] / us / 1e6, n_ops * 312.0 / us / 1e6);
        }
    hipFree(slab);
    return 0;
}
