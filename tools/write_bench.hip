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
// The slab as 64-byte chunks, one per lane (the log's 64-byte entries):
// mode 5  every chunk whole
// mode 6  even chunks only (whole 64-byte halves of each 128-byte line)
// mode 7  bytes 16..63 of every chunk (an INV's meta and value, not the key)
// mode 8  bytes 0..31 of every chunk (whole 32-byte halves)
// Four lanes per 64-byte chunk, 16 bytes a lane (how the batch kernels write entries):
// mode 9   every chunk whole
// mode 10  even chunks only
// mode 11  bytes 16..63 of every chunk
// mode 12  bytes 32..63 of every chunk
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

__global__ __launch_bounds__(256) void k_chunks(uint64_t *slab, int64_t n_chunks, int mode)
{
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n_chunks) return;
    if (mode == 6 && (c & 1)) return;
    uint64_t *p = slab + c * 8;
    const int lo = mode == 7 ? 2 : 0, hi = mode == 8 ? 4 : 8;
    for (int k = lo; k < hi; ++k) p[k] = 0x6262626262626262ull;
}

struct __attribute__((aligned(16))) V16 {
    uint64_t a, b;
};
__global__ __launch_bounds__(256) void k_quads(V16 *slab, int64_t n_chunks, int mode)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t c = t >> 2;
    const int q = (int)(t & 3);
    if (c >= n_chunks) return;
    if (mode == 10 && (c & 1)) return;
    if (mode == 11 && q < 1) return;
    if (mode == 12 && q < 2) return;
    slab[t] = V16{0x6363636363636363ull, 0x6363636363636363ull};
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
    const int64_t n_chunks = n_ops * kOpWords / 8;
    const unsigned cgrid = (unsigned)((n_chunks + 255) / 256);
    const double cb[9] = {0, 0, 0, 0, 0, 64.0, 32.0, 48.0, 32.0};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 5; mode < 9; ++mode) {
            hipLaunchKernelGGL(k_chunks, dim3(cgrid), dim3(256), 0, 0, slab, n_chunks, mode);
            hipEventRecord(e0);
            const int it = 5;
            for (int k = 0; k < it; ++k) hipLaunchKernelGGL(k_chunks, dim3(cgrid), dim3(256), 0, 0, slab, n_chunks, mode);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1000.0 / it;
            printf("rep %d mode %d: %8.1f us per launch, %6.2f TB/s of bytes stored, %6.2f TB/s of slab\n", rep, mode, us,
                   n_chunks * cb[mode] / us / 1e6, n_chunks * 64.0 / us / 1e6);
        }
    const double qb[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 64.0, 32.0, 48.0, 32.0};
    const unsigned qgrid = (unsigned)((n_chunks * 4 + 255) / 256);
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 9; mode < 13; ++mode) {
            hipLaunchKernelGGL(k_quads, dim3(qgrid), dim3(256), 0, 0, reinterpret_cast<V16 *>(slab), n_chunks, mode);
            hipEventRecord(e0);
            const int it = 5;
            for (int k = 0; k < it; ++k)
                hipLaunchKernelGGL(k_quads, dim3(qgrid), dim3(256), 0, 0, reinterpret_cast<V16 *>(slab), n_chunks, mode);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1000.0 / it;
            printf("rep %d mode %d: %8.1f us per launch, %6.2f TB/s of bytes stored, %6.2f TB/s of slab\n", rep, mode, us,
                   n_chunks * qb[mode] / us / 1e6, n_chunks * 64.0 / us / 1e6);
        }
    hipFree(slab);
    return 0;
}
