// Microbenchmark: cost of byte-masked (partial-line) stores into an array of 56-byte ops, the
// layout of spacetime_op_t, against full-line stores and read+write staging.
//   hipcc -O3 --offload-arch=gfx950 tools/partial_write_bench.hip -o tools/partial_write_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kOp = 56;

// (a) read + write every op (16-B loads and stores of the slab)
__global__ void k_rw(uint4 *p, int64_t n16)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16) {
        uint4 v = p[i];
        v.x += 1;
        p[i] = v;
    }
}

// (b) write every byte of every op, no read
__global__ void k_wfull(uint4 *p, int64_t n16)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16) p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

// (c) per op: bytes 9..15 and 18..48 (a GET hit's result), nothing else; one thread per op
__global__ void k_wpart(uint8_t *p, int64_t n)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *o = p + i * kOp;
    o[9] = 1;
    o[10] = 2;
    o[11] = 3;
    *reinterpret_cast<uint32_t *>(o + 12) = (uint32_t)i;
    *reinterpret_cast<uint16_t *>(o + 18) = 5;
    *reinterpret_cast<uint32_t *>(o + 20) = 6;
    *reinterpret_cast<uint64_t *>(o + 24) = 7;
    *reinterpret_cast<uint64_t *>(o + 32) = 8;
    *reinterpret_cast<uint64_t *>(o + 40) = 9;
    o[48] = 10;
}

// (d) read each op's 16-B header only
__global__ void k_rhdr(const uint8_t *p, int64_t n, uint64_t *sink)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t *h = reinterpret_cast<const uint64_t *>(p + i * kOp);
    uint64_t v = h[0] ^ h[1];
    if (v == 0x1234567) *sink = v;
}

// (e) per op: one state byte (the INV marshal's op state update)
__global__ void k_wbyte(uint8_t *p, int64_t n)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i * kOp + 9] = 7;
}

// (f) k_lookup's pattern: 4-lane groups, two elements per group, lane 0 loads the 16-B header
__global__ void k_rhdr_groups(const uint8_t *p, int64_t n, uint64_t *sink)
{
    const int q = threadIdx.x & 3;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int64_t gi = ((int64_t)blockIdx.x * 2 + k) * 64 + (threadIdx.x >> 2);
        if (gi < n && q == 0) {
            const uint4 h = *reinterpret_cast<const uint4 *>(p + gi * kOp);
            acc ^= h.x ^ h.z;
        }
    }
    if (acc == 0x1234567) *sink = acc;
}

// (g) the same 128 headers per block from a coalesced 16-B slab load through LDS
__global__ void k_rhdr_lds(const uint8_t *p, int64_t n, uint64_t *sink)
{
    __shared__ uint4 slab[128 * kOp / 16];
    const int64_t e0 = (int64_t)blockIdx.x * 128;
    const int cnt = n - e0 < 128 ? (int)(n - e0) : 128;
    const uint4 *src = reinterpret_cast<const uint4 *>(p + e0 * kOp);
    for (int w = threadIdx.x; w < cnt * kOp / 16; w += 256) slab[w] = src[w];
    __syncthreads();
    uint64_t acc = 0;
    const int q = threadIdx.x & 3;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int e = k * 64 + (threadIdx.x >> 2);
        if (e < cnt && q == 0) {
            const uint64_t *h = reinterpret_cast<const uint64_t *>(reinterpret_cast<const uint8_t *>(slab) + e * kOp);
            acc ^= h[0] ^ h[1];
        }
    }
    if (acc == 0x1234567) *sink = acc;
}

// evicts L2 / MALL with clean lines (a read, so no write-back lands in the timed kernel)
__global__ void k_flush(const uint4 *f, int64_t n16, uint64_t *sink)
{
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= f[i].x;
    if (acc == 0x1234567) *sink = acc;
}

int main()
{
    const int64_t n = 2048000, bytes = n * kOp, n16 = bytes / 16;
    uint8_t *p;
    uint64_t *sink;
    hipMalloc(&p, bytes + 64);
    hipMalloc(&sink, 8);
    hipMemset(p, 0, bytes);
    uint8_t *flush;
    const size_t fb = (size_t)1 << 30;  // evict L2 / MALL between runs
    hipMalloc(&flush, fb);
    hipMemset(flush, 1, fb);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[] = {"read+write 16B", "write full 16B", "write GET-result bytes", "read 16B header",
                           "write state byte", "read hdr, lookup lanes", "read hdr, LDS slab"};
    for (int k = 0; k < 7; ++k) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (const uint4 *)flush, (int64_t)(fb / 16), sink);
            hipEventRecord(a);
            if (k == 0) hipLaunchKernelGGL(k_rw, dim3((n16 + 255) / 256), dim3(256), 0, 0, (uint4 *)p, n16);
            if (k == 1) hipLaunchKernelGGL(k_wfull, dim3((n16 + 255) / 256), dim3(256), 0, 0, (uint4 *)p, n16);
            if (k == 2) hipLaunchKernelGGL(k_wpart, dim3((n + 255) / 256), dim3(256), 0, 0, p, n);
            if (k == 3) hipLaunchKernelGGL(k_rhdr, dim3((n + 255) / 256), dim3(256), 0, 0, p, n, sink);
            if (k == 4) hipLaunchKernelGGL(k_wbyte, dim3((n + 255) / 256), dim3(256), 0, 0, p, n);
            if (k == 5) hipLaunchKernelGGL(k_rhdr_groups, dim3((n + 127) / 128), dim3(256), 0, 0, p, n, sink);
            if (k == 6) hipLaunchKernelGGL(k_rhdr_lds, dim3((n + 127) / 128), dim3(256), 0, 0, p, n, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("%-24s %8.1f us  %7.0f GB/s of slab\n", names[k], best * 1e3, bytes / (best * 1e-3) / 1e9);
    }
    return 0;
}
