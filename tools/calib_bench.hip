// Counter calibration for the access shapes of the batch kernels ("Make roofline.traffic
// trustworthy"): every kernel below touches a KNOWN number of records of a known width, so the
// FETCH_SIZE / WRITE_SIZE (and TCC_EA0_* request) counters rocprofv3 reports for it can be divided by
// the bytes actually asked for. One JSON line per kernel: name, records, record bytes, distinct 128-B
// lines, span of the addresses, ms per launch (HIP events, the median of 3 launches).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/calib_bench tools/calib_bench.hip
//   tools/calib_bench            (under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / ... : tools/calib.sh)
//
// Records are visited in a scattered order that touches each slot exactly once (slot = i * odd mod 2^k,
// a bijection), so nothing is re-read by design and caches only see what the shape itself shares.
// Shapes:
//   rd_rec{8,16,64,128}_s128   one W-byte record at the start of each of 2^24 128-B lines (2 GiB span):
//                              the F word (8 B), a 16-B chunk, a bucket or entry (64 B, 4 lanes x 16 B),
//                              a whole line (8 lanes x 16 B)
//   rd_rec64_both              every 64-B record of those 2^24 lines (both halves of each line, each read once,
//                              at unrelated times): log entries, which share 128-B lines pairwise
//   rd_rec64_s{512,1024}       2^24 64-B records, one per 512-B / 1-KiB slot (8 / 16 GiB span): the same
//                              number of lines as rd_rec64_s128 behind more pages (translation reach)
//   rd_rec64_s1024_contig      rd_rec64_s1024 on a hipDeviceMallocContiguous buffer
//   rd_stream16                2 GiB read 16 B per lane, in order (the guide's calibrated case)
//   rd_ops56                   2^24 56-B ops in order, lanes 16/16/16/8 B (the op slab as k_local_fused reads it)
//   wr_rec{8,16,64,128}_s128   the write twins of rd_rec*_s128
//   wr_stream16                2 GiB written 16 B per lane, in order
//   wr_ops56                   the op slab written back as k_local_fused writes it
//   at_min8_s128               one 8-B atomicMin per line, 2^24 lines (the prepass's offers)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr uint64_t kRecs = 1ull << 24;      // records (or slots) per kernel
constexpr uint32_t kMul = 0x9E3779B1u;      // odd: i -> i * kMul mod 2^k is a bijection

__device__ __forceinline__ uint64_t slot_of(uint64_t i, uint64_t mask) { return (i * kMul) & mask; }

// W-byte record per slot, slot stride S bytes; L = W / 16 lanes per record (W >= 16), one lane for W = 8
template <int W, int S>
__device__ __forceinline__ void rd_body(const uint8_t *buf, uint64_t nrec, uint64_t mask, unsigned long long *sink)
{
    constexpr int L = W >= 16 ? W / 16 : 1;
    constexpr int RPW = 64 / L;   // records per wave instruction
    const int lane = threadIdx.x & 63, sub = lane % L;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    for (uint64_t base = wave * RPW * 4; base < nrec; base += nw * RPW * 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t i = base + (uint64_t)u * RPW + lane / L;
            v[u] = make_uint4(0, 0, 0, 0);
            if (i < nrec) {
                const uint8_t *p = buf + slot_of(i, mask) * S + sub * 16;
                if (W == 8) {
                    const uint64_t t = *reinterpret_cast<const uint64_t *>(p);
                    v[u].x = (uint32_t)t ^ (uint32_t)(t >> 32);
                } else {
                    v[u] = *reinterpret_cast<const uint4 *>(p);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

template <int W, int S>
__device__ __forceinline__ void wr_body(uint8_t *buf, uint64_t nrec, uint64_t mask)
{
    constexpr int L = W >= 16 ? W / 16 : 1;
    constexpr int RPW = 64 / L;
    const int lane = threadIdx.x & 63, sub = lane % L;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t base = wave * RPW * 4; base < nrec; base += nw * RPW * 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t i = base + (uint64_t)u * RPW + lane / L;
            if (i >= nrec) continue;
            uint8_t *p = buf + slot_of(i, mask) * S + sub * 16;
            if (W == 8) *reinterpret_cast<uint64_t *>(p) = i;
            else *reinterpret_cast<uint4 *>(p) = make_uint4((uint32_t)i, 1u, 2u, 3u);
        }
    }
}

#define RD_KERNEL(name, W, S)                                                                              \
    __global__ __launch_bounds__(256) void name(const uint8_t *b, uint64_t n, uint64_t m, unsigned long long *s) \
    {                                                                                                      \
        rd_body<W, S>(b, n, m, s);                                                                         \
    }
#define WR_KERNEL(name, W, S)                                                                              \
    __global__ __launch_bounds__(256) void name(uint8_t *b, uint64_t n, uint64_t m) { wr_body<W, S>(b, n, m); }

RD_KERNEL(rd_rec8_s128, 8, 128)
RD_KERNEL(rd_rec16_s128, 16, 128)
RD_KERNEL(rd_rec64_s128, 64, 128)
RD_KERNEL(rd_rec128_s128, 128, 128)
RD_KERNEL(rd_rec64_both, 64, 64)
RD_KERNEL(rd_rec64_s512, 64, 512)
RD_KERNEL(rd_rec64_s1024, 64, 1024)
RD_KERNEL(rd_rec64_s1024_contig, 64, 1024)
WR_KERNEL(wr_rec8_s128, 8, 128)
WR_KERNEL(wr_rec16_s128, 16, 128)
WR_KERNEL(wr_rec64_s128, 64, 128)
WR_KERNEL(wr_rec128_s128, 128, 128)

__global__ __launch_bounds__(256) void rd_stream16(const uint4 *b, uint64_t n16, unsigned long long *s)
{
    uint32_t acc = 0;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t; i < n16; i += nt) {
        const uint4 v = b[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(s, 1ull);
}

__global__ __launch_bounds__(256) void wr_stream16(uint4 *b, uint64_t n16)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t; i < n16; i += nt) b[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// four lanes per 56-B op: bytes 0..15, 16..31, 32..47 as 16-B loads, 48..55 as one 8-B load
__global__ __launch_bounds__(256) void rd_ops56(const uint8_t *b, uint64_t nops, unsigned long long *s)
{
    uint32_t acc = 0;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    const int q = t & 3;
    for (uint64_t g = t >> 2; g < nops; g += nt >> 2) {
        const uint8_t *p = b + g * 56 + 16 * q;
        if (q < 3) {
            const uint4 v = *reinterpret_cast<const uint4 *>(p);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else {
            const uint64_t v = *reinterpret_cast<const uint64_t *>(p);
            acc += (uint32_t)v ^ (uint32_t)(v >> 32);
        }
    }
    if (acc == 0x12345678u) atomicAdd(s, 1ull);
}

__global__ __launch_bounds__(256) void wr_ops56(uint8_t *b, uint64_t nops)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    const int q = t & 3;
    for (uint64_t g = t >> 2; g < nops; g += nt >> 2) {
        uint8_t *p = b + g * 56 + 16 * q;
        if (q < 3) *reinterpret_cast<uint4 *>(p) = make_uint4((uint32_t)g, 1u, 2u, 3u);
        else *reinterpret_cast<uint64_t *>(p) = g;
    }
}

__global__ __launch_bounds__(256) void at_min8_s128(uint8_t *b, uint64_t n, uint64_t m)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t; i < n; i += nt)
        atomicMin(reinterpret_cast<unsigned long long *>(b + slot_of(i, m) * 128), (unsigned long long)i);
}

static void check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

template <class F>
static float timed(F launch)
{
    hipEvent_t a, b;
    check(hipEventCreate(&a), "event");
    check(hipEventCreate(&b), "event");
    std::vector<float> ms;
    launch();   // warm (first touch of the span's pages)
    for (int r = 0; r < 3; ++r) {
        check(hipEventRecord(a), "record");
        launch();
        check(hipEventRecord(b), "record");
        check(hipEventSynchronize(b), "sync");
        float x;
        check(hipEventElapsedTime(&x, a, b), "elapsed");
        ms.push_back(x);
    }
    check(hipGetLastError(), "launch");
    std::sort(ms.begin(), ms.end());
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms[1];
}

static void line(const char *name, uint64_t recs, int w, uint64_t lines, uint64_t span, float ms)
{
    printf("{\"kernel\": \"%s\", \"records\": %llu, \"record_bytes\": %d, \"useful_bytes\": %llu, \"lines128\": %llu, "
           "\"span_bytes\": %llu, \"ms\": %.4f, \"useful_GBps\": %.1f, \"lines_per_us\": %.1f}\n",
           name, (unsigned long long)recs, w, (unsigned long long)(recs * w), (unsigned long long)lines,
           (unsigned long long)span, ms, recs * w / ms / 1e6, lines / ms / 1e3);
    fflush(stdout);
}

int main()
{
    const uint64_t span = kRecs * 1024;   // 16 GiB: the largest stride's span
    uint8_t *buf = nullptr, *cbuf = nullptr;
    unsigned long long *sink = nullptr;
    check(hipMalloc(&buf, span), "hipMalloc 16 GiB");
    check(hipMalloc(&sink, 8), "hipMalloc sink");
    check(hipMemset(buf, 1, span), "memset");
    const dim3 grid(256 * 32), blk(256);   // 32 waves per CU
    const uint64_t m24 = kRecs - 1, m25 = 2 * kRecs - 1;
#define RD(k, S, n, m, w, lines, sp)                                                                  \
    line(#k, n, w, lines, sp, timed([&] { hipLaunchKernelGGL(k, grid, blk, 0, 0, buf, n, m, sink); }))
#define WR(k, n, m, w, lines, sp) line(#k, n, w, lines, sp, timed([&] { hipLaunchKernelGGL(k, grid, blk, 0, 0, buf, n, m); }))
    RD(rd_rec8_s128, 128, kRecs, m24, 8, kRecs, kRecs * 128);
    RD(rd_rec16_s128, 128, kRecs, m24, 16, kRecs, kRecs * 128);
    RD(rd_rec64_s128, 128, kRecs, m24, 64, kRecs, kRecs * 128);
    RD(rd_rec128_s128, 128, kRecs, m24, 128, kRecs, kRecs * 128);
    RD(rd_rec64_both, 64, 2 * kRecs, m25, 64, kRecs, kRecs * 128);
    RD(rd_rec64_s512, 512, kRecs, m24, 64, kRecs, kRecs * 512);
    RD(rd_rec64_s1024, 1024, kRecs, m24, 64, kRecs, kRecs * 1024);
    line("rd_stream16", kRecs * 8, 16, kRecs, kRecs * 128,
         timed([&] { hipLaunchKernelGGL(rd_stream16, grid, blk, 0, 0, (const uint4 *)buf, kRecs * 8, sink); }));
    line("rd_ops56", kRecs, 56, kRecs * 56 / 128, kRecs * 56,
         timed([&] { hipLaunchKernelGGL(rd_ops56, grid, blk, 0, 0, buf, kRecs, sink); }));
    WR(wr_rec8_s128, kRecs, m24, 8, kRecs, kRecs * 128);
    WR(wr_rec16_s128, kRecs, m24, 16, kRecs, kRecs * 128);
    WR(wr_rec64_s128, kRecs, m24, 64, kRecs, kRecs * 128);
    WR(wr_rec128_s128, kRecs, m24, 128, kRecs, kRecs * 128);
    line("wr_stream16", kRecs * 8, 16, kRecs, kRecs * 128,
         timed([&] { hipLaunchKernelGGL(wr_stream16, grid, blk, 0, 0, (uint4 *)buf, kRecs * 8); }));
    line("wr_ops56", kRecs, 56, kRecs * 56 / 128, kRecs * 56,
         timed([&] { hipLaunchKernelGGL(wr_ops56, grid, blk, 0, 0, buf, kRecs); }));
    line("at_min8_s128", kRecs, 8, kRecs, kRecs * 128,
         timed([&] { hipLaunchKernelGGL(at_min8_s128, grid, blk, 0, 0, buf, kRecs, m24); }));
    check(hipFree(buf), "free");
    // translation reach with a physically contiguous allocation (larger fragments, if the driver grants them)
    if (hipExtMallocWithFlags((void **)&cbuf, span, hipDeviceMallocContiguous) == hipSuccess) {
        check(hipMemset(cbuf, 1, span), "memset contig");
        line("rd_rec64_s1024_contig", kRecs, 64, kRecs, span, timed([&] {
                 hipLaunchKernelGGL(rd_rec64_s1024_contig, grid, blk, 0, 0, cbuf, kRecs, m24, sink);
             }));
        hipFree(cbuf);
    } else {
        printf("{\"kernel\": \"rd_rec64_s1024_contig\", \"error\": \"hipDeviceMallocContiguous of 16 GiB refused\"}\n");
        (void)hipGetLastError();
    }
    hipFree(sink);
    return 0;
}
