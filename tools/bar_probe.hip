// Host-pointer call latency: where should a caller's batch live for one small launch?
//   pinned   the batch in pinned host memory, read by the kernel over PCIe (the library's k_hpart)
//   vram     the batch written by the host CPU straight into fine-grained device memory (through the
//            BAR, posted write-combined stores), read by the kernel from HBM
// Each call: the host fills N bytes, launches one workgroup that reads them, writes N bytes of results
// to pinned memory and then a completion word; the host spins on the word and reads the results.
// Prints whether device memory is host-writable here and the average call time of each placement.
//   tools/bar_probe [bytes] [calls]
#include <hip/hip_runtime.h>
#include <csetjmp>
#include <csignal>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>

static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }

__global__ __launch_bounds__(256) void k_echo(const uint64_t *in, uint64_t *out, uint32_t n8, uint32_t *flag,
                                              uint32_t seq)
{
    for (uint32_t i = threadIdx.x; i < n8; i += 256) out[i] = in[i] ^ 0x5A5A5A5A5A5A5A5Aull;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static bool host_writable(void *p)
{
    struct sigaction sa = {}, old;
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old);
    sigaction(SIGBUS, &sa, nullptr);
    bool ok = false;
    if (sigsetjmp(jb, 1) == 0) {
        volatile uint64_t *v = reinterpret_cast<volatile uint64_t *>(p);
        v[0] = 0x1234;
        __builtin_ia32_sfence();
        ok = v[0] == 0x1234;
    }
    sigaction(SIGSEGV, &old, nullptr);
    signal(SIGBUS, SIG_DFL);
    return ok;
}

static double run(const char *name, uint64_t *in, uint64_t *out, uint32_t *flag, size_t bytes, int calls,
                  hipStream_t s)
{
    const uint32_t n8 = (uint32_t)(bytes / 8);
    uint64_t *src = (uint64_t *)malloc(bytes);
    for (uint32_t i = 0; i < n8; ++i) src[i] = i * 0x9E3779B97F4A7C15ull;
    double total = 0;
    uint64_t bad = 0;
    for (int c = -50; c < calls; ++c) {
        const uint32_t seq = (uint32_t)(c + 1000);
        src[0] = seq;
        auto t0 = std::chrono::steady_clock::now();
        memcpy(in, src, bytes);
        __builtin_ia32_sfence();
        hipLaunchKernelGGL(k_echo, dim3(1), dim3(256), 0, s, in, out, n8, flag, seq);
        uint64_t spins = 0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq)
            if (++spins > 2000000000ull) { printf("%s: completion word never came\n", name); hipStreamSynchronize(s); return -1; }
        bad += out[0] != (seq ^ 0x5A5A5A5A5A5A5A5Aull) || out[n8 - 1] != (src[n8 - 1] ^ 0x5A5A5A5A5A5A5A5Aull);
        auto t1 = std::chrono::steady_clock::now();
        if (c >= 0) total += std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    hipStreamSynchronize(s);
    free(src);
    printf("%-8s %zu B per call: %.2f us per call (%d calls, %llu wrong)\n", name, bytes, total / calls, calls,
           (unsigned long long)bad);
    return total / calls;
}

int main(int argc, char **argv)
{
    const size_t bytes = argc > 1 ? (size_t)atol(argv[1]) : 14000;
    const int calls = argc > 2 ? atoi(argv[2]) : 2000;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    uint64_t *pin_in, *pin_out;
    uint32_t *flag;
    hipHostMalloc((void **)&pin_in, bytes, hipHostMallocDefault);
    hipHostMalloc((void **)&pin_out, bytes, hipHostMallocDefault);
    hipHostMalloc((void **)&flag, 64, hipHostMallocDefault);
    *flag = 0;
    run("pinned", pin_in, pin_out, flag, bytes, calls, s);
    const unsigned flags[2] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    const char *names[2] = {"vram-fg", "vram-uc"};
    for (int m = 0; m < 2; ++m) {
        void *d = nullptr;
        if (hipExtMallocWithFlags(&d, bytes, flags[m]) != hipSuccess) { printf("%s: alloc failed\n", names[m]); continue; }
        hipPointerAttribute_t at;
        const bool attr = hipPointerGetAttributes(&at, d) == hipSuccess;
        const bool w = host_writable(d);
        printf("%s: device %p, host pointer %p (attr %d), host-writable %d\n", names[m], d, attr ? at.hostPointer : nullptr,
               (int)attr, (int)w);
        if (w) run(names[m], (uint64_t *)d, pin_out, flag, bytes, calls, s);
        hipFree(d);
    }
    void *d = nullptr;
    hipMalloc(&d, bytes);
    printf("hipMalloc: host-writable %d\n", (int)host_writable(d));
    hipFree(d);
    return 0;
}
