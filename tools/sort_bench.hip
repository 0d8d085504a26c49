// tools/sort_bench.hip -- picks the rocPRIM onesweep configuration for the batch sort:
// stable (entry id, element index) pairs, 28 key bits, at the launch sizes bench.py uses.
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <vector>
#include <random>

template <unsigned BS, unsigned IPT, unsigned BITS>
using OS = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                      rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                                          rocprim::kernel_config<BS, IPT>, BITS,
                                                                          rocprim::block_radix_rank_algorithm::match>,
                                      0>;
using Def = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

template <class C>
void run(const char *name, size_t n, const uint32_t *k, uint32_t *k2, const uint32_t *v, uint32_t *v2)
{
    size_t tb = 0;
    rocprim::radix_sort_pairs<C>(nullptr, tb, k, k2, v, v2, n, 0u, 28u);
    void *tmp;
    hipMalloc(&tmp, tb);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) rocprim::radix_sort_pairs<C>(tmp, tb, k, k2, v, v2, n, 0u, 28u);
    hipEventRecord(a);
    const int it = 20;
    for (int i = 0; i < it; ++i) rocprim::radix_sort_pairs<C>(tmp, tb, k, k2, v, v2, n, 0u, 28u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("n=%9zu %-24s %8.1f us\n", n, name, ms * 1000 / it);
    hipFree(tmp);
}

int main()
{
    for (size_t n : {819200ul, 2048000ul, 4096000ul, 8192000ul}) {
        std::vector<uint32_t> hk(n), hv(n);
        std::mt19937 rng(1);
        for (size_t i = 0; i < n; ++i) {
            hk[i] = rng() & ((1u << 27) - 1);
            hv[i] = (uint32_t)i;
        }
        uint32_t *k, *k2, *v, *v2;
        hipMalloc(&k, n * 4);
        hipMalloc(&k2, n * 4);
        hipMalloc(&v, n * 4);
        hipMalloc(&v2, n * 4);
        hipMemcpy(k, hk.data(), n * 4, hipMemcpyHostToDevice);
        hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice);
        run<Def>("default", n, k, k2, v, v2);
        run<OS<1024, 16, 8>>("os 1024x16 b8", n, k, k2, v, v2);
        run<OS<512, 8, 8>>("os 512x8 b8", n, k, k2, v, v2);
        run<OS<256, 8, 8>>("os 256x8 b8", n, k, k2, v, v2);
        run<OS<256, 16, 8>>("os 256x16 b8", n, k, k2, v, v2);
        run<OS<512, 4, 8>>("os 512x4 b8", n, k, k2, v, v2);
        run<OS<256, 8, 7>>("os 256x8 b7", n, k, k2, v, v2);
        run<OS<512, 8, 10>>("os 512x8 b10", n, k, k2, v, v2);
        run<OS<256, 8, 10>>("os 256x8 b10", n, k, k2, v, v2);
        run<OS<1024, 8, 10>>("os 1024x8 b10", n, k, k2, v, v2);
        run<OS<512, 16, 10>>("os 512x16 b10", n, k, k2, v, v2);
        hipFree(k);
        hipFree(k2);
        hipFree(v);
        hipFree(v2);
    }
    return 0;
}
