// Development harness: LDS local sort of pre-split sub-buckets (2^msd equal ranges of
// random 32-bit keys whose top msd bits are the range id), 4 passes.
#include "proto/local_sort.hip"
#include <cstdio>
#include <vector>
#include <random>
using namespace mums;
int main(int argc, char** argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 800000000ull;
    const int msd = argc > 2 ? atoi(argv[2]) : 17;
    const uint64_t nb = 1ull << msd, bs = n / nb;
    n = bs * nb;
    std::vector<uint64_t> h(n);
    std::mt19937_64 r(7);
    for (uint64_t b = 0; b < nb; ++b)
        for (uint64_t i = 0; i < bs; ++i) {
            const uint64_t k = (b << (32 - msd)) | (r() & ((1ull << (32 - msd)) - 1));
            h[b * bs + i] = (k << 32) | (b * bs + i);
        }
    std::vector<uint64_t> rg(nb);
    for (uint64_t b = 0; b < nb; ++b) rg[b] = (b * bs) | (bs << 40);
    uint64_t *a, *o, *drg;
    (void)hipMalloc(&a, n * 8); (void)hipMalloc(&o, n * 8); (void)hipMalloc(&drg, nb * 8);
    (void)hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(drg, rg.data(), nb * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float tot = 0; const int K = 5;
    for (int it = 0; it <= K; ++it) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(local_sort_kernel<LT>, dim3((unsigned)nb), dim3(LT), 0, 0, a, o, drg, (uint32_t)nb, 32);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (it) tot += ms;
    }
    std::vector<uint64_t> out(n); (void)hipMemcpy(out.data(), o, n * 8, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 1; i < n; ++i) {
        const uint64_t a1 = out[i - 1] >> 32, a2 = out[i] >> 32;
        bad += (a2 < a1) || (a2 == a1 && (uint32_t)out[i] < (uint32_t)out[i - 1]);
    }
    printf("local T=%d n=%lu ranges=%lu (%lu each): %.3f ms (%.0f GB/s of 16 B/rec) bad=%lu\n", LT, (unsigned long)n,
           (unsigned long)nb, (unsigned long)bs, tot / K, n * 16.0 / (tot / K) / 1e6, (unsigned long)bad);
    return 0;
}
