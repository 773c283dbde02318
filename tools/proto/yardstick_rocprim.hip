// Yardstick only (not used by the product): rocPRIM/hipCUB radix sort of N uint64 records
// on the same 32 key bits our segmented sort handles, to calibrate what 4 x 8-bit LSD
// passes can reach on this MI355X.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

int main(int argc, char** argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 800000000ull;
    std::vector<uint64_t> h(n);
    std::mt19937_64 r(1);
    for (size_t i = 0; i < n; ++i) h[i] = (r() & 0xFFFFFFFF00000000ull) | i;
    uint64_t *a, *b;
    hipMalloc(&a, n * 8); hipMalloc(&b, n * 8);
    hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
    size_t tb = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, tb, a, b, (int)n, 32, 64);
    void* tmp; hipMalloc(&tmp, tb);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int it = 0; it < 2; ++it) hipcub::DeviceRadixSort::SortKeys(tmp, tb, a, b, (int)n, 32, 64);
    hipEventRecord(e0);
    const int K = 5;
    for (int it = 0; it < K; ++it) hipcub::DeviceRadixSort::SortKeys(tmp, tb, a, b, (int)n, 32, 64);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    ms /= K;
    printf("hipcub SortKeys u64 n=%zu bits[32,64): %.3f ms, %.2f GB/s (4 passes x 16 B)\n", n, ms, n * 64.0 / ms / 1e6);
    // also a plain copy for the achievable stream bandwidth
    hipEventRecord(e0);
    for (int it = 0; it < K; ++it) hipMemcpyAsync(b, a, n * 8, hipMemcpyDeviceToDevice);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1); ms /= K;
    printf("memcpy %zu B: %.3f ms, %.2f GB/s (read+write)\n", n * 8, ms, n * 16.0 / ms / 1e6);
    return 0;
}
