// Development probe: ncclAllGather of uint64 on one rank (system librccl), result check.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <vector>
int main() {
    int dev = 0;
    ncclComm_t c;
    if (ncclCommInitAll(&c, 1, &dev) != ncclSuccess) { printf("init failed\n"); return 1; }
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const size_t n = 40000;
    std::vector<uint64_t> h(n), r(n);
    for (size_t i = 0; i < n; ++i) h[i] = i * 7 + 3;
    uint64_t* d;
    hipMalloc(&d, 2 * n * 8 + 64);
    hipMemcpyAsync(d + n, h.data(), n * 8, hipMemcpyHostToDevice, st);
    ncclResult_t e = ncclAllGather(d + n, d, n, ncclUint64, c, st);
    hipMemcpyAsync(r.data(), d, n * 8, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += r[i] != h[i];
    printf("allgather rc %d bad %zu of %zu (r[0]=%lu r[1]=%lu)\n", (int)e, bad, n, (unsigned long)r[0], (unsigned long)r[1]);
    ncclCommDestroy(c);
    return 0;
}
