// scan.hip -- device-wide exclusive prefix sum of uint32 (reduce-then-scan).
//
// Used for radix-sort digit offsets, group/probe compaction and bucket offsets.
// Tiles of 4096 values per 256-lane workgroup: coalesced 16-B loads into LDS,
// per-lane serial sums, a wave64 shuffle scan, then coalesced stores.
// Partial sums are scanned recursively, so any n < 2^32 works.
#include "mums_internal.h"

namespace mums {

namespace {

constexpr int kScanTile = 4096;
constexpr int kPer = kScanTile / kBlock;  // 16

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// block-wide exclusive scan of one value per thread; returns exclusive prefix, *total = sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    #pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
        uint32_t x = s_w[k];
        wpre += (k < wv) ? x : 0;
        tot += x;
    }
    *total = tot;
    __syncthreads();
    return wpre + inc - v;
}

__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const uint32_t* __restrict__ in, uint64_t n,
                                                             uint32_t* __restrict__ partials) {
    __shared__ uint32_t s_w[kBlock / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
    uint32_t sum = 0;
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        uint64_t i = t0 + threadIdx.x + (uint64_t)k * kBlock;
        if (i < n) sum += in[i];
    }
    uint32_t tot;
    (void)block_excl_scan(sum, s_w, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_down_kernel(uint32_t* __restrict__ data, uint64_t n,
                                                           const uint32_t* __restrict__ partials,
                                                           uint32_t* __restrict__ total_out, uint64_t nblocks) {
    __shared__ uint32_t tile[kScanTile + kScanTile / 32];
    __shared__ uint32_t s_w[kBlock / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
    // coalesced load (striped), padded LDS index to avoid bank conflicts on the blocked read
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        int j = threadIdx.x + k * kBlock;
        uint64_t i = t0 + j;
        tile[j + (j >> 5)] = i < n ? data[i] : 0;
    }
    __syncthreads();
    uint32_t v[kPer];
    uint32_t s = 0;
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        int j = threadIdx.x * kPer + k;
        v[k] = tile[j + (j >> 5)];
        s += v[k];
    }
    uint32_t tot;
    uint32_t pre = block_excl_scan(s, s_w, &tot) + partials[blockIdx.x];
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        int j = threadIdx.x * kPer + k;
        tile[j + (j >> 5)] = pre;
        pre += v[k];
    }
    __syncthreads();
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        int j = threadIdx.x + k * kBlock;
        uint64_t i = t0 + j;
        if (i < n) data[i] = tile[j + (j >> 5)];
    }
    if (total_out && blockIdx.x == nblocks - 1 && threadIdx.x == kBlock - 1) *total_out = pre;
}

// single-workgroup scan for <= kScanTile values
__global__ __launch_bounds__(kBlock) void scan_small_kernel(uint32_t* __restrict__ data, uint64_t n,
                                                            uint32_t* __restrict__ total_out) {
    __shared__ uint32_t s_w[kBlock / 64];
    uint32_t v[kPer];
    uint32_t s = 0;
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        uint64_t i = (uint64_t)threadIdx.x * kPer + k;
        v[k] = i < n ? data[i] : 0;
        s += v[k];
    }
    uint32_t tot;
    uint32_t pre = block_excl_scan(s, s_w, &tot);
    #pragma unroll
    for (int k = 0; k < kPer; ++k) {
        uint64_t i = (uint64_t)threadIdx.x * kPer + k;
        if (i < n) data[i] = pre;
        pre += v[k];
    }
    if (total_out && threadIdx.x == 0) *total_out = tot;
}

uint64_t nblk(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

}  // namespace

size_t scan_tmp_bytes(uint64_t n) {
    size_t b = 0;
    while (n > (uint64_t)kScanTile) {
        n = nblk(n);
        b += (n + 64) * sizeof(uint32_t);
    }
    return b + 256;
}

hipError_t exclusive_scan_u32(uint32_t* d_data, uint64_t n, void* d_tmp, uint32_t* d_total, hipStream_t st) {
    if (n == 0) {
        if (d_total) return hipMemsetAsync(d_total, 0, sizeof(uint32_t), st);
        return hipSuccess;
    }
    if (n <= (uint64_t)kScanTile) {
        hipLaunchKernelGGL(scan_small_kernel, dim3(1), dim3(kBlock), 0, st, d_data, n, d_total);
        return hipGetLastError();
    }
    const uint64_t nb = nblk(n);
    uint32_t* partials = (uint32_t*)d_tmp;
    void* rest = (void*)(partials + nb + 64);
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, d_data, n, partials);
    hipError_t e = exclusive_scan_u32(partials, nb, rest, nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(scan_down_kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, d_data, n, partials, d_total,
                       nb);
    return hipGetLastError();
}

}  // namespace mums
