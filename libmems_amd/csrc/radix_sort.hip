// radix_sort.hip -- stable LSD radix sort of (key, uint32 value) pairs for gfx950 (row A5).
//
// Replaces MemorySML::Create's std::sort of 16-B bmer records (MemorySML.cpp:54,
// bmer_lessthan SortedMerList.h:311-314) and, because every genome's keys are
// sorted together with the genome in the value, also the G-way list merge of
// MatchFinder::SearchRange (MatchFinder.cpp:236-333).
//
// Per 8-bit digit pass, three launches (reduce-then-scan):
//   upsweep   : per-4096-key tile digit histogram (wave-private LDS counters)
//   scan      : exclusive scan of the digit-major [256 x tiles] histogram
//   downsweep : stable in-tile ranking with wave64 ballot "match-any" over the
//               8 digit bits + per-wave LDS digit counters, reorder through LDS,
//               then digit-run-contiguous global stores.
// HBM bytes per key per pass: upsweep K, downsweep 2(K+V)  (first pass: values
// are the implicit indices and are not read).
#include <cstdlib>
#include "mums_internal.h"

namespace mums {

namespace {

constexpr int kRTile = 4096;
constexpr int kRounds = kRTile / kBlock;  // 16 rounds of 64 per wave (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kDigits = 256;

template <typename K>
__global__ __launch_bounds__(kBlock) void rs_upsweep(const K* __restrict__ keys, uint64_t n, int shift,
                                                     uint32_t* __restrict__ hist, uint32_t nblocks, int agg) {
    __shared__ uint32_t h[kWaves][kDigits];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * kDigits; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * kRTile + (uint64_t)wv * (kRTile / kWaves);
    if (agg) {   // uniform: one LDS add per distinct digit of the wave (keys with a hot digit,
                 // e.g. the probes' hash buckets of related genomes, serialise per-key atomics)
        #pragma unroll 4
        for (int r = 0; r < kRounds; ++r) {
            const uint64_t i = b0 + (uint64_t)r * 64 + lane;
            const bool valid = i < n;
            const uint32_t d = valid ? (uint32_t)(keys[i] >> shift) & 0xFFu : 0u;
            uint32_t tot;
            const uint32_t rk = wave_match_rank<8>(d, valid, &tot);
            if (valid && rk == 0) atomicAdd(&h[wv][d], tot);
        }
    } else {
        #pragma unroll 4
        for (int r = 0; r < kRounds; ++r) {
            uint64_t i = b0 + (uint64_t)r * 64 + lane;
            if (i < n) {
                uint32_t d = (uint32_t)(keys[i] >> shift) & 0xFFu;
                atomicAdd(&h[wv][d], 1u);
            }
        }
    }
    __syncthreads();
    const int t = threadIdx.x;
    uint32_t s = 0;
    #pragma unroll
    for (int w = 0; w < kWaves; ++w) s += h[w][t];
    hist[(uint64_t)t * nblocks + blockIdx.x] = s;
}

template <typename K, bool kImplicitVals>
__global__ __launch_bounds__(kBlock) void rs_downsweep(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                       uint64_t n, int shift, const uint32_t* __restrict__ hist,
                                                       uint32_t nblocks, K* __restrict__ kout,
                                                       uint32_t* __restrict__ vout) {
    __shared__ K skeys[kRTile];
    __shared__ uint32_t svals[kRTile];
    __shared__ uint32_t wcnt[kWaves][kDigits];
    __shared__ uint32_t lstart[kDigits];
    __shared__ uint32_t gofs[kDigits];
    __shared__ uint32_t s_w[kWaves];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * kDigits; i += kBlock) (&wcnt[0][0])[i] = 0;
    __syncthreads();

    const uint64_t tile0 = (uint64_t)blockIdx.x * kRTile;
    const uint64_t b0 = tile0 + (uint64_t)wv * (kRTile / kWaves);
    K key[kRounds];
    uint32_t val[kRounds];
    uint32_t rank[kRounds];
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t i = b0 + (uint64_t)r * 64 + lane;
        const bool valid = i < n;
        key[r] = valid ? kin[i] : (K)0;
        val[r] = kImplicitVals ? (uint32_t)i : (valid ? vin[i] : 0u);
        const uint32_t d = (uint32_t)(key[r] >> shift) & 0xFFu;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<8>(d, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][d];
        if (valid && rk == 0) wcnt[wv][d] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();

    // per-digit wave offsets and block-local digit starts
    {
        const int t = threadIdx.x;  // digit
        uint32_t acc = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            uint32_t c = wcnt[w][t];
            wcnt[w][t] = acc;
            acc += c;
        }
        // block exclusive scan of acc over digits
        uint32_t v = acc;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t x = __shfl_up(v, d, 64);
            if (lane >= d) v += x;
        }
        if (lane == 63) s_w[wv] = v;
        __syncthreads();
        uint32_t wpre = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) wpre += (w < wv) ? s_w[w] : 0u;
        lstart[t] = wpre + v - acc;
        gofs[t] = hist[(uint64_t)t * nblocks + blockIdx.x];
    }
    __syncthreads();

    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t i = b0 + (uint64_t)r * 64 + lane;
        if (i < n) {
            const uint32_t d = (uint32_t)(key[r] >> shift) & 0xFFu;
            const uint32_t lp = lstart[d] + wcnt[wv][d] + rank[r];
            skeys[lp] = key[r];
            svals[lp] = val[r];
        }
    }
    __syncthreads();

    const uint64_t cnt = (n - tile0) < (uint64_t)kRTile ? (n - tile0) : (uint64_t)kRTile;
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t s = threadIdx.x + r * kBlock;
        if (s < cnt) {
            const K k = skeys[s];
            const uint32_t d = (uint32_t)(k >> shift) & 0xFFu;
            const uint64_t o = (uint64_t)gofs[d] + (s - lstart[d]);
            kout[o] = k;
            vout[o] = svals[s];
        }
    }
}

uint64_t tiles(uint64_t n) { return (n + kRTile - 1) / kRTile; }

}  // namespace

size_t radix_tmp_bytes(uint64_t n) {
    uint64_t h = (uint64_t)kDigits * tiles(n);
    return (h + 64) * sizeof(uint32_t) + scan_tmp_bytes(h) + 256;
}

template <typename K>
hipError_t radix_sort(const K* keys_in, const uint32_t* vals_in, uint64_t n, int bits, K* kA, uint32_t* vA,
                      K* kB, uint32_t* vB, void* d_tmp, int* out_buf, hipStream_t st, hipEvent_t* ev_ds) {
    const int passes = (bits + 7) / 8;
    *out_buf = (passes - 1) % 2;
    if (n == 0 || passes == 0) return hipSuccess;
    const uint32_t nb = (uint32_t)tiles(n);
    uint32_t* hist = (uint32_t*)d_tmp;
    void* stmp = (void*)(hist + (uint64_t)kDigits * nb + 64);
    const K* ksrc = keys_in;
    const uint32_t* vsrc = vals_in;
    for (int p = 0; p < passes; ++p) {
        K* kdst = (p % 2 == 0) ? kA : kB;
        uint32_t* vdst = (p % 2 == 0) ? vA : vB;
        const int shift = 8 * p;
        const bool agg = !getenv("MUMS_DEV_RS_NOAGG");   // A/B round 4: bucket sort 1.56 -> 1.34 ms
        hipLaunchKernelGGL(rs_upsweep<K>, dim3(nb), dim3(kBlock), 0, st, ksrc, n, shift, hist, nb, agg ? 1 : 0);
        hipError_t e = exclusive_scan_u32(hist, (uint64_t)kDigits * nb, stmp, nullptr, st);
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p], st);
        if (vsrc == nullptr)
            hipLaunchKernelGGL((rs_downsweep<K, true>), dim3(nb), dim3(kBlock), 0, st, ksrc, vsrc, n, shift, hist,
                               nb, kdst, vdst);
        else
            hipLaunchKernelGGL((rs_downsweep<K, false>), dim3(nb), dim3(kBlock), 0, st, ksrc, vsrc, n, shift, hist,
                               nb, kdst, vdst);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p + 1], st);
        ksrc = kdst;
        vsrc = vdst;
    }
    return hipSuccess;
}

template hipError_t radix_sort<uint32_t>(const uint32_t*, const uint32_t*, uint64_t, int, uint32_t*, uint32_t*,
                                         uint32_t*, uint32_t*, void*, int*, hipStream_t, hipEvent_t*);
template hipError_t radix_sort<uint64_t>(const uint64_t*, const uint32_t*, uint64_t, int, uint64_t*, uint32_t*,
                                         uint64_t*, uint32_t*, void*, int*, hipStream_t, hipEvent_t*);

}  // namespace mums
