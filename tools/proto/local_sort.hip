// local_sort.hip -- LDS-resident stable radix sort of small record ranges (row A5).
//
// After the MSD splits (seed scatter + one onesweep pass) every sub-bucket of the
// packed-record stream holds a few thousand records.  One 1024-lane workgroup
// loads a range of <= kLocalCap records once, runs all remaining 8-bit LSD passes
// through LDS (wave64 ballot match-any ranking, per-wave digit counters), and
// writes the sorted range once: 16 HBM bytes per record for the whole tail of the
// sort instead of 16 per pass.
#include "../../libmems_amd/csrc/mums_internal.h"

namespace mums {

namespace {

constexpr int kLDigits = 256;

}  // namespace

// Sorts ranges[u] = [start, start + count) of rin into rout (same positions) by key
// bits [32, 32 + key_bits) of each record, stable.  count <= kLThreads * kLocalIPT.
template <int kLThreads>
__global__ __launch_bounds__(kLThreads) void local_sort_kernel(const uint64_t* __restrict__ rin,
                                                               uint64_t* __restrict__ rout,
                                                               const uint64_t* __restrict__ ranges, uint32_t nranges,
                                                               int key_bits) {
    constexpr int kLWaves = kLThreads / 64;
    __shared__ uint64_t srec[kLThreads * kLocalIPT];
    __shared__ uint32_t wcnt[kLWaves][kLDigits];
    __shared__ uint32_t lstart[kLDigits];
    __shared__ uint32_t s_w[4];
    const uint32_t u = blockIdx.x;
    if (u >= nranges) return;
    const uint64_t rg = ranges[u];
    const uint64_t start = rg & ((1ull << 40) - 1);
    const uint32_t n = (uint32_t)(rg >> 40);
    if (n == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // blocked assignment: wave wv owns positions [wv * chunk, (wv + 1) * chunk)
    const uint32_t chunk = ((n + kLWaves * 64 - 1) / (kLWaves * 64)) * 64;
    const uint32_t q0 = wv * chunk;
    const uint32_t nr = chunk / 64;
    uint64_t key[kLocalIPT];
    uint32_t rank[kLocalIPT];
    #pragma unroll
    for (int r = 0; r < kLocalIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        key[r] = (r < (int)nr && q < n) ? rin[start + q] : 0ull;
    }
    const int npass = (key_bits + 7) / 8;
    for (int p = 0; p < npass; ++p) {
        const int shift = 32 + 8 * p;
        for (int i = tid; i < kLWaves * kLDigits; i += kLThreads) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kLocalIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            const bool valid = r < (int)nr && q < n;
            const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
            uint32_t tot;
            const uint32_t rk = wave_match_rank<8>(dg, valid, &tot);
            uint32_t old = 0;
            if (valid) old = wcnt[wv][dg];
            if (valid && rk == 0) wcnt[wv][dg] = old + tot;
            rank[r] = old + rk;
        }
        __syncthreads();
        if (tid < kLDigits) {
            const int dg = tid;
            uint32_t acc = 0;
            #pragma unroll
            for (int w = 0; w < kLWaves; ++w) { const uint32_t c = wcnt[w][dg]; wcnt[w][dg] = acc; acc += c; }
            uint32_t v = acc;
            #pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t x = __shfl_up(v, dd, 64);
                if (lane >= dd) v += x;
            }
            if (lane == 63) s_w[wv] = v;
            lstart[dg] = v - acc;   // wave-local exclusive; wave offsets added below
        }
        __syncthreads();
        if (tid < kLDigits) {
            uint32_t pre = 0;
            #pragma unroll
            for (int w = 0; w < kLDigits / 64; ++w) pre += (w < wv) ? s_w[w] : 0u;
            lstart[tid] += pre;
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kLocalIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            if (r < (int)nr && q < n) {
                const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
                srec[lstart[dg] + wcnt[wv][dg] + rank[r]] = key[r];
            }
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kLocalIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            if (r < (int)nr && q < n) key[r] = srec[q];
        }
    }
    #pragma unroll
    for (int r = 0; r < kLocalIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        if (r < (int)nr && q < n) rout[start + q] = key[r];
    }
}

}  // namespace mums
