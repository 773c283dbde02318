// msd_pass.hip -- one stable MSD partition pass of the packed seed records on a
// kBits-wide digit (kBits 8..10), inside every MSD bucket (row A5).
//
// After the seed scatter has split the records by the top B key bits, this pass
// splits every bucket again by the next kBits bits, so the resulting sub-buckets are
// small enough for the LDS-resident local sort (local_sort.hip).  Same onesweep
// machinery as radix_seg.hip (one histogram read, decoupled look-back between the
// consecutive tiles of a bucket, interleaved claim order), with D = 2^kBits digits:
// every thread owns D/256 consecutive digits of the scan and the look-back.
// HBM bytes per record: 8 (histogram read) + 8 + 8 (the pass).
#include "../../libmems_amd/csrc/mums_internal.h"

namespace mums {

namespace {

constexpr int kMTile = kSegTile;
constexpr int kMIPT = kMTile / kBlock;
constexpr int kMWaves = kBlock / 64;
constexpr uint32_t kMFlagAgg = 1u << 30;
constexpr uint32_t kMFlagInc = 2u << 30;
constexpr uint32_t kMValMask = (1u << 30) - 1;
constexpr int kMLookback = 4;
constexpr int kMHistTilesPerBlock = 16;

// per-bucket digit histogram: ghist[b * D + d]
template <int kBits>
__global__ __launch_bounds__(kBlock) void msd_hist_kernel(const uint64_t* __restrict__ rec,
                                                          const SegTile* __restrict__ tiles, uint64_t ntiles_ub,
                                                          int shift, uint32_t* __restrict__ ghist) {
    constexpr int D = 1 << kBits;
    __shared__ uint32_t h[D];
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * kMHistTilesPerBlock;
    uint32_t cur_b = 0xFFFFFFFFu;
    for (int i = tid; i < D; i += kBlock) h[i] = 0;
    __syncthreads();
    for (int k = 0; k < kMHistTilesPerBlock; ++k) {
        const uint64_t t = t0 + k;
        if (t >= ntiles_ub) break;
        const SegTile d = tiles[t];
        if (d.count == 0) break;
        if (d.bucket != cur_b) {
            if (cur_b != 0xFFFFFFFFu) {
                __syncthreads();
                for (int i = tid; i < D; i += kBlock) {
                    if (h[i]) atomicAdd(&ghist[(uint64_t)cur_b * D + i], h[i]);
                    h[i] = 0;
                }
                __syncthreads();
            }
            cur_b = d.bucket;
        }
        for (uint32_t q = tid; q < d.count; q += kBlock)
            atomicAdd(&h[(uint32_t)(rec[d.start + q] >> shift) & (D - 1)], 1u);
    }
    __syncthreads();
    if (cur_b != 0xFFFFFFFFu)
        for (int i = tid; i < D; i += kBlock)
            if (h[i]) atomicAdd(&ghist[(uint64_t)cur_b * D + i], h[i]);
}

// one block per bucket: dbase[b * D + d] = bstart[b] + exclusive scan over digits
template <int kBits>
__global__ __launch_bounds__(kBlock) void msd_dbase_kernel(const uint32_t* __restrict__ ghist,
                                                           const uint32_t* __restrict__ bstart,
                                                           uint32_t* __restrict__ dbase) {
    constexpr int D = 1 << kBits, PER = D / kBlock;
    __shared__ uint32_t s_w[kMWaves];
    const uint64_t b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t v[PER], sum = 0;
    #pragma unroll
    for (int k = 0; k < PER; ++k) { v[k] = ghist[b * D + tid * PER + k]; sum += v[k]; }
    uint32_t inc = sum;
    #pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t x = __shfl_up(inc, dd, 64);
        if (lane >= dd) inc += x;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = bstart[b] + inc - sum;
    #pragma unroll
    for (int w = 0; w < kMWaves; ++w) pre += (w < wv) ? s_w[w] : 0u;
    #pragma unroll
    for (int k = 0; k < PER; ++k) { dbase[b * D + tid * PER + k] = pre; pre += v[k]; }
}

template <int kBits>
__global__ __launch_bounds__(kBlock) void msd_onesweep_kernel(const uint64_t* __restrict__ rin,
                                                              uint64_t* __restrict__ rout,
                                                              const SegTile* __restrict__ tiles, uint32_t nclaims,
                                                              int shift, const uint32_t* __restrict__ dbase,
                                                              uint32_t* status, uint32_t* tile_counter,
                                                              uint32_t* err) {
    constexpr int D = 1 << kBits, PER = D / kBlock;
    __shared__ uint64_t srec[kMTile];
    __shared__ uint32_t wcnt[kMWaves][D];
    __shared__ uint32_t lstart[D];
    __shared__ uint32_t gofs[D];
    __shared__ uint32_t hcnt[D];
    __shared__ uint32_t s_w[kMWaves];
    __shared__ uint32_t s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    for (int i = tid; i < kMWaves * D; i += kBlock) (&wcnt[0][0])[i] = 0;
    for (int i = tid; i < D; i += kBlock) hcnt[i] = 0;
    __syncthreads();
    const uint32_t c = __builtin_amdgcn_readfirstlane(s_tile);
    if (c >= nclaims) return;
    const uint32_t t = __builtin_amdgcn_readfirstlane(tiles[c].order);
    const SegTile d = tiles[t];
    if (d.count == 0) return;
    const uint32_t q0 = wv * (kMTile / kMWaves);
    uint64_t key[kMIPT];
    uint32_t rank[kMIPT];
    #pragma unroll
    for (int r = 0; r < kMIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
    }
    #pragma unroll
    for (int r = 0; r < kMIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        if (q < d.count) atomicAdd(&hcnt[(uint32_t)(key[r] >> shift) & (D - 1)], 1u);
    }
    __syncthreads();
    if (d.tb != 0)
        for (int i = tid; i < D; i += kBlock)
            __hip_atomic_store(status + (uint64_t)t * D + i, kMFlagAgg | hcnt[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    #pragma unroll
    for (int r = 0; r < kMIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        const bool valid = q < d.count;
        const uint32_t dg = (uint32_t)(key[r] >> shift) & (D - 1);
        uint32_t tot;
        const uint32_t rk = wave_match_rank<kBits>(dg, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][dg];
        if (valid && rk == 0) wcnt[wv][dg] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();
    // this thread's digits [tid * PER, tid * PER + PER): wave offsets, look-back, totals
    uint32_t acc[PER], tsum = 0;
    #pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int dg = tid * PER + k;
        uint32_t a = 0;
        #pragma unroll
        for (int w = 0; w < kMWaves; ++w) { const uint32_t x = wcnt[w][dg]; wcnt[w][dg] = a; a += x; }
        acc[k] = a;
        tsum += a;
    }
    const int64_t tfirst = (int64_t)t - (int64_t)d.tb;
    #pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int dg = tid * PER + k;
        uint32_t* st = status + (uint64_t)t * D + dg;
        uint32_t prefix = 0;
        if (d.tb == 0) {
            __hip_atomic_store(st, kMFlagInc | acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int64_t j = (int64_t)t - 1;
            uint32_t spins = 0;
            bool done = false;
            while (!done) {
                uint32_t sv[kMLookback];
                #pragma unroll
                for (int m = 0; m < kMLookback; ++m)
                    sv[m] = (j - m >= tfirst) ? __hip_atomic_load(status + (uint64_t)(j - m) * D + dg,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : kMFlagInc;
                int used = 0;
                bool stall = false;
                #pragma unroll
                for (int m = 0; m < kMLookback; ++m) {
                    if (done || stall) continue;
                    const uint32_t sx = sv[m];
                    if ((sx >> 30) == 0u) { stall = true; continue; }
                    prefix += sx & kMValMask;
                    ++used;
                    if ((sx & kMFlagInc) != 0u) done = true;
                }
                j -= used;
                if (stall && !done) {
                    if (++spins > (1u << 24)) { atomicOr(err, 2u); break; }
                    if (spins < 8) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(8);
                }
            }
            __hip_atomic_store(st, kMFlagInc | ((prefix + acc[k]) & kMValMask), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        gofs[dg] = dbase[(uint64_t)d.bucket * D + dg] + prefix;
    }
    // block-local digit starts: exclusive scan of the per-thread digit totals
    uint32_t v = tsum;
    #pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t x = __shfl_up(v, dd, 64);
        if (lane >= dd) v += x;
    }
    if (lane == 63) s_w[wv] = v;
    __syncthreads();
    uint32_t pre = v - tsum;
    #pragma unroll
    for (int w = 0; w < kMWaves; ++w) pre += (w < wv) ? s_w[w] : 0u;
    #pragma unroll
    for (int k = 0; k < PER; ++k) { lstart[tid * PER + k] = pre; pre += acc[k]; }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kMIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        if (q < d.count) {
            const uint32_t dg = (uint32_t)(key[r] >> shift) & (D - 1);
            srec[lstart[dg] + wcnt[wv][dg] + rank[r]] = key[r];
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kMIPT; ++r) {
        const uint32_t sidx = tid + r * kBlock;
        if (sidx < d.count) {
            const uint64_t k = srec[sidx];
            const uint32_t dg = (uint32_t)(k >> shift) & (D - 1);
            rout[(uint64_t)gofs[dg] + (sidx - lstart[dg])] = k;
        }
    }
}

template <int kBits>
hipError_t msd_pass_impl(const uint64_t* rin, uint64_t* rout, uint64_t n, int shift, int msd_bits,
                         const SegTile* d_tiles, uint64_t ntiles_ub, const uint32_t* d_bstart, void* d_tmp,
                         uint32_t* d_err, uint32_t* d_dbase_out, hipStream_t st) {
    constexpr int D = 1 << kBits;
    const uint64_t nb = 1ull << msd_bits;
    uint32_t* status = (uint32_t*)d_tmp;             // [ub][D]
    uint32_t* ghist = status + ntiles_ub * D;        // [nb][D]
    uint32_t* counter = ghist + nb * D;
    hipError_t e = hipMemsetAsync(status, 0, ((uint64_t)(counter - status) + 64) * 4, st);
    if (e != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    const unsigned hb = (unsigned)((ntiles_ub + kMHistTilesPerBlock - 1) / kMHistTilesPerBlock);
    hipLaunchKernelGGL(msd_hist_kernel<kBits>, dim3(hb), dim3(kBlock), 0, st, rin, d_tiles, ntiles_ub, shift, ghist);
    hipLaunchKernelGGL(msd_dbase_kernel<kBits>, dim3((unsigned)nb), dim3(kBlock), 0, st, ghist, d_bstart, d_dbase_out);
    hipLaunchKernelGGL(msd_onesweep_kernel<kBits>, dim3((unsigned)ntiles_ub), dim3(kBlock), 0, st, rin, rout, d_tiles,
                       (uint32_t)ntiles_ub, shift, d_dbase_out, status, counter, d_err);
    return hipGetLastError();
}

}  // namespace

size_t msd_pass_tmp_bytes(uint64_t n, int msd_bits, int digit_bits) {
    const uint64_t ub = seg_tiles_upper(n, msd_bits);
    return (ub + (1ull << msd_bits)) * (1ull << digit_bits) * 4 + 1024;
}

hipError_t msd_pass(const uint64_t* rin, uint64_t* rout, uint64_t n, int shift, int msd_bits, int digit_bits,
                    const SegTile* d_tiles, uint64_t ntiles_ub, const uint32_t* d_bstart, void* d_tmp,
                    uint32_t* d_err, uint32_t* d_dbase_out, hipStream_t st) {
    switch (digit_bits) {
        case 8: return msd_pass_impl<8>(rin, rout, n, shift, msd_bits, d_tiles, ntiles_ub, d_bstart, d_tmp, d_err,
                                        d_dbase_out, st);
        case 9: return msd_pass_impl<9>(rin, rout, n, shift, msd_bits, d_tiles, ntiles_ub, d_bstart, d_tmp, d_err,
                                        d_dbase_out, st);
        case 10: return msd_pass_impl<10>(rin, rout, n, shift, msd_bits, d_tiles, ntiles_ub, d_bstart, d_tmp, d_err,
                                          d_dbase_out, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mums
