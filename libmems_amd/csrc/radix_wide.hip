// radix_wide.hip -- three-pass variant of the segmented onesweep sort (row A5,
// MemorySML::Create's std::sort, MemorySML.cpp:45-60, over all genomes at once).
//
// Under the default tolerances a masked-key group's probe does not depend on the order of
// its records (MemHash.cpp:139-203 reads only the group's genome set and first starts), so
// key bit 0 -- the parity / orientation bit -- need not be sorted: records of one masked key
// stay in index order and seg_parity_fix (radix_seg.hip) restores the exact SML order
// before a MER_REPEAT_LIMIT restart.  With the 8-bit MSD scatter a w19 record holds 31 key
// bits (key_low << 32 | index, 2w+1 = 39 = 8 + 31); leaving the parity bit out leaves 30
// bits: three 10-bit onesweep passes instead of four 8-bit ones (12.8 GB of record traffic
// per pass at BASELINE config 3).
//
// One pass = one launch: each block claims a tile (atomic counter, claim order of
// claim_order_kernel), ranks its records on the 10-bit digit (wave64 match-any, per-wave
// counts aliased into the exchange buffer), publishes its per-digit counts, looks back over
// the preceding tiles of its MSD bucket, reorders the tile in LDS and stores digit runs.
// A 1024-digit tile needs more digit state than the 256-digit one: each digit-owning
// thread owns 1024 / min(OB, 1024) consecutive digits, keeps their output offsets in
// registers and folds them into ONE LDS array after the reorder offsets are taken, so the
// 9216-record tile still fits two blocks per CU.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "mums_internal.h"

namespace mums {

namespace {

constexpr uint32_t kWFlagAgg = 1u << 30;
constexpr uint32_t kWFlagInc = 2u << 30;
constexpr uint32_t kWValMask = (1u << 30) - 1;
constexpr int kWLookback = 4;
constexpr int kWHistTiles = 16;   // tiles per histogram block

// all passes' per-bucket digit histograms in one read: ghist[(b * npass + p) * kD + d]
template <int DB>
__global__ __launch_bounds__(kBlock) void wide_ghist_kernel(const uint64_t* __restrict__ rec,
                                                            const SegTile* __restrict__ tiles, uint64_t ntiles_ub,
                                                            int npass, int shift0, uint32_t* __restrict__ ghist) {
    constexpr int kD = 1 << DB;
    constexpr uint32_t kM = kD - 1;
    __shared__ uint32_t h[3][kD];
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * kWHistTiles;
    uint32_t cur_b = 0xFFFFFFFFu;
    for (int i = tid; i < 3 * kD; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    auto flush = [&](uint32_t b) {
        for (int p = 0; p < npass; ++p)
            for (int dg = tid; dg < kD; dg += kBlock) {
                const uint32_t v = h[p][dg];
                if (v) atomicAdd(&ghist[((uint64_t)b * npass + p) * kD + dg], v);
                h[p][dg] = 0;
            }
    };
    for (int k = 0; k < kWHistTiles; ++k) {
        const uint64_t t = t0 + k;
        if (t >= ntiles_ub) break;
        const SegTile d = tiles[t];
        if (d.count == 0) break;
        if (d.bucket != cur_b) {   // uniform
            if (cur_b != 0xFFFFFFFFu) {
                __syncthreads();
                flush(cur_b);
                __syncthreads();
            }
            cur_b = d.bucket;
        }
        constexpr int kB = 8;   // records per lane in flight
        for (uint32_t q0 = 0; q0 < d.count; q0 += kBlock * kB) {
            uint64_t kk[kB];
            #pragma unroll
            for (int u = 0; u < kB; ++u) {
                const uint32_t q = q0 + u * kBlock + tid;
                kk[u] = q < d.count ? rec[d.start + q] : 0ull;
            }
            #pragma unroll
            for (int u = 0; u < kB; ++u) {
                if (q0 + u * kBlock + tid >= d.count) break;
                const uint64_t key = kk[u] >> shift0;
                for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(uint32_t)(key >> (DB * p)) & kM], 1u);
            }
        }
    }
    __syncthreads();
    if (cur_b != 0xFFFFFFFFu) flush(cur_b);
}

// one block per (bucket, pass): dbase = bucket start + exclusive scan over the kD digits
template <int DB>
__global__ __launch_bounds__(kBlock) void wide_dbase_kernel(const uint32_t* __restrict__ ghist,
                                                            const uint32_t* __restrict__ bstart, int npass,
                                                            uint32_t* __restrict__ dbase) {
    constexpr int kD = 1 << DB;
    constexpr int kPer = kD / kBlock;
    __shared__ uint32_t s_w[kBlock / 64];
    const uint64_t bp = blockIdx.x;
    const uint32_t b = (uint32_t)(bp / npass);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t v[kPer], sum = 0;
    #pragma unroll
    for (int i = 0; i < kPer; ++i) {
        v[i] = ghist[bp * kD + tid * kPer + i];
        sum += v[i];
    }
    uint32_t inc = sum;
    #pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t x = __shfl_up(inc, dd, 64);
        if (lane >= dd) inc += x;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
    #pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) pre += (w < wv) ? s_w[w] : 0u;
    uint32_t o = bstart[b] + pre + inc - sum;
    #pragma unroll
    for (int i = 0; i < kPer; ++i) {
        dbase[bp * kD + tid * kPer + i] = o;
        o += v[i];
    }
}

// two blocks per CU (OB <= 768): at least 2 * OB / 256 waves per SIMD, i.e. <= 80 VGPRs at 768
template <int OB, int kIPT, int DB>
__global__ __launch_bounds__(OB, (OB <= 768 ? 2 * OB / 256 : OB / 256)) void wide_onesweep_kernel(const uint64_t* __restrict__ rin,
                                                           uint64_t* __restrict__ rout,
                                                           const SegTile* __restrict__ tiles, uint32_t nclaims,
                                                           int shift, int pass, int npass,
                                                           const uint32_t* __restrict__ dbase, uint32_t* status,
                                                           uint32_t* tile_counter, uint32_t* err) {
    constexpr int kD = 1 << DB;
    constexpr uint32_t kM = kD - 1;
    constexpr int kT = kIPT * OB;
    constexpr int kW = OB / 64;
    constexpr int kNT = kD <= OB ? kD : (OB >= 512 ? 512 : 256);   // digit-owning threads (whole waves)
    constexpr int kDPT = kD / kNT;           // consecutive digits per owning thread
    static_assert(kD % kNT == 0 && kNT % 64 == 0, "digit owners are whole waves");
    static_assert(kW * kD * 4 <= kT * 8, "per-wave counts alias the exchange buffer");
    __shared__ uint64_t srec[kT];
    uint32_t (*wcnt)[kD] = reinterpret_cast<uint32_t (*)[kD]>(srec);
    __shared__ uint32_t lstart[kD];   // tile-local digit starts, then (output offset - tile start) per digit
    __shared__ uint32_t s_w[kW];
    __shared__ uint32_t s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    for (int i = tid; i < kW * kD; i += OB) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t c = __builtin_amdgcn_readfirstlane(s_tile);
    if (c >= nclaims) return;
    const uint32_t t = __builtin_amdgcn_readfirstlane(tiles[c].order);
    const SegTile d = tiles[t];
    if (d.count == 0) return;
    const uint32_t q0 = wv * (kT / kW);
    uint64_t key[kIPT];
    uint32_t rank[kIPT];
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t q = q0 + (uint32_t)r * 64u + (uint32_t)lane;
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
    }
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const bool valid = q0 + (uint32_t)r * 64u + (uint32_t)lane < d.count;
        const uint32_t dg = (uint32_t)(key[r] >> shift) & kM;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<DB>(dg, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][dg];
        if (valid && rk == 0) wcnt[wv][dg] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();
    uint32_t acc[kDPT], gof[kDPT];
    uint32_t tsum = 0, v = 0;
    if (tid < kNT) {
        #pragma unroll
        for (int i = 0; i < kDPT; ++i) {
            const int dg = tid * kDPT + i;
            uint32_t a = 0;
            #pragma unroll
            for (int w = 0; w < kW; ++w) { const uint32_t x = wcnt[w][dg]; wcnt[w][dg] = a; a += x; }
            acc[i] = a;
            tsum += a;
            __hip_atomic_store(status + (uint64_t)t * kD + dg, (d.tb == 0 ? kWFlagInc : kWFlagAgg) | a,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const int64_t tfirst = (int64_t)t - (int64_t)d.tb;
        #pragma unroll
        for (int i = 0; i < kDPT; ++i) {
            const int dg = tid * kDPT + i;
            uint32_t prefix = 0;
            if (d.tb != 0) {   // windowed look-back over the bucket's preceding tiles
                int64_t j = (int64_t)t - 1;
                uint32_t spins = 0;
                bool done = false;
                while (!done) {
                    uint32_t sv[kWLookback];
                    #pragma unroll
                    for (int k = 0; k < kWLookback; ++k)
                        sv[k] = (j - k >= tfirst) ? __hip_atomic_load(status + (uint64_t)(j - k) * kD + dg,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : kWFlagInc;
                    int used = 0;
                    bool stall = false;
                    #pragma unroll
                    for (int k = 0; k < kWLookback; ++k) {
                        if (done || stall) continue;
                        const uint32_t sx = sv[k];
                        if ((sx >> 30) == 0u) { stall = true; continue; }
                        prefix += sx & kWValMask;
                        ++used;
                        if ((sx & kWFlagInc) != 0u) done = true;
                    }
                    j -= used;
                    if (stall && !done) {
                        if (++spins > (1u << 24)) { atomicOr(err, 2u); break; }
                        if (spins < 8) __builtin_amdgcn_s_sleep(1);
                        else __builtin_amdgcn_s_sleep(8);
                    }
                }
                __hip_atomic_store(status + (uint64_t)t * kD + dg, kWFlagInc | ((prefix + acc[i]) & kWValMask),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            gof[i] = dbase[((uint64_t)d.bucket * npass + pass) * kD + dg] + prefix;
        }
        v = tsum;   // block-exclusive scan of the owners' digit sums
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t x = __shfl_up(v, dd, 64);
            if (lane >= dd) v += x;
        }
        if (lane == 63) s_w[wv] = v;
    }
    __syncthreads();
    if (tid < kNT) {
        uint32_t base = v - tsum;
        #pragma unroll
        for (int w = 0; w < kNT / 64; ++w) base += (w < wv) ? s_w[w] : 0u;
        #pragma unroll
        for (int i = 0; i < kDPT; ++i) {
            lstart[tid * kDPT + i] = base;
            base += acc[i];
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {   // slots first: the exchange overwrites the counts
        const uint32_t dg = (uint32_t)(key[r] >> shift) & kM;
        rank[r] += lstart[dg] + wcnt[wv][dg];
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kIPT; ++r)
        if (q0 + (uint32_t)r * 64u + (uint32_t)lane < d.count) srec[rank[r]] = key[r];
    if (tid < kNT) {   // own digits only: lstart becomes (output offset - tile slot), mod 2^32
        #pragma unroll
        for (int i = 0; i < kDPT; ++i) lstart[tid * kDPT + i] = gof[i] - lstart[tid * kDPT + i];
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t sidx = tid + r * OB;
        if (sidx < d.count) {
            const uint64_t k = srec[sidx];
            const uint32_t dg = (uint32_t)(k >> shift) & kM;
            rout[(uint64_t)(uint32_t)(lstart[dg] + sidx)] = k;
        }
    }
}

// block shapes (MUMS_DEV_SORT3, read per call): 1 = <768, 12> (9216-record tiles, two
// blocks per CU), 2 = <512, 16> (8192), 3 = <1024, 16> (16384, one block per CU)
int wide_variant() {
    const char* e = getenv("MUMS_DEV_SORT3");
    if (!e) return 1;
    const int v = atoi(e);
    return v >= 1 && v <= 3 ? v : 1;
}
uint32_t wide_tile(int v) { return v == 2 ? 8192u : v == 3 ? 16384u : 9216u; }

}  // namespace

bool seg_wide_sort_enabled() {
    const char* e = getenv("MUMS_DEV_SORT3");
    return e && atoi(e) > 0;
}

int seg_wide_passes(int key_bits) { return (key_bits - 1 + 9) / 10; }

size_t onesweep_wide_tmp_bytes(uint64_t n, int msd_bits, int key_bits) {
    constexpr uint64_t kD = 1024;
    const uint64_t ub = seg_tiles_upper(n, msd_bits, 8192);
    const uint64_t npass = (uint64_t)seg_wide_passes(key_bits);
    const uint64_t nb = 1ull << msd_bits;
    return (ub * kD * npass + 2 * nb * npass * kD + 128) * 4 + 2 * (ub * sizeof(SegTile) + 256) +
           (nb + 128) * 4 + scan_tmp_bytes(nb + 1) + 8192;
}

// the stream sorted by key bits [1, key_bits) of the record's key part (bits key_shift ..):
// equal masked keys keep index order (parity bit unsorted; seg_parity_fix restores it)
hipError_t seg_onesweep_sort_wide(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, int msd_bits,
                                  const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, int* out_buf,
                                  hipStream_t st, hipEvent_t* ev_ds, int key_shift) {
    constexpr int DB = 10;
    constexpr uint64_t kD = 1u << DB;
    const int npass = seg_wide_passes(key_bits);
    *out_buf = npass % 2;
    if (n == 0 || npass == 0) return hipSuccess;
    if (npass > 3) return hipErrorInvalidValue;
    const int var = wide_variant();
    const uint32_t tile = wide_tile(var);
    const uint64_t nb = 1ull << msd_bits;
    const uint64_t ub = seg_tiles_upper(n, msd_bits, tile);
    uint32_t* status = (uint32_t*)d_tmp;                         // [npass][ub][kD]
    uint32_t* ghist = status + ub * kD * (uint64_t)npass;        // [nb][npass][kD]
    uint32_t* dbase = ghist + nb * npass * kD;                   // [nb][npass][kD]
    uint32_t* counters = dbase + nb * npass * kD;                // [npass] + ntiles
    const size_t zero_bytes = ((uint64_t)(counters - status) + 64) * 4;
    SegTile* stiles = (SegTile*)((char*)d_tmp + ((zero_bytes + 255) & ~(size_t)255));
    void* btmp = (void*)((char*)stiles + ((ub * sizeof(SegTile) + 255) & ~(size_t)255));
    hipError_t e = hipMemsetAsync(status, 0, zero_bytes, st);
    if (e != hipSuccess) return e;
    e = build_seg_tiles_from_starts(d_bstart, msd_bits, n, stiles, counters + 32, btmp, st, tile);
    if (e != hipSuccess) return e;
    const int shift0 = key_shift + 1;
    hipLaunchKernelGGL((wide_ghist_kernel<DB>), dim3((unsigned)((ub + kWHistTiles - 1) / kWHistTiles)), dim3(kBlock),
                       0, st, recA, stiles, ub, npass, shift0, ghist);
    hipLaunchKernelGGL((wide_dbase_kernel<DB>), dim3((unsigned)(nb * npass)), dim3(kBlock), 0, st, ghist, d_bstart,
                       npass, dbase);
    uint64_t* src = recA;
    uint64_t* dst = recB;
    for (int p = 0; p < npass; ++p) {
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p], st);
        uint32_t* sp = status + (uint64_t)p * ub * kD;
        const int sh = shift0 + DB * p;
        if (var == 2)
            hipLaunchKernelGGL((wide_onesweep_kernel<512, 16, DB>), dim3((unsigned)ub), dim3(512), 0, st, src, dst,
                               stiles, (uint32_t)ub, sh, p, npass, dbase, sp, counters + p, d_err);
        else if (var == 3)
            hipLaunchKernelGGL((wide_onesweep_kernel<1024, 16, DB>), dim3((unsigned)ub), dim3(1024), 0, st, src, dst,
                               stiles, (uint32_t)ub, sh, p, npass, dbase, sp, counters + p, d_err);
        else
            hipLaunchKernelGGL((wide_onesweep_kernel<768, 12, DB>), dim3((unsigned)ub), dim3(768), 0, st, src, dst,
                               stiles, (uint32_t)ub, sh, p, npass, dbase, sp, counters + p, d_err);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p + 1], st);
        std::swap(src, dst);
    }
    return hipSuccess;
}

}  // namespace mums
