// msdsplit.hip -- second level of the MSD split for seed keys wider than the packed
// record's key field plus 8 MSD bits (rows A3-A5 at seed weights 20-21: the default seed
// of genomes above ~1.07 Gbp, getDefaultSeedWeight SeedMasks.h:389-401 via
// MatchList.h:351-357).
//
// A 2w+1 = 43-bit key (w21) leaves 11 key bits outside a (key_low32 << 32 | index32)
// record.  Scattering by all 11 at once writes runs of ~2 records per 4096-position tile
// (2048 buckets), which costs 16 ms at BASELINE config-3 size.  Instead the keys pass
// scatters by the top 8 bits (runs of ~16 records, the w19 kernel) and writes the S <= 4
// key bits between the record's key field and those 8 bits into a side byte per record;
// this pass then partitions every 8-bit parent bucket stably by its side digit, giving
// the 2^(8+S) buckets the segmented LSD sort runs in (bucket = parent << S | side).
//
//   split_count_kernel  : per 4096-record tile of a parent bucket, counts of its 2^S side
//                         digits (reads 1 B per record, byte-packed per-lane counters);
//   one exclusive scan  : hist[tfirst_b * 2^S + d * ntb_b + tb] -> output offsets (the
//                         order bucket-major, digit-major, tile-minor is the output order);
//   split_scatter_kernel: wave64 match-any rank on the side digit, LDS reorder,
//                         digit-run stores (runs of ~4096 / 2^S records).
// HBM bytes per record: 1 (count) + 9 read + 8 written (scatter).
#include "mums_internal.h"

namespace mums {

namespace {

constexpr int kTile = kSegTile;
constexpr int kRounds = kTile / kBlock;
constexpr int kWaves = kBlock / 64;
constexpr int kMaxSide = 16;   // S <= 4

__global__ __launch_bounds__(kBlock) void split_count_kernel(const uint8_t* __restrict__ side,
                                                             const SegTile* __restrict__ tiles, int nd,
                                                             uint32_t* __restrict__ hist) {
    static_assert(kTile == 16 * kBlock, "one 16-B load of side bytes per lane");
    __shared__ uint32_t h[kWaves][kMaxSide];
    const SegTile d = tiles[blockIdx.x];
    if (d.count == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // 16 side bytes per lane (the tile start is not 16-B aligned: byte loads at the edges)
    const uint64_t a0 = d.start + 16ull * tid;
    uint32_t w4[4] = {0, 0, 0, 0};
    uint32_t valid = 0;   // bytes of this lane inside the tile
    if (16u * tid < d.count) {
        valid = d.count - 16u * tid < 16u ? d.count - 16u * tid : 16u;
        if (valid == 16 && (a0 & 3) == 0) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(side + a0);
            #pragma unroll
            for (int k = 0; k < 4; ++k) w4[k] = p[k];
        } else {
            for (uint32_t k = 0; k < valid; ++k) w4[k >> 2] |= (uint32_t)side[a0 + k] << (8 * (k & 3));
        }
    }
    // per-lane counts of the 16 digit values in byte fields (<= 16 each): c[v / 4] byte v % 4
    uint32_t c[4] = {0, 0, 0, 0};
    #pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = (w4[k >> 2] >> (8 * (k & 3))) & 15u;
        const uint32_t inc = (uint32_t)k < valid ? 1u << (8 * (v & 3)) : 0u;
        c[0] += (v >> 2) == 0 ? inc : 0u;
        c[1] += (v >> 2) == 1 ? inc : 0u;
        c[2] += (v >> 2) == 2 ? inc : 0u;
        c[3] += (v >> 2) == 3 ? inc : 0u;
    }
    // wave sum: 8 lanes in byte fields (<= 128), then 16-bit fields (<= 1024)
    #pragma unroll
    for (int o = 1; o <= 4; o <<= 1)
        #pragma unroll
        for (int i = 0; i < 4; ++i) c[i] += __shfl_xor(c[i], o, 64);
    uint32_t h16[8];
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
        h16[2 * i] = c[i] & 0x00FF00FFu;            // values 4i, 4i + 2
        h16[2 * i + 1] = (c[i] >> 8) & 0x00FF00FFu; // values 4i + 1, 4i + 3
    }
    #pragma unroll
    for (int o = 8; o <= 32; o <<= 1)
        #pragma unroll
        for (int i = 0; i < 8; ++i) h16[i] += __shfl_xor(h16[i], o, 64);
    if (lane < kMaxSide) {   // lane v picks value v: byte v % 4 of c[v / 4]
        const uint32_t i = (uint32_t)lane >> 2, j = (uint32_t)lane & 3u;
        uint32_t x = 0;
        #pragma unroll
        for (int q = 0; q < 8; ++q) x = (q == (int)(2 * i + (j & 1))) ? h16[q] : x;
        h[wv][lane] = (j >> 1) ? (x >> 16) : (x & 0xFFFFu);
    }
    __syncthreads();
    if (tid < nd) {
        uint32_t c = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) c += h[w][tid];
        const uint64_t tfirst = d.hbase / 256;   // SegTile.hbase = tfirst_b * 256
        hist[tfirst * nd + (uint64_t)tid * d.ntb + d.tb] = c;
    }
}

// out bucket starts: bstart_out[(b << S) + d] = first output record of side digit d of
// parent bucket b; bstart_out[nb << S] = n
__global__ void split_starts_kernel(const uint32_t* __restrict__ scanned, const uint32_t* __restrict__ bstart_in,
                                    const uint32_t* __restrict__ tfirst, int nbp, int S, uint64_t n,
                                    uint32_t* __restrict__ bstart_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nout = (uint64_t)nbp << S;
    if (i > nout) return;
    if (i == nout) { bstart_out[i] = (uint32_t)n; return; }
    const uint32_t b = (uint32_t)(i >> S), dg = (uint32_t)(i & ((1u << S) - 1));
    const uint32_t ntb = tfirst[b + 1] - tfirst[b];
    bstart_out[i] = ntb == 0 ? bstart_in[b] : scanned[(uint64_t)tfirst[b] * (1u << S) + (uint64_t)dg * ntb];
}

template <int S>
__global__ __launch_bounds__(kBlock) void split_scatter_kernel(const uint64_t* __restrict__ rin,
                                                               const uint8_t* __restrict__ side,
                                                               const SegTile* __restrict__ tiles,
                                                               const uint32_t* __restrict__ hist,
                                                               uint64_t* __restrict__ rout) {
    constexpr int ND = 1 << S;
    __shared__ uint64_t srec[kTile];
    __shared__ uint8_t sdig[kTile];
    __shared__ uint32_t wcnt[kWaves][ND];
    __shared__ uint32_t lstart[ND];
    __shared__ uint32_t gofs[ND];
    const SegTile d = tiles[blockIdx.x];
    if (d.count == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < kWaves * ND) (&wcnt[0][0])[tid] = 0;
    __syncthreads();
    const uint32_t q0 = wv * (kTile / kWaves);
    uint64_t key[kRounds];
    uint32_t dg[kRounds];
    uint32_t rank[kRounds];
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
    }
    {   // the tile's side bytes: 16 per lane into LDS
        const uint64_t a0 = d.start + 16ull * tid;
        if (16u * tid < d.count) {
            const uint32_t valid = d.count - 16u * tid < 16u ? d.count - 16u * tid : 16u;
            if (valid == 16 && (a0 & 3) == 0) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(side + a0);
                #pragma unroll
                for (int k = 0; k < 4; ++k) reinterpret_cast<uint32_t*>(sdig)[4 * tid + k] = p[k];
            } else {
                for (uint32_t k = 0; k < valid; ++k) sdig[16 * tid + k] = side[a0 + k];
            }
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        dg[r] = q < d.count ? (uint32_t)sdig[q] : 0u;
    }
    __syncthreads();   // sdig is rewritten in slot order below
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        const bool valid = q < d.count;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<S>(dg[r], valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][dg[r]];
        if (valid && rk == 0) wcnt[wv][dg[r]] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();
    if (tid < ND) {
        uint32_t acc = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) { const uint32_t c = wcnt[w][tid]; wcnt[w][tid] = acc; acc += c; }
        lstart[tid] = acc;   // digit totals; made exclusive below
        const uint64_t tfirst = d.hbase / 256;
        gofs[tid] = hist[tfirst * ND + (uint64_t)tid * d.ntb + d.tb];
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        #pragma unroll
        for (int k = 0; k < ND; ++k) { const uint32_t c = lstart[k]; lstart[k] = acc; acc += c; }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        if (q < d.count) {
            const uint32_t s = lstart[dg[r]] + wcnt[wv][dg[r]] + rank[r];
            srec[s] = key[r];
            sdig[s] = (uint8_t)dg[r];
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t s = tid + r * kBlock;
        if (s < d.count) {
            const uint32_t k = sdig[s];
            rout[(uint64_t)gofs[k] + (s - lstart[k])] = srec[s];
        }
    }
}

}  // namespace

size_t msd_split_tmp_bytes(uint64_t n, int parent_bits) {
    const uint64_t ub = seg_tiles_upper(n, parent_bits);
    const uint64_t h = ub * kMaxSide + 64;
    return ((ub * sizeof(SegTile) + 255) & ~(size_t)255) + h * 4 + scan_tmp_bytes(h) +
           ((1ull << parent_bits) + 128) * 4 + scan_tmp_bytes((1ull << parent_bits) + 1) + 8192;
}

hipError_t msd_split(const uint64_t* rin, const uint8_t* side, uint64_t* rout, uint64_t n, int parent_bits, int S,
                     const uint32_t* bstart_in, uint32_t* bstart_out, void* d_tmp, hipStream_t st) {
    if (S < 1 || S > 4) return hipErrorInvalidValue;
    const int nbp = 1 << parent_bits, nd = 1 << S;
    const uint64_t ub = seg_tiles_upper(n, parent_bits);
    SegTile* tiles = (SegTile*)d_tmp;
    uint32_t* hist = (uint32_t*)((char*)d_tmp + ((ub * sizeof(SegTile) + 255) & ~(size_t)255));
    const uint64_t h = ub * kMaxSide + 64;
    void* stmp = (void*)(hist + h);
    uint32_t* ctr = hist + h - 32;   // ntiles (unused here)
    void* btmp = (char*)stmp + ((scan_tmp_bytes(h) + 255) & ~(size_t)255);
    hipError_t e = build_seg_tiles_from_starts(bstart_in, parent_bits, n, tiles, ctr, btmp, st);
    if (e != hipSuccess) return e;
    // tfirst (tiles per parent bucket, scanned) is left at the start of btmp
    const uint32_t* tfirst = (const uint32_t*)btmp;
    e = hipMemsetAsync(hist, 0, ub * nd * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(split_count_kernel, dim3((unsigned)ub), dim3(kBlock), 0, st, side, tiles, nd, hist);
    e = exclusive_scan_u32(hist, ub * nd, stmp, nullptr, st);
    if (e != hipSuccess) return e;
    const uint64_t nout = (uint64_t)nbp << S;
    hipLaunchKernelGGL(split_starts_kernel, dim3((unsigned)((nout + 256) / 256)), dim3(256), 0, st, hist, bstart_in,
                       tfirst, nbp, S, n, bstart_out);
    switch (S) {
        case 1: hipLaunchKernelGGL(split_scatter_kernel<1>, dim3((unsigned)ub), dim3(kBlock), 0, st, rin, side, tiles, hist, rout); break;
        case 2: hipLaunchKernelGGL(split_scatter_kernel<2>, dim3((unsigned)ub), dim3(kBlock), 0, st, rin, side, tiles, hist, rout); break;
        case 3: hipLaunchKernelGGL(split_scatter_kernel<3>, dim3((unsigned)ub), dim3(kBlock), 0, st, rin, side, tiles, hist, rout); break;
        default: hipLaunchKernelGGL(split_scatter_kernel<4>, dim3((unsigned)ub), dim3(kBlock), 0, st, rin, side, tiles, hist, rout); break;
    }
    return hipGetLastError();
}

}  // namespace mums
