// groups.hip -- segmented equal-range scan over the merged sorted key stream (rows A7-A9).
//
// Reference: MatchFinder::SearchRange (MatchFinder.cpp:172-340) walks the G
// sorted mer lists in masked-key order and hands every group of equal masked
// keys to MemHash::EnumerateMatches (MemHash.cpp:139-162), which accepts it or
// not and builds the seed probe (HashMatch :167-187, SetDirection :189-203,
// CalculateOffset MatchHashEntry.cpp:141-160) whose hash bucket is
// ((offset % T) + T) % T (MemHash.cpp:213).
//
// Here the merged stream is the radix-sorted record array; a group is a run of
// equal ckey>>1.  One workgroup per 4096-record tile (probe_tile_rec_kernel for
// the packed records: the tile is staged in LDS and the default-tolerance probe is
// branch-free; probe_tile_kernel for the (key, index) pair path):
//   1. lane-contiguous head detection (16 rounds), heads compacted into an LDS
//      list in stream order (ballot + per-(round, wave) counts);
//   2. every lane builds the probe of one head (no lane idles on non-heads);
//   3. accepted probes are compacted in head order into the tile's slot range
//      (a group needs >= 2 records, so <= 2048 probes per tile).
// A second kernel concatenates the tiles' slots using the scanned tile counts, so
// the probes end up in ascending key order = the reference's AddHashEntry order.
#include <cstdlib>
#include <type_traits>

#include "match_device.h"
#include "seed_device.h"

namespace mums {

namespace {

constexpr int kGTile = kSegTile;
constexpr int kGRounds = kGTile / kBlock;
constexpr int kSlots = kGTile / 2;
// packed-record probe stage: kGSplit workgroups per sort tile (half the LDS per block,
// twice the blocks per CU to hide the record loads behind the other blocks' probe work)
#ifndef MUMS_GROUP_SPLIT
#define MUMS_GROUP_SPLIT 2
#endif
constexpr int kGSplit = MUMS_GROUP_SPLIT;
constexpr int kGSub = kGTile / kGSplit;
constexpr int kGSubRounds = kGSub / kBlock;
constexpr int kSubSlots = kGSub / 2;
static_assert(kGSub % kBlock == 0 && kGSubRounds * (kBlock / 64) <= 64, "probe sub-tile");

__device__ __forceinline__ uint32_t blk_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = v;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    #pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint32_t x = s_w[w];
        pre += (w < wv) ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void probe_tile_kernel(View v, const SegTile* __restrict__ tiles, uint64_t N,
                                                            GenomeTable gt, MatchParams mp, int L,
                                                            uint32_t* __restrict__ tile_count,
                                                            uint64_t* __restrict__ slot_info,
                                                            uint32_t* __restrict__ slot_bucket,
                                                            DevCounters* __restrict__ ctr) {
    __shared__ uint16_t heads[kGTile];
    __shared__ uint32_t okb[kGTile];        // bucket | (ok << 31) per head (bucket < 2^31)
    __shared__ uint16_t gsz16[kGTile];
    __shared__ uint32_t wcnt[kGRounds][kBlock / 64];
    __shared__ uint32_t s_w[kBlock / 64];
    __shared__ uint32_t s_red[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const SegTile td = tiles[blockIdx.x];
    if (td.count == 0) {
        if (threadIdx.x == 0) {
            tile_count[blockIdx.x] = 0;
            tile_count[gridDim.x + 32 + blockIdx.x] = 0;
        }
        return;
    }
    const uint64_t tile0 = td.start;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    // 1) heads in stream order
    uint32_t hmask = 0;
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const uint32_t q = r * kBlock + threadIdx.x;
        const uint64_t i = tile0 + q;
        bool head = false;
        if (q < td.count) head = (i == td.bstart) || (v.gkey(i) != v.gkey(i - 1));
        hmask |= (head ? 1u : 0u) << r;
        const uint64_t bal = __ballot(head);
        if (lane == 0) wcnt[r][wv] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int r = 0; r < kGRounds; ++r)
            for (int w = 0; w < kBlock / 64; ++w) { const uint32_t c = wcnt[r][w]; wcnt[r][w] = acc; acc += c; }
        s_red[0] = acc;
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const bool head = (hmask >> r) & 1u;
        const uint64_t bal = __ballot(head);
        if (head) heads[wcnt[r][wv] + (uint32_t)__popcll(bal & lt)] = (uint16_t)(r * kBlock + threadIdx.x);
    }
    __syncthreads();
    const uint32_t H = s_red[0];

    // 2) one probe per lane (offset only: the replay rebuilds the starts)
    uint32_t nrep = 0;
    const bool fast = mp.repeat_tol == 0 && mp.enum_tol == 1;
    for (uint32_t j = threadIdx.x; j < H; j += kBlock) {
        uint32_t gsz = 0;
        int64_t off = 0;
        bool ok;
        if (fast) {
            ok = probe_offset_fast<MG, View>(v, tile0 + heads[j], td.bend, gt, mp, L, &off, &gsz);
        } else {
            Mhe<MG> P;
            ok = build_probe<MG, View>(v, tile0 + heads[j], td.bend, gt, mp, L, P, &gsz);
            off = P.offset;
        }
        nrep += gsz > (uint32_t)kRepeatLimit;
        okb[j] = ok ? (0x80000000u | bucket_of(off, mp.table_size)) : 0u;
        gsz16[j] = (uint16_t)(gsz > 65535u ? 65535u : gsz);
    }
    if (nrep) atomicAdd(&ctr->repeat_limit, (unsigned long long)nrep);   // rare (repeat-rich input only)
    __syncthreads();

    // 3) compact accepted probes in head order into this tile's slots
    uint32_t base = 0;
    const uint64_t sb = (uint64_t)blockIdx.x * kSlots;
    for (uint32_t c = 0; c < H; c += kBlock) {
        const uint32_t j = c + threadIdx.x;
        const uint32_t vv = j < H ? okb[j] : 0u;
        const uint32_t ok = vv >> 31;
        uint32_t tot;
        const uint32_t o = blk_excl_scan(ok, s_w, &tot);
        if (ok) {
            slot_info[sb + base + o] = (tile0 + heads[j]) | ((uint64_t)gsz16[j] << 32);
            slot_bucket[sb + base + o] = vv & 0x7FFFFFFFu;
        }
        base += tot;
    }
    if (threadIdx.x == 0) {
        tile_count[blockIdx.x] = base;
        tile_count[gridDim.x + 32 + blockIdx.x] = H;   // per-tile group count (summed by the host side)
    }
}

// Packed-record path: the tile's records are staged in LDS once; head detection and
// the probes read them there (a group that runs past the tile end falls back to the
// global stream), and the compaction is fused into the probe loop, so a block makes one
// global load round and one store round.
typedef __attribute__((address_space(3))) const uint64_t lds_u64;

template <int IB>
struct TileRecViewT {
    lds_u64* lds;           // records [t0, t0 + count) of the sorted stream (LDS)
    const uint64_t* glob;   // the whole sorted stream
    uint64_t t0;
    uint32_t count;
    __device__ __forceinline__ uint64_t raw(uint64_t i) const {
        const uint64_t k = i - t0;
        return k < count ? lds[k] : glob[i];
    }
    __device__ __forceinline__ uint64_t gkey(uint64_t i) const { return raw(i) >> (IB + 1); }
    __device__ __forceinline__ uint32_t par(uint64_t i) const { return (uint32_t)(raw(i) >> IB) & 1u; }
    __device__ __forceinline__ uint64_t gidx(uint64_t i) const { return raw(i) & ((1ull << IB) - 1); }
    __device__ __forceinline__ RecFields get(uint64_t i) const {
        const uint64_t r = raw(i);
        return RecFields{r >> (IB + 1), (uint32_t)(r >> IB) & 1u, r & ((1ull << IB) - 1)};
    }
};

// kFastOnly: default tolerances only (repeat_tol 0, enum_tol 1) -- the general build_probe path
// is not compiled in, so its registers do not weigh on the branch-free probe
template <int MG, int IB, bool kGl = false, bool kFastOnly = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kGl ? 6 : 1))) void probe_tile_rec_kernel(const uint64_t* __restrict__ rec,
                                                                const SegTile* __restrict__ tiles, GenomeTable gt,
                                                                MatchParams mp, int L,
                                                                uint32_t* __restrict__ tile_count,
                                                                uint64_t* __restrict__ slot_info,
                                                                uint32_t* __restrict__ slot_bucket,
                                                                DevCounters* __restrict__ ctr,
                                                                double inv_table) {
    constexpr int kGRounds = kGSubRounds;   // this block's part of the tile
    __shared__ uint64_t srec[kGSub];
    __shared__ uint16_t heads[kSubSlots];  // heads of groups of >= 2 records (<= kGSub / 2)
    __shared__ uint32_t wcnt[kGRounds * (kBlock / 64)];
    __shared__ uint32_t s_w[kBlock / 64];
    __shared__ uint32_t s_red[2];
    __shared__ uint64_t s_prev, s_next;
    __shared__ uint8_t s_gl[256];
    __shared__ uint32_t s_gb[kMaxG + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const SegTile td = tiles[blockIdx.x / kGSplit];
    const uint32_t part0 = (blockIdx.x % kGSplit) * (uint32_t)kGSub;
    if (td.count <= part0) {
        if (threadIdx.x == 0) {
            tile_count[blockIdx.x] = 0;
            tile_count[gridDim.x + 32 + blockIdx.x] = 0;
        }
        return;
    }
    const uint64_t tile0 = td.start + part0;
    const uint32_t cnt = td.count - part0 < (uint32_t)kGSub ? td.count - part0 : (uint32_t)kGSub;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    // 1) stage the tile (lane-contiguous, coalesced) + the records just before and after
    //    it.  The loads use clamped indices so all kGRounds are in flight before the
    //    first LDS store.
    {
        uint64_t x[kGRounds];
        #pragma unroll
        for (int r = 0; r < kGRounds; ++r) {
            const uint32_t q = r * kBlock + threadIdx.x;
            x[r] = rec[tile0 + (q < cnt ? q : cnt - 1)];
        }
        #pragma unroll
        for (int r = 0; r < kGRounds; ++r) {
            const uint32_t q = r * kBlock + threadIdx.x;
            if (q < cnt) srec[q] = x[r];
        }
    }
    if (threadIdx.x == 0) s_prev = (tile0 > td.bstart) ? rec[tile0 - 1] : ~0ull;
    if (threadIdx.x == 64) s_next = (tile0 + cnt < td.bend) ? rec[tile0 + cnt] : ~0ull;
    // the coarse genome lookup in LDS (GenomeTable gl_*; 32-bit indices)
    constexpr bool use_gl = kGl && IB == 32;   // (the launcher checks gt.gl_n)
    if constexpr (use_gl) {   // gl_n <= 256 = kBlock, kMaxG + 1 <= kBlock: one element a thread
        static_assert(kBlock >= 256 && kBlock > kMaxG, "one lookup entry per thread");
        if (threadIdx.x < gt.gl_n) s_gl[threadIdx.x] = gt.gl[threadIdx.x];
        if (threadIdx.x <= kMaxG) s_gb[threadIdx.x] = (uint32_t)gt.base[threadIdx.x];
    }
    const GLook glk{(lds_u8c*)s_gl, (lds_u32c*)s_gb, gt.gl_shift, gt.gl_n ? gt.gl_n - 1 : 0};
    __syncthreads();

    // 2) group heads in stream order; a head is kept only when its group has >= 2
    //    records (a single record is never an AddHashEntry call)
    uint32_t hmask = 0, ngrp = 0;
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const uint32_t q = r * kBlock + threadIdx.x;
        bool keep = false;
        if (q < cnt) {
            const uint64_t here = srec[q] >> (IB + 1);
            const uint64_t prev = (q == 0) ? ((tile0 == td.bstart) ? ~0ull : (s_prev >> (IB + 1)))
                                           : (srec[q - 1] >> (IB + 1));
            const uint64_t next = (q + 1 < cnt) ? (srec[q + 1] >> (IB + 1)) : (s_next >> (IB + 1));
            const bool head = (q == 0 && tile0 == td.bstart) || here != prev;
            ngrp += head ? 1u : 0u;
            keep = head && next == here;
        }
        hmask |= (keep ? 1u : 0u) << r;
        const uint64_t bal = __ballot(keep);
        if (lane == 0) wcnt[r * (kBlock / 64) + wv] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    if (wv == 0) {   // exclusive scan of the kGRounds x waves counts (one wave, <= 64 entries)
        constexpr int kE = kGRounds * (kBlock / 64);
        const uint32_t c0 = lane < kE ? wcnt[lane] : 0u;
        uint32_t inc = c0;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        if (lane < kE) wcnt[lane] = inc - c0;
        if (lane == 63) s_red[0] = inc;
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const bool keep = (hmask >> r) & 1u;
        const uint64_t bal = __ballot(keep);
        if (keep) heads[wcnt[r * (kBlock / 64) + wv] + (uint32_t)__popcll(bal & lt)] = (uint16_t)(r * kBlock + threadIdx.x);
    }
    __syncthreads();
    const uint32_t H = s_red[0];

    // 3) one probe per lane, compacted in head order into this tile's slots
    const TileRecViewT<IB> v{(lds_u64*)srec, rec, tile0, cnt};
    const bool fast = kFastOnly || (mp.repeat_tol == 0 && mp.enum_tol == 1);
    const double inv_t = inv_table;   // 1 / table_size from the host (a double division per block otherwise)
    const uint64_t sb = (uint64_t)blockIdx.x * kSubSlots;
    uint32_t nrep = 0, base = 0;
    for (uint32_t c = 0; c < H; c += kBlock) {
        const uint32_t j = c + threadIdx.x;
        bool ok = false;
        uint32_t gsz = 0, bkt = 0;
        uint64_t h = 0;
        if (j < H) {
            h = tile0 + heads[j];
            int64_t off = 0;
            if (fast) {
                // the batch (records h .. h + G) from LDS when it lies in the tile, without
                // branches; a group crossing the tile end reads the global stream
                const uint32_t q = heads[j];
                uint64_t xb[MG + 1];
                if (q + (uint32_t)gt.G < cnt) {
                    #pragma unroll
                    for (int k = 0; k <= MG; ++k) {
                        const uint32_t qk = q + ((uint32_t)k <= (uint32_t)gt.G ? (uint32_t)k : 0u);
                        xb[k] = ((uint32_t)k <= (uint32_t)gt.G) ? v.lds[qk] : ~0ull;
                    }
                } else {
                    #pragma unroll
                    for (int k = 0; k <= MG; ++k)
                        xb[k] = ((uint32_t)k <= (uint32_t)gt.G && h + k < td.bend) ? rec[h + k] : ~0ull;
                }
                ok = probe_fast_raw<MG, IB, use_gl>(xb, gt, mp, L, &off, &gsz, &glk);
                if (gsz > (uint32_t)gt.G) {   // oversize group: rejected; count on for the report
                    uint64_t i = h + gsz;
                    const uint32_t k0 = (uint32_t)(xb[0] >> (IB + 1));
                    while (i < td.bend && gsz <= (uint32_t)kRepeatLimit && (uint32_t)v.gkey(i) == k0) { ++gsz; ++i; }
                }
            } else if constexpr (!kFastOnly) {
                Mhe<MG> P;
                ok = build_probe<MG, TileRecViewT<IB>>(v, h, td.bend, gt, mp, L, P, &gsz);
                off = P.offset;
            }
            nrep += gsz > (uint32_t)kRepeatLimit;
            if (ok) bkt = bucket_of_fast(off, mp.table_size, inv_t);
        }
        uint32_t tot;
        const uint32_t o = blk_excl_scan(ok ? 1u : 0u, s_w, &tot);
        if (ok) {
            slot_info[sb + base + o] = h | ((uint64_t)(gsz > 65535u ? 65535u : gsz) << 32);
            slot_bucket[sb + base + o] = bkt;
        }
        base += tot;
    }
    if (nrep) atomicAdd(&ctr->repeat_limit, (unsigned long long)nrep);   // rare (repeat-rich input only)
    uint32_t gtot;
    (void)blk_excl_scan(ngrp, s_w, &gtot);
    if (threadIdx.x == 0) {
        tile_count[blockIdx.x] = base;
        tile_count[gridDim.x + 32 + blockIdx.x] = gtot;   // per-tile group count (summed by the host side)
    }
}

__global__ __launch_bounds__(kBlock) void probe_compact_kernel(const uint32_t* __restrict__ tile_count,
                                                               const uint32_t* __restrict__ tile_off,
                                                               const uint64_t* __restrict__ slot_info,
                                                               const uint32_t* __restrict__ slot_bucket,
                                                               uint64_t* __restrict__ probe_info,
                                                               uint32_t* __restrict__ probe_bucket,
                                                               uint32_t slots_per_block) {
    const uint32_t n = tile_count[blockIdx.x];
    const uint64_t o = tile_off[blockIdx.x];
    const uint64_t sb = (uint64_t)blockIdx.x * slots_per_block;
    for (uint32_t k = threadIdx.x; k < n; k += kBlock) {
        probe_info[o + k] = slot_info[sb + k];
        probe_bucket[o + k] = slot_bucket[sb + k];
    }
}

__global__ void flat_tiles_kernel(uint64_t N, uint64_t nt, SegTile* __restrict__ tiles) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    SegTile d{};
    d.start = t * kGTile;
    d.bstart = 0;
    d.bend = N;
    const uint64_t rem = N - d.start;
    d.count = (uint32_t)(rem < (uint64_t)kGTile ? rem : (uint64_t)kGTile);
    d.hbase = 0;
    d.ntb = (uint32_t)nt;
    d.tb = (uint32_t)t;
    tiles[t] = d;
}

// probe k (key order) -> MatProbes row k: build_probe once per probe for the replay.
// Packed records under the default tolerances load the group (<= G records, size in
// probe_info) as one batch of independent loads (probe_row_fast).  lkey / fsk (optional):
// the chain labelling's line key (chains.hip) and the first-genome start of probe k, so
// neither re-reads the rows.
#ifndef MUMS_MAT_WIDE
#define MUMS_MAT_WIDE 1   // materialize: a group's records as 16-B loads (0: one 8-B load each)
#endif
constexpr bool kMatWide = MUMS_MAT_WIDE != 0;
struct __attribute__((aligned(8))) Rec2 { uint64_t a, b; };

template <int MG, typename View, bool kGl = false>
__global__ __launch_bounds__(kBlock) void probe_materialize_kernel(View v, const uint64_t* __restrict__ probe_info,
                                                                   uint64_t P, GenomeTable gt, MatchParams mp, int L,
                                                                   int64_t* __restrict__ rows, uint64_t* __restrict__ lkey,
                                                                   uint32_t* __restrict__ fsk, uint32_t* __restrict__ lhash,
                                                                   int32_t* __restrict__ rows32) {
    const uint64_t k0 = (uint64_t)blockIdx.x * kBlock;
    const uint64_t k = k0 + threadIdx.x;
    const int W = gt.G + 1;
    Mhe<MG> Q;
    __shared__ uint8_t s_gl[256];
    __shared__ uint32_t s_gb[kMaxG + 1];
    constexpr bool use_gl = kGl && RecIB<View>::value == 32;   // (the launcher checks gt.gl_n)
    if constexpr (use_gl) {   // the coarse genome lookup in LDS (GenomeTable gl_*)
        for (uint32_t i = threadIdx.x; i < gt.gl_n; i += kBlock) s_gl[i] = gt.gl[i];
        for (int i = threadIdx.x; i <= kMaxG; i += kBlock) s_gb[i] = (uint32_t)gt.base[i];
        __syncthreads();
    }
    const GLook glk{(lds_u8c*)s_gl, (lds_u32c*)s_gb, gt.gl_shift, gt.gl_n ? gt.gl_n - 1 : 0};
    if (k < P) {
        const uint64_t info = probe_info[k];
        const uint64_t h = info & 0xFFFFFFFFull;
        const uint32_t gsz = (uint32_t)((info >> 32) & 0xFFFFull);
        bool done = false;
        if constexpr (RecIB<View>::value > 0) {
            if (mp.repeat_tol == 0 && mp.enum_tol == 1 && gsz <= (uint32_t)MG) {
                uint64_t x[MG];
                if constexpr (MG % 2 == 0 && kMatWide) {
                    // two records per 16-B load: the lanes' groups lie apart, so each load
                    // instruction is an address-unit pass over up to 64 cache lines; the record
                    // after a group's last is read and dropped (the buffers end in >= 8 spare)
                    #pragma unroll
                    for (int q = 0; q < MG; q += 2) {
                        Rec2 t{~0ull, ~0ull};
                        if ((uint32_t)q < gsz) t = *reinterpret_cast<const Rec2*>(v.rec + h + q);
                        x[q] = t.a;
                        x[q + 1] = (uint32_t)(q + 1) < gsz ? t.b : ~0ull;
                    }
                } else {
                    #pragma unroll
                    for (int q = 0; q < MG; ++q) x[q] = (uint32_t)q < gsz ? v.rec[h + q] : ~0ull;
                }
                probe_row_fast<MG, RecIB<View>::value, use_gl>(x, gsz, gt, L, Q, &glk);
                done = true;
            }
        }
        if (!done) {
            uint32_t gs;
            build_probe<MG, View>(v, h, h + gsz, gt, mp, L, Q, &gs);
        }
        if (lkey) {
            const uint64_t xs = (uint64_t)start_at(Q, first_start(Q));
            if (lhash) {   // the line sort's first records (chain_line_slots) and the hashes apart
                lkey[k] = (xs << 32) | k;
                lhash[k] = line_hash<MG>(Q, gt.G);
            } else {
                lkey[k] = ((uint64_t)line_hash<MG>(Q, gt.G) << 32) | (xs & 0xFFFFFFFFull);
            }
            fsk[k] = (uint32_t)xs;
        }
    }
    if constexpr (MG % 4 == 0 && MG <= 16) {
        if (rows32) {   // uniform: int32 starts (MatProbes::rows32); fsk[P] |= 1 when one does not fit
            if (k >= P) return;
            bool ok = probe_offset<MG>(Q, L) == Q.offset;
            #pragma unroll
            for (int g = 0; g < MG; ++g) ok = ok && Q.s[g] == (int64_t)(int32_t)Q.s[g];
            int32_t* out = rows32 + k * (uint64_t)line_row_stride(gt.G);
            #pragma unroll
            for (int q = 0; q < MG / 4; ++q)
                if (4 * q < gt.G)
                    *reinterpret_cast<int4*>(out + 4 * q) = make_int4((int32_t)Q.s[4 * q], (int32_t)Q.s[4 * q + 1],
                                                                      (int32_t)Q.s[4 * q + 2], (int32_t)Q.s[4 * q + 3]);
            if (!ok) atomicOr(fsk + P, 1u);
            return;
        }
    }
    if constexpr (MG <= 16) {
        // the block's rows are one contiguous range: staged in LDS, stored with consecutive
        // lanes on consecutive words (one lane per row would touch a 128-B line per lane and
        // word: W x 64 lines per store instruction)
        __shared__ int64_t srow[kBlock * (MG + 1)];
        if (k < P) {
            int64_t* r = srow + threadIdx.x * W;
            #pragma unroll
            for (int g = 0; g < MG; ++g)
                if (g < gt.G) r[g] = Q.s[g];
            r[gt.G] = Q.offset;
        }
        __syncthreads();
        const uint64_t nk = P - k0 < (uint64_t)kBlock ? P - k0 : (uint64_t)kBlock;
        int64_t* out = rows + k0 * (uint64_t)W;
        for (uint32_t i = threadIdx.x; i < nk * (uint64_t)W; i += kBlock) out[i] = srow[i];
    } else {
        if (k >= P) return;
        int64_t* row = rows + k * (uint64_t)W;
        #pragma unroll
        for (int g = 0; g < MG; ++g)
            if (g < gt.G) row[g] = Q.s[g];
        row[gt.G] = Q.offset;
    }
}

// bucket (MemHash.cpp:213) of every row; dest = owning rank of that bucket when bounds
// (nranks + 1 bucket boundaries) are given
__global__ __launch_bounds__(kBlock) void row_bucket_kernel(const int64_t* __restrict__ rows, uint64_t P, int G,
                                                            uint32_t table_size, double inv_t,
                                                            const uint32_t* __restrict__ bounds, uint32_t nranks,
                                                            uint32_t* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    const uint32_t b = bucket_of_fast(rows[k * (uint64_t)(G + 1) + G], table_size, inv_t);
    if (!bounds) { out[k] = b; return; }
    uint32_t r = 0;
    while (r + 1 < nranks && bounds[r + 1] <= b) ++r;
    out[k] = r;
}

// the same with kGatherIPT elements per thread, all loads in flight together (consecutive
// lanes stay on consecutive words: a row is read by W neighbouring lanes)
constexpr int kGatherIPT = 8;
__global__ __launch_bounds__(kBlock) void gather_rows_ilp_kernel(const int64_t* __restrict__ src,
                                                                 const uint32_t* __restrict__ perm, uint64_t n, uint32_t W,
                                                                 int64_t* __restrict__ dst) {
    const uint64_t e0 = (uint64_t)blockIdx.x * (kBlock * kGatherIPT) + threadIdx.x;
    uint64_t k = e0 / W;
    uint32_t c = (uint32_t)(e0 - k * W);
    const uint32_t dk = kBlock / W, dc = kBlock % W;
    int64_t x[kGatherIPT];
    #pragma unroll
    for (int i = 0; i < kGatherIPT; ++i) {
        const uint64_t e = e0 + (uint64_t)i * kBlock;
        x[i] = e < n ? src[(uint64_t)perm[k] * W + c] : 0;
        k += dk;
        c += dc;
        if (c >= W) { c -= W; ++k; }
    }
    #pragma unroll
    for (int i = 0; i < kGatherIPT; ++i) {
        const uint64_t e = e0 + (uint64_t)i * kBlock;
        if (e < n) dst[e] = x[i];
    }
}

// the probes' bucket partition as packed records (bucket << 32 | probe) for the onesweep
// sort, and back to the two arrays the consumers read
__global__ __launch_bounds__(kBlock) void bucket_rec_kernel(const uint32_t* __restrict__ b, uint64_t P,
                                                            uint64_t* __restrict__ rec) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < P) rec[k] = ((uint64_t)b[k] << 32) | k;
}

__global__ __launch_bounds__(kBlock) void bucket_split_kernel(const uint64_t* __restrict__ rec, uint64_t P,
                                                              uint32_t* __restrict__ b, uint32_t* __restrict__ ids) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    const uint64_t r = rec[k];
    b[k] = (uint32_t)(r >> 32);
    ids[k] = (uint32_t)r;
}

// ---- sharded FindMatches: chains labelled where the probes are (mums_shard_chain_*) -----
// cdest[c] = destination rank of chain c = the rank owning its first probe's bucket (all
// probes of a chain share one line, hence one offset and one bucket, MemHash.cpp:213)
__global__ __launch_bounds__(kBlock) void chain_dest_kernel(const uint32_t* __restrict__ fk, uint64_t nch,
                                                            const uint32_t* __restrict__ pdest,
                                                            uint32_t* __restrict__ cdest) {
    const uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c < nch) cdest[c] = pdest[fk[c]];
}

__global__ __launch_bounds__(kBlock) void inverse_perm_kernel(const uint32_t* __restrict__ perm, uint64_t n,
                                                              uint32_t* __restrict__ inv) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < n) inv[perm[k]] = (uint32_t)k;
}

// the k-th exported row's chain: its entry's index inside the destination's entry block
__global__ __launch_bounds__(kBlock) void chain_tag_kernel(const uint32_t* __restrict__ chain_of,
                                                           const uint32_t* __restrict__ perm,
                                                           const uint32_t* __restrict__ sdest, uint64_t P,
                                                           const uint32_t* __restrict__ cinv,
                                                           const uint32_t* __restrict__ cstart,
                                                           uint32_t* __restrict__ tags) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < P) tags[k] = cinv[chain_of[perm[k]]] - cstart[sdest[k]];
}

// the k-th exported entry: chain cperm[k] (G + 2 words) and its first probe's index inside
// the destination's row block
__global__ __launch_bounds__(kBlock) void chain_entry_out_kernel(const int64_t* __restrict__ pool,
                                                                 const uint32_t* __restrict__ fk,
                                                                 const uint32_t* __restrict__ cperm,
                                                                 const uint32_t* __restrict__ scdest, uint64_t nch,
                                                                 int G, const uint32_t* __restrict__ pinv,
                                                                 const uint32_t* __restrict__ rstart,
                                                                 int64_t* __restrict__ eout, uint32_t* __restrict__ fout) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= nch) return;
    const uint32_t c = cperm[k];
    const uint64_t W = (uint64_t)(G + 2);
    for (uint64_t w = 0; w < W; ++w) eout[k * W + w] = pool[(uint64_t)c * W + w];
    if (fout) fout[k] = pinv[fk[c]] - rstart[scdest[k]];   // (null: the entries alone, mums_shard_chain_entries)
}

// ---- the sharded kept-probe export (mums_shard_kept_export) ----------
// probe k of chain c (export position x = cinv[c], owner's answer thr[x] = {next_s, first}) is
// sent when the owner's replay needs it -- the chain's first AddHashEntry call (the first probe of
// a chain whose first call sits on this rank) or a probe starting at or past next_s (suspicious:
// another chain of the bucket and genome set starts in [chain start, probe start]); every other
// probe collides with its chain entry.  dest = pdest (sent) or nranks + pdest (dropped), so one
// stable sort by dest groups the sent rows by rank in key order and counts the dropped ones.
__global__ __launch_bounds__(kBlock) void kept_dest_kernel(const int64_t* __restrict__ rows, uint64_t P, int G,
                                                           const uint32_t* __restrict__ chain_of,
                                                           const uint32_t* __restrict__ cinv,
                                                           const uint2* __restrict__ thr,
                                                           const uint32_t* __restrict__ fk,
                                                           const uint32_t* __restrict__ pdest, uint32_t nranks,
                                                           uint32_t* __restrict__ dest) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    const uint32_t c = chain_of[k];
    const uint2 t = thr[cinv[c]];
    bool keep = t.y != 0u && fk[c] == (uint32_t)k;
    if (!keep) {
        const int64_t* r = rows + k * (uint64_t)(G + 1);
        int64_t fs = 0;   // the first present genome's start (forward by SetDirection: > 0)
        for (int g = 0; g < G && fs == 0; ++g) fs = r[g];
        keep = (uint64_t)fs >= (uint64_t)t.x;
    }
    dest[k] = keep ? pdest[k] : nranks + pdest[k];
}

// first[d] = the first sorted position holding dest d (P when none)
__global__ __launch_bounds__(kBlock) void dest_first_kernel(const uint32_t* __restrict__ sdest, uint64_t P,
                                                            uint32_t* __restrict__ first) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < P && (i == 0 || sdest[i - 1] != sdest[i])) first[sdest[i]] = (uint32_t)i;
}

// per exported entry: its first sent row inside its destination's row block (the block's end when
// none of the chain's probes on this rank was sent)
__global__ __launch_bounds__(kBlock) void entry_first_init_kernel(const uint32_t* __restrict__ scdest, uint64_t nch,
                                                                  const uint32_t* __restrict__ rcount,
                                                                  uint32_t* __restrict__ efirst) {
    const uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (x < nch) efirst[x] = rcount[scdest[x]];
}

__global__ __launch_bounds__(kBlock) void entry_first_kernel(const uint32_t* __restrict__ perm,
                                                             const uint32_t* __restrict__ sdest, uint64_t K,
                                                             const uint32_t* __restrict__ chain_of,
                                                             const uint32_t* __restrict__ cinv,
                                                             const uint32_t* __restrict__ rstart,
                                                             uint32_t* __restrict__ efirst) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < K) atomicMin(&efirst[cinv[chain_of[perm[i]]]], (uint32_t)i - rstart[sdest[i]]);
}

// A sharded rank's merged packed records (its MSD buckets [kfirst, kfirst + nb), starts
// bst[0..nb]) as (full ckey, 32-bit global index) pairs: the group scans that need a
// group's whole key (enumeration tolerance, pairwise.hip) then never merge two buckets.
template <typename I, int IB>
__global__ __launch_bounds__(kBlock) void rec_pairs_kernel(const uint64_t* __restrict__ rec, uint64_t n,
                                                           const uint32_t* __restrict__ bst, uint32_t nb,
                                                           uint32_t kfirst, int kb_rec, uint64_t* __restrict__ key,
                                                           I* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = nb;   // last bucket j with bst[j] <= i (empty buckets skipped)
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (bst[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    const uint64_t r = rec[i];
    key[i] = ((uint64_t)(kfirst + lo) << kb_rec) | (r >> IB);
    idx[i] = (I)(r & ((1ull << IB) - 1));
}

}  // namespace

hipError_t launch_rec_pairs(const uint64_t* rec, uint64_t n, const uint32_t* d_bst, uint32_t nb, uint32_t kfirst,
                            int kb_rec, uint64_t* key, uint32_t* idx, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((rec_pairs_kernel<uint32_t, 32>), dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       rec, n, d_bst, nb, kfirst, kb_rec, key, idx);
    return hipGetLastError();
}

hipError_t launch_rec_pairs33(const uint64_t* rec, uint64_t n, const uint32_t* d_bst, uint32_t nb, uint32_t kfirst,
                              int kb_rec, uint64_t* key, uint64_t* idx, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((rec_pairs_kernel<uint64_t, 33>), dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       rec, n, d_bst, nb, kfirst, kb_rec, key, idx);
    return hipGetLastError();
}

hipError_t launch_chain_dest(const uint32_t* fk, uint64_t nch, const uint32_t* pdest, uint32_t* cdest, hipStream_t st) {
    if (nch == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_dest_kernel, dim3((unsigned)((nch + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, fk, nch,
                       pdest, cdest);
    return hipGetLastError();
}

hipError_t launch_inverse_perm(const uint32_t* perm, uint64_t n, uint32_t* inv, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(inverse_perm_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, perm, n,
                       inv);
    return hipGetLastError();
}

hipError_t launch_chain_tags(const uint32_t* chain_of, const uint32_t* perm, const uint32_t* sdest, uint64_t P,
                             const uint32_t* cinv, const uint32_t* cstart, uint32_t* tags, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_tag_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, chain_of,
                       perm, sdest, P, cinv, cstart, tags);
    return hipGetLastError();
}

hipError_t launch_chain_entries_out(const int64_t* pool, const uint32_t* fk, const uint32_t* cperm,
                                    const uint32_t* scdest, uint64_t nch, int G, const uint32_t* pinv,
                                    const uint32_t* rstart, int64_t* eout, uint32_t* fout, hipStream_t st) {
    if (nch == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_entry_out_kernel, dim3((unsigned)((nch + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       pool, fk, cperm, scdest, nch, G, pinv, rstart, eout, fout);
    return hipGetLastError();
}

hipError_t launch_kept_dest(const int64_t* rows, uint64_t P, int G, const uint32_t* chain_of, const uint32_t* cinv,
                            const uint2* thr, const uint32_t* fk, const uint32_t* pdest, uint32_t nranks, uint32_t* dest,
                            hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(kept_dest_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, rows, P, G,
                       chain_of, cinv, thr, fk, pdest, nranks, dest);
    return hipGetLastError();
}

hipError_t launch_dest_first(const uint32_t* sdest, uint64_t P, uint32_t* first, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(dest_first_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, sdest, P,
                       first);
    return hipGetLastError();
}

hipError_t launch_entry_first(const uint32_t* scdest, uint64_t nch, const uint32_t* rcount, const uint32_t* perm,
                              const uint32_t* sdest, uint64_t K, const uint32_t* chain_of, const uint32_t* cinv,
                              const uint32_t* rstart, uint32_t* efirst, hipStream_t st) {
    if (nch == 0) return hipSuccess;
    hipLaunchKernelGGL(entry_first_init_kernel, dim3((unsigned)((nch + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       scdest, nch, rcount, efirst);
    if (K)
        hipLaunchKernelGGL(entry_first_kernel, dim3((unsigned)((K + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, perm,
                           sdest, K, chain_of, cinv, rstart, efirst);
    return hipGetLastError();
}

hipError_t launch_bucket_records(const uint32_t* b, uint64_t P, uint64_t* rec, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(bucket_rec_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, b, P, rec);
    return hipGetLastError();
}

hipError_t launch_bucket_split(const uint64_t* rec, uint64_t P, uint32_t* b, uint32_t* ids, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(bucket_split_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, rec, P, b,
                       ids);
    return hipGetLastError();
}

uint64_t group_slot_count(uint64_t ntiles) { return ntiles * kSlots; }
uint64_t group_blocks(uint64_t ntiles, bool packed) { return packed ? ntiles * kGSplit : ntiles; }

template <int MG, typename View>
hipError_t launch_materialize(View v, const uint64_t* probe_info, uint64_t P, const GenomeTable& gt,
                              const MatchParams& mp, int L, int64_t* rows, hipStream_t st, uint64_t* lkey,
                              uint32_t* fsk, uint32_t* lhash, int32_t* rows32) {
    if (P == 0) return hipSuccess;
    if (RecIB<View>::value == 32 && gt.gl_n > 0)   // the coarse genome lookup (GenomeTable gl_*)
        hipLaunchKernelGGL((probe_materialize_kernel<MG, View, true>), dim3((unsigned)((P + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, v, probe_info, P, gt, mp, L, rows, lkey, fsk, lhash, rows32);
    else
        hipLaunchKernelGGL((probe_materialize_kernel<MG, View>), dim3((unsigned)((P + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, v, probe_info, P, gt, mp, L, rows, lkey, fsk, lhash, rows32);
    return hipGetLastError();
}

hipError_t launch_row_buckets(const int64_t* rows, uint64_t P, int G, uint32_t table_size, const uint32_t* d_bounds,
                              uint32_t nranks, uint32_t* out, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(row_bucket_kernel, dim3((unsigned)((P + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, rows, P, G,
                       table_size, 1.0 / (double)table_size, d_bounds, nranks, out);
    return hipGetLastError();
}

hipError_t launch_gather_rows(const int64_t* src, const uint32_t* perm, uint64_t P, int G, int64_t* dst,
                              hipStream_t st) {
    if (P == 0) return hipSuccess;
    const uint64_t n = P * (uint64_t)(G + 1);
    const uint64_t per = (uint64_t)kBlock * kGatherIPT;
    hipLaunchKernelGGL(gather_rows_ilp_kernel, dim3((unsigned)((n + per - 1) / per)), dim3(kBlock), 0, st, src, perm, n,
                       (uint32_t)(G + 1), dst);
    return hipGetLastError();
}

hipError_t launch_flat_tiles(uint64_t N, SegTile* d_tiles, hipStream_t st) {
    const uint64_t nt = (N + kGTile - 1) / kGTile;
    if (nt == 0) return hipSuccess;
    hipLaunchKernelGGL(flat_tiles_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, N, nt, d_tiles);
    return hipGetLastError();
}

template <int MG, typename View>
hipError_t launch_probe_tiles(View v, const SegTile* tiles, uint64_t ntiles, uint64_t N, const GenomeTable& gt,
                              const MatchParams& mp, int L, uint32_t* tile_count, uint64_t* slot_info,
                              uint32_t* slot_bucket, void* counters, hipStream_t st) {
    if (ntiles == 0) return hipSuccess;
    if constexpr (RecIB<View>::value > 0) {
        const bool fast = mp.repeat_tol == 0 && mp.enum_tol == 1;
        const double inv_t = 1.0 / (double)mp.table_size;
        if (RecIB<View>::value == 32 && gt.gl_n > 0 && fast && !getenv("MUMS_DEV_PROBE_GENERAL"))
            hipLaunchKernelGGL((probe_tile_rec_kernel<MG, RecIB<View>::value, true, true>),
                               dim3((unsigned)(ntiles * kGSplit)), dim3(kBlock), 0, st, v.rec, tiles, gt, mp, L,
                               tile_count, slot_info, slot_bucket, (DevCounters*)counters, inv_t);
        else if (RecIB<View>::value == 32 && gt.gl_n > 0)   // the coarse genome lookup (GenomeTable gl_*)
            hipLaunchKernelGGL((probe_tile_rec_kernel<MG, RecIB<View>::value, true>), dim3((unsigned)(ntiles * kGSplit)),
                               dim3(kBlock), 0, st, v.rec, tiles, gt, mp, L, tile_count, slot_info, slot_bucket,
                               (DevCounters*)counters, inv_t);
        else
            hipLaunchKernelGGL((probe_tile_rec_kernel<MG, RecIB<View>::value>), dim3((unsigned)(ntiles * kGSplit)),
                               dim3(kBlock), 0, st, v.rec, tiles, gt, mp, L, tile_count, slot_info, slot_bucket,
                               (DevCounters*)counters, inv_t);
    } else
        hipLaunchKernelGGL((probe_tile_kernel<MG, View>), dim3((unsigned)ntiles), dim3(kBlock), 0, st, v, tiles, N, gt,
                           mp, L, tile_count, slot_info, slot_bucket, (DevCounters*)counters);
    return hipGetLastError();
}

hipError_t launch_probe_compact(uint64_t nblocks, const uint32_t* tile_count, const uint32_t* tile_off,
                                const uint64_t* slot_info, const uint32_t* slot_bucket, uint64_t* probe_info,
                                uint32_t* probe_bucket, hipStream_t st, bool packed) {
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(probe_compact_kernel, dim3((unsigned)nblocks), dim3(kBlock), 0, st, tile_count, tile_off,
                       slot_info, slot_bucket, probe_info, probe_bucket, (uint32_t)(packed ? kSubSlots : kSlots));
    return hipGetLastError();
}

#define MUMS_INST_PROBE(MG, V)                                                                                     \
    template hipError_t launch_probe_tiles<MG, V>(V, const SegTile*, uint64_t, uint64_t, const GenomeTable&,      \
                                                  const MatchParams&, int, uint32_t*, uint64_t*, uint32_t*, void*, \
                                                  hipStream_t);
MUMS_INST_PROBE(4, PairView<uint32_t>)
MUMS_INST_PROBE(8, PairView<uint32_t>)
MUMS_INST_PROBE(16, PairView<uint32_t>)
MUMS_INST_PROBE(32, PairView<uint32_t>)
MUMS_INST_PROBE(64, PairView<uint32_t>)
MUMS_INST_PROBE(4, PairView<uint64_t>)
MUMS_INST_PROBE(8, PairView<uint64_t>)
MUMS_INST_PROBE(16, PairView<uint64_t>)
MUMS_INST_PROBE(32, PairView<uint64_t>)
MUMS_INST_PROBE(64, PairView<uint64_t>)
#define MUMS_INST_MAT(MG, V)                                                                                      \
    template hipError_t launch_materialize<MG, V>(V, const uint64_t*, uint64_t, const GenomeTable&,                \
                                                  const MatchParams&, int, int64_t*, hipStream_t, uint64_t*,      \
                                                  uint32_t*, uint32_t*, int32_t*);
MUMS_INST_MAT(4, PairView<uint32_t>)
MUMS_INST_MAT(8, PairView<uint32_t>)
MUMS_INST_MAT(16, PairView<uint32_t>)
MUMS_INST_MAT(32, PairView<uint32_t>)
MUMS_INST_MAT(64, PairView<uint32_t>)
MUMS_INST_MAT(4, PairView<uint64_t>)
MUMS_INST_MAT(8, PairView<uint64_t>)
MUMS_INST_MAT(16, PairView<uint64_t>)
MUMS_INST_MAT(32, PairView<uint64_t>)
MUMS_INST_MAT(64, PairView<uint64_t>)
MUMS_INST_MAT(4, RecView)
MUMS_INST_MAT(8, RecView)
MUMS_INST_MAT(16, RecView)
MUMS_INST_MAT(32, RecView)
MUMS_INST_MAT(64, RecView)
MUMS_INST_PROBE(4, RecView)
MUMS_INST_PROBE(8, RecView)
MUMS_INST_PROBE(16, RecView)
MUMS_INST_PROBE(32, RecView)
MUMS_INST_PROBE(64, RecView)
// chunked mode (> 2^32 seed-mers): 33-bit record indices
MUMS_INST_MAT(4, RecViewT<33>)
MUMS_INST_MAT(8, RecViewT<33>)
MUMS_INST_MAT(16, RecViewT<33>)
MUMS_INST_MAT(32, RecViewT<33>)
MUMS_INST_MAT(64, RecViewT<33>)
MUMS_INST_PROBE(4, RecViewT<33>)
MUMS_INST_PROBE(8, RecViewT<33>)
MUMS_INST_PROBE(16, RecViewT<33>)
MUMS_INST_PROBE(32, RecViewT<33>)
MUMS_INST_PROBE(64, RecViewT<33>)

}  // namespace mums
