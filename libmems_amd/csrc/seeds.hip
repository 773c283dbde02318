// seeds.hip -- ASCII -> 2-bit packed genome + canonical spaced-seed keys (rows A2-A4).
//
// Reference: translate32 (SortedMerList.cpp:425-460) packs 2 bits/base with the
// BasicDNATable (:29-47); GetSeedMer (:726-762) gathers the care bases of the
// pattern; RevCompMer (:597-614) + GetDnaSeedMer (:764-769) pick the smaller of
// the forward and reverse-complement seeds (reverse gets bit 0 set);
// FillDnaSeedSML (:771-783) does this for positions 0..n-L.
//
// MI355X mapping: one workgroup per 4096-position tile of one genome.
//   seed_pack_kernel   : the tile's ASCII (+L-1 halo) is read once with 16-B loads,
//                        2-bit packed in LDS (written out: the packed genome is the only
//                        copy of the sequence the later stages read), keys derived
//                        from LDS windows; then either the per-position key array
//                        (pair path) or a per-tile histogram of the top B key bits
//                        (packed path, MSD split of the sort).
//   seed_scatter_kernel: packed path, second pass: re-derives the keys from the packed
//                        words (0.25 B/base), ranks them stably by MSD bucket with
//                        wave64 ballot match-any, reorders through LDS and writes
//                        (ckey_low << 32 | index) records into their buckets.
// HBM bytes per seed-mer: pack 1 + 0.25 (packed path) ; scatter 0.25 + 8.
#include <cstdlib>
#include <type_traits>

#include "seed_device.h"

namespace mums {

namespace {

constexpr int kTile = kSeedTile;            // positions per workgroup
constexpr int kPerThread = kTile / kBlock;  // 16
constexpr int kHalo = 32;                   // >= L-1, rounded to 16
constexpr int kTileBytes = kTile + kHalo;
constexpr int kTileWords = kTileBytes / 16 + 3;
constexpr int kWaves = kBlock / 64;

struct AsciiPtrs { const char* p[kMaxG]; };

// MSD bits of the default split for a static pattern: 2w + 1 - 32 (0 when the key fits
// the record); the keys pass builds only this top digit
template <uint64_t PAT>
constexpr int kStaticMsd = PAT == 0 ? 0 : (2 * seed_runs(PAT).w + 1 > 32 ? 2 * seed_runs(PAT).w + 1 - 32 : 0);

// BasicDNATable (SortedMerList.cpp:29-47): c,b,y->1  g,s,k->2  t->3 (either case), else 0.
__device__ __forceinline__ uint32_t dna2(uint32_t c) {
    const uint32_t lc = c | 0x20u;
    const uint32_t one = (lc == 'c') | (lc == 'b') | (lc == 'y');
    const uint32_t two = (lc == 'g') | (lc == 's') | (lc == 'k');
    const uint32_t three = (lc == 't');
    return one | (two << 1) | (three * 3u);
}

__device__ __forceinline__ int tile_genome(const GenomeTable& gt, uint32_t t) {
    int g = 0;
    for (int k = 1; k < gt.G; ++k) g += (t >= gt.tfirst[k]) ? 1 : 0;
    return g;
}

template <int kMode, typename K, uint64_t PAT = 0>
__global__ __launch_bounds__(kBlock) void seed_pack_kernel(SeedSpec ss, GenomeTable gt, AsciiPtrs ap,
                                                           uint32_t* __restrict__ packed, K* __restrict__ ckey,
                                                           int msd_bits, uint32_t* __restrict__ hist, uint32_t T,
                                                           uint32_t* __restrict__ err, int swz) {
    __shared__ uint8_t bytes[kTileBytes + 16];
    __shared__ uint32_t words[kTileWords];
    __shared__ uint32_t bh[1 << kMaxMsdBits];
    // XCD-grouped tiles (as the scatter below): the digit-major histogram columns hist[i * T + t]
    // of neighbouring tiles share cache lines, which merge in one XCD's L2 instead of reaching
    // HBM as 4-B partial lines from eight L2s
    const uint32_t t = swz ? xcd_grouped_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const int g = tile_genome(gt, t);
    const uint32_t x = t - gt.tfirst[g];
    const uint64_t n = gt.n[g];
    const uint64_t m = gt.m[g];
    const uint64_t p0 = (uint64_t)x * kTile;
    const char* src = ap.p[g];
    const uint64_t avail = n - p0 < (uint64_t)kTileBytes ? n - p0 : (uint64_t)kTileBytes;
    const int tid = threadIdx.x;
    const int nb = kMode == 1 ? (1 << msd_bits) : 0;
    for (int i = tid; i < nb; i += kBlock) bh[i] = 0;

    // 1) stage the tile's ASCII in LDS (16-B loads when aligned)
    const bool aligned = (((uintptr_t)(src + p0)) & 15) == 0;
    if (aligned) {
        for (int c = tid; c * 16 < kTileBytes; c += kBlock) {
            const uint64_t off = (uint64_t)c * 16;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (off + 16 <= avail) {
                v = *reinterpret_cast<const uint4*>(src + p0 + off);
            } else if (off < avail) {
                uint32_t wv[4] = {0, 0, 0, 0};
                for (uint64_t k = 0; k < avail - off; ++k)
                    wv[k >> 2] |= (uint32_t)(uint8_t)src[p0 + off + k] << (8 * (k & 3));
                v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            }
            *reinterpret_cast<uint4*>(&bytes[off]) = v;
        }
    } else {
        for (int c = tid; c < kTileBytes; c += kBlock) bytes[c] = (uint64_t)c < avail ? (uint8_t)src[p0 + c] : 0;
    }
    __syncthreads();

    // 2) 2-bit pack 16 bases per word (MSB first, as translate32); detect '-'
    uint32_t bad = 0;
    for (int wi = tid; wi < kTileWords; wi += kBlock) {
        uint32_t word = 0;
        #pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = wi * 16 + k;
            const uint32_t c = b < kTileBytes ? bytes[b] : 0;
            bad |= (c == '-') && ((uint64_t)b < avail);
            word |= dna2(c) << (30 - 2 * k);
        }
        words[wi] = word;
    }
    if (bad) atomicOr(err, 1u);
    __syncthreads();
    {   // this tile's packed words (the last tile also writes the two pad words)
        const uint64_t pw = packed_words(n);
        uint32_t* out = packed + gt.woff[g];
        for (int k = tid; k < kTile / 16 + 2; k += kBlock) {
            const uint64_t wi = (uint64_t)x * (kTile / 16) + k;
            if ((k < kTile / 16 || p0 + kTile >= n) && wi < pw) out[wi] = words[k];
        }
    }

    // 3) keys
    if (kMode == 1 && nb <= 1) return;   // no MSD split: the scatter pass derives the keys
    const uint64_t base = gt.base[g];
    const int klow = 2 * ss.w + 1 - msd_bits;
    if constexpr (kMode == 1 && PAT != 0 && kStaticMsd<PAT> >= 1 && kStaticMsd<PAT> <= kMaxMsdBits) {
        // the default split: top digit only; keys wider than 32 + 8 bits split by their top
        // 8 bits first (msdsplit.hip)
        constexpr int kTop = kStaticMsd<PAT> > 8 ? 8 : kStaticMsd<PAT>;
        if (msd_bits == kTop) {
            #pragma unroll 4
            for (int j = 0; j < kPerThread; ++j) {
                const int q = tid + j * kBlock;
                const uint64_t p = p0 + (uint64_t)q;
                if (p >= m) break;
                const int wi = q >> 4, sh = 2 * (q & 15);
                const uint64_t hi = ((uint64_t)words[wi] << 32) | words[wi + 1];
                const uint64_t lo = words[wi + 2];
                atomicAdd(&bh[ckey_top_static<PAT, kTop>((hi << sh) | ((lo << sh) >> 32))], 1u);
            }
            __syncthreads();
            for (int i = tid; i < nb; i += kBlock) hist[(uint64_t)i * T + t] = bh[i];
            return;
        }
    }
    #pragma unroll 4
    for (int j = 0; j < kPerThread; ++j) {
        const int q = tid + j * kBlock;
        const uint64_t p = p0 + (uint64_t)q;
        if (p >= m) break;
        const int wi = q >> 4, sh = 2 * (q & 15);
        const uint64_t hi = ((uint64_t)words[wi] << 32) | words[wi + 1];
        const uint64_t lo = words[wi + 2];
        const uint64_t kv = ckey_of<PAT>((hi << sh) | ((lo << sh) >> 32), ss);
        if (kMode == 0) ckey[base + p] = (K)kv;
        else if (nb > 1) atomicAdd(&bh[(uint32_t)(kv >> klow)], 1u);
    }
    if (kMode == 1 && nb > 1) {
        __syncthreads();
        for (int i = tid; i < nb; i += kBlock) hist[(uint64_t)i * T + t] = bh[i];
    }
}

// Chunked mode (IB-bit record indices): kChunk keeps only the records whose MSD digit
// lies in [dlo, dlo + nbc) (hist = that digit range's scanned slice); with cbase != null
// every record is kept and lands at cbase[digit >> cbits_low] + its offset inside its
// chunk (hist = all slices, each scanned on its own: 32-bit offsets inside a chunk).
// four waves per SIMD for the <= 256-digit forms (the 2^11-digit development form
// cannot reach it: its LDS alone allows two blocks per CU)
#ifndef MUMS_SCATTER_SWZ
#define MUMS_SCATTER_SWZ 1
#endif
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
// kSide: the key has side_bits (<= 4) bits between the record's 64 - IB key bits and the
// msd_bits MSD digit; they go to side[] at the record's position (msdsplit.hip splits the
// buckets by them)
template <int kMaxDig, uint64_t PAT = 0, int IB = 32, bool kChunk = false, int kSide = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void seed_scatter_kernel(SeedSpec ss, GenomeTable gt,
                                                              const uint32_t* __restrict__ packed, int msd_bits,
                                                              const uint32_t* __restrict__ hist, uint32_t T,
                                                              uint64_t* __restrict__ rec, uint32_t dlo = 0,
                                                              uint32_t nbc = 0,
                                                              const uint64_t* __restrict__ cbase = nullptr,
                                                              int mb = 0, uint8_t* __restrict__ side = nullptr,
                                                              int side_bits = 0) {
    // LDS (<= 40 KB at kMaxDig 256, four blocks per CU): the packed words alias the
    // record staging area (read only before the records are placed), wave digit
    // offsets are 16-bit (<= kTile) and fold in the block-local digit starts, and gofs
    // folds in minus those starts (u32 arithmetic: the sum is < 2^32).
    using DigT = typename std::conditional<(kMaxDig <= 256 && kSide == 0), uint8_t, uint16_t>::type;
    __shared__ uint64_t srec[kTile];
    __shared__ DigT sdig[kTile];
    __shared__ uint16_t wcnt[kWaves][kMaxDig];
    __shared__ uint32_t gofs[kMaxDig];
    __shared__ uint32_t s_w[kWaves];
    __shared__ uint32_t s_kept;
    static_assert(kTileWords * 4 <= kTile * 8, "words alias srec");
    static_assert(kTile <= 65535, "16-bit wave digit offsets");
    static_assert(kSide == 0 || kTile <= 4096, "side digits sit in bits 28-31 above a 12-bit rank");
    uint32_t* words = reinterpret_cast<uint32_t*>(srec);
#if MUMS_SCATTER_SWZ
    // XCD-grouped tiles (a bijective blockIdx swizzle, cdna_hip_programming.md T1): blocks
    // b, b + 8, b + 16 ... share an XCD (round-robin dispatch, speed only) and take
    // consecutive seed tiles, so the digit runs consecutive tiles store into one MSD bucket
    // -- which abut in the output -- meet in that XCD's L2 and their partial lines merge
    const uint32_t t = xcd_grouped_block(blockIdx.x, gridDim.x);
#else
    const uint32_t t = blockIdx.x;
#endif
    const int g = tile_genome(gt, t);
    const uint32_t x = t - gt.tfirst[g];
    const uint64_t m = gt.m[g];
    const uint64_t p0 = (uint64_t)x * kTile;
    if (p0 >= m) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool all_chunks = kChunk && cbase != nullptr;
    const int nd = (kChunk && !all_chunks) ? (int)nbc : (1 << msd_bits);
    if (kChunk && tid == 0) s_kept = 0;
    const int klow = 2 * ss.w + 1 - msd_bits;
    const uint64_t lmask = (klow >= 64) ? ~0ull : ((1ull << klow) - 1);   // klow <= 64 - IB + kSide
    const uint64_t pw = packed_words(gt.n[g]);
    const uint32_t* W = packed + gt.woff[g];
    for (int k = tid; k < kTileWords; k += kBlock) {
        const uint64_t wi = (uint64_t)x * (kTile / 16) + k;
        words[k] = wi < pw ? W[wi] : 0u;
    }
    for (int i = tid; i < kWaves * kMaxDig; i += kBlock) (&wcnt[0][0])[i] = 0;
    __syncthreads();

    const uint64_t base = gt.base[g];
    const int q0 = wv * (kTile / kWaves);
    // the record's key part (<= 64 - IB <= 32 bits); its index part is base + p0 + q
    uint32_t r_key[kPerThread];
    uint32_t r_pk[kPerThread];   // wave rank << 16 | digit; ~0 = not stored
    #pragma unroll
    for (int r = 0; r < kPerThread; ++r) {
        const int q = q0 + r * 64 + lane;
        const uint64_t p = p0 + (uint64_t)q;
        bool valid = p < m;
        const int wi = q >> 4, sh = 2 * (q & 15);
        const uint64_t hi = ((uint64_t)words[wi] << 32) | words[wi + 1];
        const uint64_t lo = words[wi + 2];
        const uint64_t kv = ckey_of<PAT>((hi << sh) | ((lo << sh) >> 32), ss);
        uint32_t d = valid ? (uint32_t)(kv >> klow) : 0u;
        if (kChunk && !all_chunks) {
            d -= dlo;
            valid = valid && d < nbc;
            d = valid ? d : 0u;
        }
        r_key[r] = (uint32_t)(kv & lmask);   // the record keeps the low 64 - IB bits
        uint32_t tot;
        // digits are < 2^msd_bits <= kMaxDig: the unused high bits rank as equal
        const uint32_t rk = wave_match_rank<(kMaxDig > 256 ? kMaxMsdBits : 8)>(d, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][d];
        if (valid && rk == 0) wcnt[wv][d] = (uint16_t)(old + tot);
        r_pk[r] = valid ? (((old + rk) << 16) | d) : 0xFFFFFFFFu;
        if constexpr (kSide > 0)   // rank < 2^12: bits 28-31 are free (d < 256 here)
            if (valid) r_pk[r] |= ((uint32_t)(kv >> (64 - IB)) & ((1u << side_bits) - 1)) << 28;
    }
    __syncthreads();
    // per-digit wave offsets + block-local digit starts (each thread owns nd/256 digits)
    {
        constexpr int kPer = (kMaxDig + kBlock - 1) / kBlock;
        const int per = (nd + kBlock - 1) / kBlock;
        uint32_t dt[kPer];
        uint32_t tot_mine = 0;
        #pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int d = tid * per + k;
            dt[k] = 0;
            if (k >= per || d >= nd) continue;
            uint32_t acc = 0;
            #pragma unroll
            for (int w = 0; w < kWaves; ++w) { const uint32_t c = wcnt[w][d]; wcnt[w][d] = (uint16_t)acc; acc += c; }
            dt[k] = acc;
            tot_mine += acc;
        }
        if (kChunk && tot_mine) atomicAdd(&s_kept, tot_mine);
        uint32_t v = tot_mine;
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(v, dd, 64);
            if (lane >= dd) v += y;
        }
        if (lane == 63) s_w[wv] = v;
        __syncthreads();
        uint32_t pre = v - tot_mine;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) pre += (w < wv) ? s_w[w] : 0u;
        #pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int d = tid * per + k;
            if (k >= per || d >= nd) continue;
            #pragma unroll
            for (int w = 0; w < kWaves; ++w) wcnt[w][d] = (uint16_t)(wcnt[w][d] + pre);
            gofs[d] = hist[(uint64_t)d * T + t] - pre;
            pre += dt[k];
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kPerThread; ++r) {
        const uint32_t pk = r_pk[r];
        if (pk != 0xFFFFFFFFu) {
            const uint32_t d = pk & 0xFFFFu;
            const uint32_t lp = (uint32_t)wcnt[wv][d] + ((pk >> 16) & (kSide > 0 ? 0xFFFu : 0xFFFFu));
            srec[lp] = ((uint64_t)r_key[r] << IB) | (base + p0 + (uint64_t)(q0 + r * 64 + lane));
            sdig[lp] = (DigT)(kSide > 0 ? (d | ((pk >> 28) << 8)) : d);   // + the side digit
        }
    }
    __syncthreads();
    const uint64_t cnt = kChunk ? (uint64_t)s_kept : ((m - p0) < (uint64_t)kTile ? (m - p0) : (uint64_t)kTile);
    #pragma unroll
    for (int r = 0; r < kPerThread; ++r) {
        const uint32_t s = tid + r * kBlock;
        if (s < cnt) {
            const uint32_t dd = sdig[s];
            const uint32_t d = kSide > 0 ? (dd & 0xFFu) : dd;
            const uint64_t b = (kChunk && all_chunks) ? cbase[d >> mb] : 0ull;
            const uint64_t o = b + (uint64_t)(uint32_t)(gofs[d] + s);
            rec[o] = srec[s];
            if constexpr (kSide > 0) side[o] = (uint8_t)(dd >> 8);   // run order, like the records
        }
    }
}

#pragma clang diagnostic pop

// B == 0: one bucket, records land at their global index
template <uint64_t PAT = 0>
__global__ __launch_bounds__(kBlock) void seed_scatter_flat_kernel(SeedSpec ss, GenomeTable gt,
                                                                   const uint32_t* __restrict__ packed,
                                                                   uint64_t* __restrict__ rec) {
    __shared__ uint32_t words[kTileWords];
    const uint32_t t = blockIdx.x;
    const int g = tile_genome(gt, t);
    const uint32_t x = t - gt.tfirst[g];
    const uint64_t m = gt.m[g];
    const uint64_t p0 = (uint64_t)x * kTile;
    if (p0 >= m) return;
    const uint64_t pw = packed_words(gt.n[g]);
    const uint32_t* W = packed + gt.woff[g];
    for (int k = threadIdx.x; k < kTileWords; k += kBlock) {
        const uint64_t wi = (uint64_t)x * (kTile / 16) + k;
        words[k] = wi < pw ? W[wi] : 0u;
    }
    __syncthreads();
    const uint64_t base = gt.base[g];
    #pragma unroll 4
    for (int j = 0; j < kPerThread; ++j) {
        const int q = threadIdx.x + j * kBlock;
        const uint64_t p = p0 + (uint64_t)q;
        if (p >= m) break;
        const int wi = q >> 4, sh = 2 * (q & 15);
        const uint64_t hi = ((uint64_t)words[wi] << 32) | words[wi + 1];
        const uint64_t lo = words[wi + 2];
        const uint64_t kv = ckey_of<PAT>((hi << sh) | ((lo << sh) >> 32), ss);
        rec[base + p] = (kv << 32) | (base + p);
    }
}

__global__ void keys_of_genome_kernel(SeedSpec ss, const uint32_t* __restrict__ W, uint64_t m,
                                      uint64_t* __restrict__ out, int ref_form) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    const uint64_t k = ckey_at(W, p, ss);
    out[p] = ref_form ? (((k >> 1) << (64 - 2 * ss.w)) | (k & 1))   // GetDnaSeedMer's left-aligned form
                      : k;                                          // ckey = v << 1 | parity (same order)
}


// Patterns with compiled-in run tables: ranks 0-2 of getSeed(11..19) (SeedMasks.h; the
// default weights of genomes up to ~2 Gbp and ProgressiveAligner's seed families,
// ProgressiveAligner.cpp:619-625).  Any other pattern takes its run table from the kernel
// argument (SeedSpec); the output is the same.
#if MUMS_FEW_STATIC_SEEDS   // A/B build: only the BASELINE seeds compiled in
constexpr uint64_t kStaticSeeds[] = {kSeedW19, kSeedW15};
#else
constexpr uint64_t kStaticSeeds[] = {
    kSeedW21,                                             // w21 (3 Gbp genomes' default)
    kSeedW19, 0x7d6735full, 0x1edd74full,                 // w19
    0x3E6B59Full, 0x3EB335Full, 0x7B3566Full,             // w18
    0x6dbedbull,                                          // w17
    0xf599afull, 0xEE5A77ull, 0x7CD59Full,                // w16
    kSeedW15, 0x7b2a6full, 0x79aacfull,                   // w15
    0x1e6acfull, 0xF59AFull, 0x3D4CAFull,                 // w14
    0x792a4full, 0x1d64d7ull, 0x1d3597ull,                // w13
    0x7954full, 0x3D32Full, 0x768B7ull,                   // w12 (rank 0 = w11's)
    0x75257ull, 0x1c9527ull,                              // w11 ranks 1-2
};
#endif
constexpr int kNumStaticSeeds = (int)(sizeof(kStaticSeeds) / sizeof(kStaticSeeds[0]));

// calls f(std::integral_constant<uint64_t, PAT>) with PAT = pattern when it is compiled in,
// else PAT = 0 (run table from the argument)
template <int I = 0, class F>
void with_static_seed(uint64_t pattern, F&& f) {
    if constexpr (I == kNumStaticSeeds) {
        f(std::integral_constant<uint64_t, 0>{});
    } else {
        if (pattern == kStaticSeeds[I]) f(std::integral_constant<uint64_t, kStaticSeeds[I]>{});
        else with_static_seed<I + 1>(pattern, f);
    }
}

}  // namespace

hipError_t launch_seed_pack(const SeedSpec& ss, const GenomeTable& gt, const char* const* d_ascii,
                            uint32_t* d_packed, int mode, bool key64, void* d_ckey, int msd_bits,
                            uint32_t* d_hist, uint32_t ntiles, uint32_t* d_err, hipStream_t st) {
    AsciiPtrs ap{};
    for (int g = 0; g < gt.G; ++g) ap.p[g] = d_ascii[g];
    if (ntiles == 0) return hipSuccess;
    const int swz = getenv("MUMS_DEV_PACK_LINEAR") ? 0 : 1;   // (development A/B, read per call)
    if (mode == 0) {
        if (key64)
            hipLaunchKernelGGL((seed_pack_kernel<0, uint64_t>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt, ap,
                               d_packed, (uint64_t*)d_ckey, 0, d_hist, ntiles, d_err, swz);
        else
            hipLaunchKernelGGL((seed_pack_kernel<0, uint32_t>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt, ap,
                               d_packed, (uint32_t*)d_ckey, 0, d_hist, ntiles, d_err, swz);
    } else {
        with_static_seed(ss.pattern, [&](auto pc) {
            constexpr uint64_t PAT = decltype(pc)::value;
            hipLaunchKernelGGL((seed_pack_kernel<1, uint64_t, PAT>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt, ap,
                               d_packed, (uint64_t*)nullptr, msd_bits, d_hist, ntiles, d_err, swz);
        });
    }
    return hipGetLastError();
}

hipError_t launch_seed_scatter(const SeedSpec& ss, const GenomeTable& gt, const uint32_t* d_packed, int msd_bits,
                               const uint32_t* d_hist_scanned, uint32_t ntiles, uint64_t* d_rec, hipStream_t st,
                               uint8_t* d_side, int side_bits) {
    if (ntiles == 0) return hipSuccess;
    if (side_bits > 0) {   // 8 MSD bits + side_bits in side[] (msdsplit.hip)
        if (msd_bits != 8 || side_bits > 4 || 2 * ss.w + 1 != 32 + 8 + side_bits) return hipErrorInvalidValue;
        with_static_seed(ss.pattern, [&](auto pc) {
            constexpr uint64_t PAT = decltype(pc)::value;
            if constexpr (PAT == 0 || 2 * seed_runs(PAT).w + 1 > 40)
                hipLaunchKernelGGL((seed_scatter_kernel<256, PAT, 32, false, 1>), dim3(ntiles), dim3(kBlock), 0, st,
                                   ss, gt, d_packed, msd_bits, d_hist_scanned, ntiles, d_rec, 0u, 0u,
                                   (const uint64_t*)nullptr, 0, d_side, side_bits);
            else
                hipLaunchKernelGGL((seed_scatter_kernel<256, 0, 32, false, 1>), dim3(ntiles), dim3(kBlock), 0, st,
                                   ss, gt, d_packed, msd_bits, d_hist_scanned, ntiles, d_rec, 0u, 0u,
                                   (const uint64_t*)nullptr, 0, d_side, side_bits);
        });
        return hipGetLastError();
    }
    if (msd_bits > 8) {
        hipLaunchKernelGGL((seed_scatter_kernel<(1 << kMaxMsdBits), 0>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt,
                           d_packed, msd_bits, d_hist_scanned, ntiles, d_rec);
        return hipGetLastError();
    }
    with_static_seed(ss.pattern, [&](auto pc) {
        constexpr uint64_t PAT = decltype(pc)::value;
        if (msd_bits == 0)
            hipLaunchKernelGGL(seed_scatter_flat_kernel<PAT>, dim3(ntiles), dim3(kBlock), 0, st, ss, gt, d_packed,
                               d_rec);
        else
            hipLaunchKernelGGL((seed_scatter_kernel<256, PAT>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt, d_packed,
                               msd_bits, d_hist_scanned, ntiles, d_rec);
    });
    return hipGetLastError();
}

// chunked mode: records of MSD digits [dlo, dlo + nbc) only, 33-bit indices
// (requires 2w+1 - msd_bits == 31); hist_slice = the scanned histogram rows of those digits
hipError_t launch_seed_scatter_chunk(const SeedSpec& ss, const GenomeTable& gt, const uint32_t* d_packed, int msd_bits,
                                     const uint32_t* d_hist_slice, uint32_t ntiles, uint32_t dlo, uint32_t nbc,
                                     uint64_t* d_rec, hipStream_t st, const uint64_t* d_cbase, int mb, uint8_t* d_side,
                                     int side_bits) {
    if (ntiles == 0) return hipSuccess;
    if (side_bits > 0) {   // w20-21: 8 MSD bits + side_bits in side[] (msdsplit.hip), every chunk at once
        if (msd_bits != 8 || side_bits > 4 || 2 * ss.w + 1 != 31 + 8 + side_bits || !d_cbase)
            return hipErrorInvalidValue;
        const uint64_t pat = ss.pattern == kSeedW21 ? ss.pattern : 0;
        with_static_seed(pat, [&](auto pc) {
            constexpr uint64_t PAT = decltype(pc)::value;
            if constexpr (PAT == 0 || PAT == kSeedW21)
                hipLaunchKernelGGL((seed_scatter_kernel<256, PAT, 33, true, 1>), dim3(ntiles), dim3(kBlock), 0, st,
                                   ss, gt, d_packed, msd_bits, d_hist_slice, ntiles, d_rec, dlo, nbc, d_cbase, mb,
                                   d_side, side_bits);
        });
        return hipGetLastError();
    }
    if (2 * ss.w + 1 - msd_bits != 64 - 33 || msd_bits > 8 || (nbc == 0 && !d_cbase)) return hipErrorInvalidValue;
    // chunked contexts hold > 2^32 seed-mers: w 16-19 (compiled-in tables for the w19 seeds)
    const uint64_t pat = (ss.pattern == kSeedW19 || ss.pattern == 0x7d6735full || ss.pattern == 0x1edd74full)
                             ? ss.pattern : 0;
    with_static_seed(pat, [&](auto pc) {
        constexpr uint64_t PAT = decltype(pc)::value;
        if constexpr (PAT == 0 || seed_runs(PAT).w == 19)
            hipLaunchKernelGGL((seed_scatter_kernel<256, PAT, 33, true>), dim3(ntiles), dim3(kBlock), 0, st, ss, gt,
                               d_packed, msd_bits, d_hist_slice, ntiles, d_rec, dlo, nbc, d_cbase, mb);
    });
    return hipGetLastError();
}

hipError_t launch_keys_of_genome(const SeedSpec& ss, const uint32_t* d_words, uint64_t m, uint64_t* d_out,
                                 hipStream_t st, bool ref_form) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(keys_of_genome_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, ss, d_words, m,
                       d_out, ref_form ? 1 : 0);
    return hipGetLastError();
}

}  // namespace mums
