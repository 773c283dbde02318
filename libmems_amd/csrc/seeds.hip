// seeds.hip -- ASCII -> canonical spaced-seed keys, one pass over HBM (rows A2-A4).
//
// Reference: translate32 (SortedMerList.cpp:425-460) packs 2 bits/base with the
// BasicDNATable (:29-47); GetSeedMer (:726-762) gathers the care bases of the
// pattern; RevCompMer (:597-614) + GetDnaSeedMer (:764-769) pick the smaller of
// the forward and reverse-complement seeds (reverse gets bit 0 set);
// FillDnaSeedSML (:771-783) does this for positions 0..n-L.
//
// MI355X mapping: one workgroup per 4096-position tile of one genome.  The tile's
// ASCII (+L-1 halo) is read once with 16-B loads, 2-bit packed into LDS, and
// each lane derives 16 keys from LDS windows; key stores are lane-contiguous.
// HBM traffic per seed-mer: 1 B read + 4/8 B written.
#include "mums_internal.h"

namespace mums {

namespace {

constexpr int kTile = 4096;                 // positions per workgroup
constexpr int kPerThread = kTile / kBlock;  // 16
constexpr int kHalo = 32;                   // >= L-1, rounded to 16
constexpr int kTileBytes = kTile + kHalo;
constexpr int kTileWords = kTileBytes / 16 + 3;

struct AsciiPtrs { const char* p[kMaxG]; };

// BasicDNATable (SortedMerList.cpp:29-47): c,b,y->1  g,s,k->2  t->3 (either case), else 0.
__device__ __forceinline__ uint32_t dna2(uint32_t c) {
    uint32_t lc = c | 0x20u;
    uint32_t one = (lc == 'c') | (lc == 'b') | (lc == 'y');
    uint32_t two = (lc == 'g') | (lc == 's') | (lc == 'k');
    uint32_t three = (lc == 't');
    return one | (two << 1) | (three * 3u);
}

// reverse complement of a 2w-bit value (RevCompMer restated on bottom-aligned bits)
__device__ __forceinline__ uint64_t revcomp2w(uint64_t v, int w) {
    uint64_t x = ~v;
    x = __builtin_bitreverse64(x);
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    return x >> (64 - 2 * w);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void seed_keys_kernel(SeedSpec ss, GenomeTable gt, AsciiPtrs ap,
                                                           K* __restrict__ ckey, uint32_t* __restrict__ err) {
    __shared__ uint8_t bytes[kTileBytes + 16];
    __shared__ uint32_t words[kTileWords];
    const int g = blockIdx.y;
    const uint64_t n = gt.n[g];
    const uint64_t m = gt.m[g];
    const uint64_t p0 = (uint64_t)blockIdx.x * kTile;
    if (p0 >= n && !(p0 == 0 && n > 0)) return;
    const char* src = ap.p[g];
    const uint64_t avail = n - p0 < (uint64_t)kTileBytes ? n - p0 : (uint64_t)kTileBytes;
    const int tid = threadIdx.x;

    // 1) stage the tile's ASCII in LDS (16-B loads when aligned)
    uint32_t bad = 0;
    const bool aligned = (((uintptr_t)(src + p0)) & 15) == 0;
    if (aligned) {
        for (int c = tid; c * 16 < kTileBytes; c += kBlock) {
            uint64_t off = (uint64_t)c * 16;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (off + 16 <= avail) {
                v = *reinterpret_cast<const uint4*>(src + p0 + off);
            } else if (off < avail) {
                uint8_t tmp[16] = {0};
                for (uint64_t k = 0; k < avail - off; ++k) tmp[k] = (uint8_t)src[p0 + off + k];
                v = *reinterpret_cast<uint4*>(tmp);
            }
            *reinterpret_cast<uint4*>(&bytes[off]) = v;
        }
    } else {
        for (int c = tid; c < kTileBytes; c += kBlock)
            bytes[c] = (uint64_t)c < avail ? (uint8_t)src[p0 + c] : 0;
    }
    __syncthreads();

    // 2) 2-bit pack 16 bases per word (MSB first, as translate32); detect '-'
    for (int wi = tid; wi < kTileWords; wi += kBlock) {
        uint32_t word = 0;
        #pragma unroll
        for (int k = 0; k < 16; ++k) {
            int b = wi * 16 + k;
            uint32_t c = b < kTileBytes ? bytes[b] : 0;
            bad |= (c == '-') && ((uint64_t)b < avail);
            word |= dna2(c) << (30 - 2 * k);
        }
        words[wi] = word;
    }
    if (bad) atomicOr(err, 1u);
    __syncthreads();

    // 3) canonical key per position
    const uint64_t base = gt.base[g];
    const uint64_t vmask = (ss.w >= 32) ? ~0ull : ((1ull << (2 * ss.w)) - 1);
    #pragma unroll 4
    for (int j = 0; j < kPerThread; ++j) {
        const int q = tid + j * kBlock;
        const uint64_t p = p0 + (uint64_t)q;
        if (p >= m) break;
        const int wi = q >> 4, sh = 2 * (q & 15);
        uint64_t hi = ((uint64_t)words[wi] << 32) | words[wi + 1];
        uint64_t lo = words[wi + 2];
        uint64_t mer = (hi << sh) | ((lo << sh) >> 32);
        uint64_t v = 0;
        for (int r = 0; r < ss.nruns; ++r) {
            const int s = ss.run_start[r], l = ss.run_len[r];
            uint64_t bits = (mer >> (64 - 2 * (s + l))) & ((1ull << (2 * l)) - 1);
            v |= bits << ss.run_dst[r];
        }
        v &= vmask;
        const uint64_t rc = revcomp2w(v, ss.w);
        const uint64_t par = rc < v ? 1ull : 0ull;
        const uint64_t kv = ((par ? rc : v) << 1) | par;
        ckey[base + p] = (K)kv;
    }
}

}  // namespace

hipError_t launch_seed_keys(const SeedSpec& ss, const GenomeTable& gt, const char* const* d_ascii,
                            void* d_ckey, bool key64, uint32_t* d_err, hipStream_t st) {
    AsciiPtrs ap{};
    uint64_t maxn = 0;
    for (int g = 0; g < gt.G; ++g) {
        ap.p[g] = d_ascii[g];
        if (gt.n[g] > maxn) maxn = gt.n[g];
    }
    if (maxn == 0) return hipSuccess;
    dim3 grid((unsigned)((maxn + kTile - 1) / kTile), (unsigned)gt.G);
    if (key64)
        hipLaunchKernelGGL(seed_keys_kernel<uint64_t>, grid, dim3(kBlock), 0, st, ss, gt, ap,
                           (uint64_t*)d_ckey, d_err);
    else
        hipLaunchKernelGGL(seed_keys_kernel<uint32_t>, grid, dim3(kBlock), 0, st, ss, gt, ap,
                           (uint32_t*)d_ckey, d_err);
    return hipGetLastError();
}

}  // namespace mums
