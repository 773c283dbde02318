// chains.hip -- seed-chain labelling of every probe before the bucket replay (rows A9, A11).
//
// MatchFinder::ExtendMatch (MatchFinder.h:218-374) grows a probe to the maximal
// chain of seed hits with gaps <= L through the probe's column 0.
// That chain depends only on the probe's "line" -- its genome set, the strands
// (SetDirection, MemHash.cpp:189-203) and the diagonal of every component -- and on
// which hit columns the chain contains, so every probe of one chain extends to the
// SAME MatchHashEntry.  Instead of extending the first new probe of a chain inside
// the (sequential) per-bucket replay, all probes are labelled here in parallel:
//
//   1. chain_key_kernel   : line hash (32 b) | reference-genome start -> sort key
//   2. radix sort (64-bit) : probes of one line become adjacent, by position
//   3. chain_link_kernel  : neighbours on one line are in one chain iff a chain of
//                           hits (gaps <= L) joins them: gap <= L, else a walk of
//                           the hit columns between them; segment ends walk on to
//                           the chain's end (left walks in chain_left_kernel).  Walks
//                           test 64 columns per step with packed-word XORs (hit_word)
//   4. chain_walk_kernel  : walks longer than a per-lane budget, a group of 16 lanes each
//                           (one 64-column hit word per lane, break found by ballot)
//   5. chain_seg / chain_entry kernels: segment ids (scan), the extended entry of
//                           every chain and chain_of[probe].
// The replay (replay.hip) then inserts chain entries without extending anything.
// A line-hash collision whose two lines interleave in x order splits a chain into two
// segments with the same extended entry, and the replay then sees it twice: with a 16-bit
// hash the 4 x 10 Mbp related known answer gains 4 matches (MUMS_LINE_HASH_BITS A/B,
// round 4).  32 bits: only colliding multi-probe lines whose x ranges overlap do this --
// none in the test corpus or the C3 known answer; the residual risk is noted in DESIGN.md.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "match_device.h"
#include "seed_device.h"

namespace mums {

namespace {

#ifndef MUMS_WALK_BUDGET
#define MUMS_WALK_BUDGET 8
#endif
constexpr int kWalkBudget = MUMS_WALK_BUDGET;   // words per lane in chain_walk_short_kernel
#ifndef MUMS_WALK_SORT_SHIFT
#define MUMS_WALK_SORT_SHIFT 11
#endif
constexpr int kWalkSortShift = MUMS_WALK_SORT_SHIFT;   // walk order granule: 2^11 columns
#ifndef MUMS_WALK_SWZ
#define MUMS_WALK_SWZ 0   // 1: walk kernels in XCD-grouped block order (measured slower)
#endif
__device__ __forceinline__ unsigned walk_block() {
#if MUMS_WALK_SWZ
    return xcd_grouped_block(blockIdx.x, gridDim.x);
#else
    return blockIdx.x;
#endif
}
// waves per SIMD the walk kernels are compiled for (0: the compiler's choice, 3 at MG = 8 --
// ~150 VGPRs); more waves keep more of the walks' dependent loads in flight
#ifndef MUMS_WALK_WPE
#define MUMS_WALK_WPE 0
#endif
#if MUMS_WALK_WPE
#define MUMS_WALK_ATTR __attribute__((amdgpu_waves_per_eu(MUMS_WALK_WPE)))
#else
#define MUMS_WALK_ATTR
#endif
// the lean lane-group walks (chain_walk_kernel, kGen = false) at four waves per SIMD (<= 128 VGPRs:
// C3 long walks 5.8 -> 5.0 ms; the short walks spill at that target and stay at three);
// MUMS_WALK_LEAN_WPE=0: no target
#ifndef MUMS_WALK_LEAN_WPE
#define MUMS_WALK_LEAN_WPE 4
#endif
#if MUMS_WALK_LEAN_WPE
#define MUMS_WALK_LEAN_ATTR __attribute__((amdgpu_waves_per_eu(kGen ? 1 : MUMS_WALK_LEAN_WPE)))
#else
#define MUMS_WALK_LEAN_ATTR
#endif
#ifndef MUMS_HIT_VEC
#define MUMS_HIT_VEC 1   // hit_word's window loads as one 16-B + one 12-B load (0: one load per word)
#endif
#ifndef MUMS_HIT_BATCH
#define MUMS_HIT_BATCH 2   // components whose window loads are in flight together (hit_word; A/B round 4: 1 / 2 / 4 / 8)
#endif   // 64-column hit words per lane before a walk goes to a workgroup

struct WalkItem {
    uint32_t j;      // position in line order
    int32_t kind;    // 0: bridge j -> j+1, 1: right end, 2: left end
    int64_t cur;     // column reached so far (frame of probe ord[j])
    int64_t stop;    // bridge: done once cur >= stop
};


// probe of sorted-stream group k (the AddHashEntry argument), see build_probe
template <int MG, typename View>
__device__ __forceinline__ void probe_of(const View& v, const uint64_t* __restrict__ /*probe_info*/, uint32_t k,
                                         const GenomeTable& gt, const MatchParams& /*mp*/, int L, Mhe<MG>& P) {
    load_probe<MG>(v, k, gt.G, L, P);
}

template <int MG>
__device__ __forceinline__ bool same_line(const Mhe<MG>& a, const Mhe<MG>& b) {
    const int ra = first_start(a), rb = first_start(b);
    if (ra != rb) return false;
    const int64_t xa = start_at(a, ra), xb = start_at(b, rb);
    bool ok = true;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t sa = a.s[g], sb = b.s[g];
        const bool za = sa == 0, zb = sb == 0;
        ok = ok && (za == zb) && ((sa < 0) == (sb < 0));
        if (!za && !zb) {
            const int64_t da = sa > 0 ? sa - xa : -sa + xa;
            const int64_t db = sb > 0 ? sb - xb : -sb + xb;
            ok = ok && (da == db);
        }
    }
    return ok;
}

// column range where every component's seed window lies inside its sequence
template <int MG>
__device__ __forceinline__ void frame_bounds(const Mhe<MG>& P, const GenomeTable& gt, int64_t* clo, int64_t* chi) {
    int64_t lo = INT64_MIN, hi = INT64_MAX;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t s = P.s[g];
        if (g < gt.G && s != 0) {
            const int64_t m = (int64_t)gt.m[g];
            const int64_t l = s > 0 ? 1 - s : -s - m;
            const int64_t u = s > 0 ? m - s : -s - 1;
            lo = l > lo ? l : lo;
            hi = u < hi ? u : hi;
        }
    }
    *clo = lo;
    *chi = hi;
}

// seed hit at column c (MatchFinder.h:265-293): all present components have the same
// canonical seed and strand-relative parity there, all windows inside the sequences
template <int MG>
__device__ __forceinline__ bool hit_lane(int64_t c, const Mhe<MG>& P, const GenomeTable& gt, int64_t clo, int64_t chi,
                                         const uint32_t* __restrict__ packed, const SeedSpec& ss) {
    if (c < clo || c > chi) return false;
    bool first = true, ok = true;
    uint64_t v0 = 0;
    uint32_t o0 = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t s = P.s[g];
        if (ok && g < gt.G && s != 0) {
            const int64_t p = s > 0 ? s - 1 + c : -s - 1 - c;
            const uint64_t k = ckey_at(packed + gt.woff[g], (uint64_t)p, ss);
            const uint64_t v = k >> 1;
            const uint32_t o = s > 0 ? (uint32_t)((k & 1) ^ 1) : (uint32_t)(k & 1);
            if (first) { v0 = v; o0 = o; first = false; }
            else ok = (v == v0) && (o == o0);
        }
    }
    return ok;
}

// ---- bit-parallel hit words -----------------------------------------------------------
// For a palindromic care set (every rank-0 pattern of SeedMasks.h) the
// canonical-key test of hit_lane reduces to base comparisons along the line (A.9): a
// forward component hits at column c iff its care bases equal the reference's, a reverse
// component iff its reverse-complemented window's care bases do (and, for even w only,
// the window is not its own reverse complement: then both parities are 0 and the strand
// test of hit_lane fails).  So 64 columns are tested at once: per component the 96 bases
// under the 64 windows are XORed with the reference's (2 bits per base, reverse
// components reverse-complemented word-wise), OR-ed into one mismatch mask, and a column
// hits iff no care offset of its window sees a mismatch.

// 96 bases (3 x 32, first base in bits 63-62) from base position p of the genome at word
// gw of the packed array; words outside [0, nwords) read as 0 (masked by the caller)
__device__ __forceinline__ void bases96(const uint32_t* __restrict__ W, uint64_t nwords, uint64_t gw, int64_t p,
                                        uint64_t c[3]) {
    const int64_t wi = (int64_t)gw + (p >> 4);
    const int sh = 2 * (int)(p & 15);
    uint64_t w[7];
    #pragma unroll
    for (int i = 0; i < 7; ++i) {
        const int64_t k = wi + i;
        w[i] = (k >= 0 && (uint64_t)k < nwords) ? W[k] : 0u;
    }
    #pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t hi = (w[2 * k] << 32) | w[2 * k + 1];
        const uint64_t lo = w[2 * k + 2];
        c[k] = (hi << sh) | ((lo << sh) >> 32);
    }
}

// reverse complement of 32 packed bases
__device__ __forceinline__ uint64_t rc32(uint64_t x) {
    x = __builtin_bitreverse64(x);
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    return ~x;
}

// 2-bit XOR word of 32 bases -> 32-bit mismatch mask, base i at bit i
__device__ __forceinline__ uint32_t mism32(uint64_t x) {
    x = (x | (x >> 1)) & 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
    x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
    x = (x | (x >> 16)) & 0x00000000ffffffffull;
    return __builtin_bitreverse32((uint32_t)x);
}

struct LineSpec {
    uint64_t care;     // bit k: offset k of the window is a care position
    int L;
    int bitpar;        // 1: palindromic care set (hit words by base comparison)
    int even_w;        // even weight: self-reverse-complement windows need hit_lane
    uint64_t nwords;   // packed words (bounds of the loads)
};

__device__ __forceinline__ LineSpec line_spec(const SeedSpec& ss, const GenomeTable& gt) {
    LineSpec ls;
    const uint64_t pat = ss.pattern >> __builtin_ctzll(ss.pattern);
    const uint64_t rev = __builtin_bitreverse64(pat) >> (64 - ss.L);
    ls.care = rev;   // bit k <-> pattern bit L-1-k
    ls.L = ss.L;
    ls.bitpar = rev == pat;
    ls.even_w = !(ss.w & 1);
    ls.nwords = gt.woff[gt.G];
    return ls;
}

// 4 / 3 packed words at a dword-aligned address (global_load_dwordx4 / _dwordx3)
struct __attribute__((aligned(4))) Words4 { uint32_t x, y, z, w; };
struct __attribute__((aligned(4))) Words3 { uint32_t x, y, z; };

// hit bits of columns c0 .. c0+63 (bit i = column c0 + i) of the line of P.
// kGen = false: palindromic care set and odd weight only (every default seed, getSeed rank 0):
// the column-by-column canonical-key fallback and the self-reverse-complement test are not
// compiled in, so their registers do not weigh on the walks (the caller checks the seed)
template <int MG, bool kGen = true>
__device__ uint64_t hit_word(int64_t c0, const Mhe<MG>& P, const GenomeTable& gt, int64_t clo, int64_t chi,
                             const uint32_t* __restrict__ packed, const SeedSpec& ss, const LineSpec& ls) {
    if (c0 > chi || c0 + 63 < clo) return 0;
    uint64_t valid = ~0ull;
    if (c0 < clo) valid &= ~0ull << (clo - c0);
    if (c0 + 63 > chi) valid &= ~0ull >> (c0 + 63 - chi);
    const int ref = first_start(P);
    const int64_t sref = start_at(P, ref);
    if constexpr (kGen) {
        if (!ls.bitpar || sref <= 0) {   // generic: canonical keys column by column
            uint64_t h = 0;
            for (int i = 0; i < 64; ++i)
                if ((valid >> i) & 1) h |= (uint64_t)hit_lane<MG>(c0 + i, P, gt, clo, chi, packed, ss) << i;
            return h;
        }
    }
    // per batch of (up to) 8 components: every window load is issued before the first
    // use, so a word costs one memory round trip per batch, not one per genome
    uint64_t R[3] = {0, 0, 0};
    uint64_t acc0 = 0, acc1 = 0, acc2 = 0;
    bool rev = false;
    constexpr int kBatch = MG < MUMS_HIT_BATCH ? MG : MUMS_HIT_BATCH;
    // wide loads: a window's 7 words as one 16-B and one 12-B load (dword-aligned; the
    // walks' divergent loads are bound by vector memory instructions -- one address-unit pass
    // per cache line touched -- not by bytes); the edges of the packed array take the guarded
    // word loads
    const bool vec = MUMS_HIT_VEC != 0;
    #pragma unroll
    for (int g0 = 0; g0 < MG; g0 += kBatch) {
        uint32_t w[kBatch][7];
        int sh[kBatch];
        #pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int g = g0 + k;
            const int64_t s = P.s[g];
            sh[k] = 0;
            if (g < gt.G && s != 0) {
                const int64_t p = s > 0 ? s - 1 + c0 : -s + ls.L - 2 - c0 - 95;
                const int64_t wi = (int64_t)gt.woff[g] + (p >> 4);
                sh[k] = 2 * (int)(p & 15);
                if (vec && wi >= 0 && (uint64_t)wi + 7 <= ls.nwords) {
                    const Words4 a = *reinterpret_cast<const Words4*>(packed + wi);
                    const Words3 b = *reinterpret_cast<const Words3*>(packed + wi + 4);
                    w[k][0] = a.x;
                    w[k][1] = a.y;
                    w[k][2] = a.z;
                    w[k][3] = a.w;
                    w[k][4] = b.x;
                    w[k][5] = b.y;
                    w[k][6] = b.z;
                } else {
                    #pragma unroll
                    for (int i = 0; i < 7; ++i) {
                        const int64_t q = wi + i;
                        w[k][i] = (q >= 0 && (uint64_t)q < ls.nwords) ? packed[q] : 0u;
                    }
                }
            }
        }
        #pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int g = g0 + k;
            const int64_t s = P.s[g];
            if (!(g < gt.G && s != 0)) continue;
            uint64_t C[3];
            #pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint64_t hi = ((uint64_t)w[k][2 * j] << 32) | w[k][2 * j + 1];
                const uint64_t lo = w[k][2 * j + 2];
                C[j] = (hi << sh[k]) | ((lo << sh[k]) >> 32);
            }
            if (g == ref) {
                R[0] = C[0];
                R[1] = C[1];
                R[2] = C[2];
            } else if (s > 0) {
                acc0 |= R[0] ^ C[0];
                acc1 |= R[1] ^ C[1];
                acc2 |= R[2] ^ C[2];
            } else {   // column t <-> complement of base |s| + L - 2 - c0 - t
                acc0 |= R[0] ^ rc32(C[2]);
                acc1 |= R[1] ^ rc32(C[1]);
                acc2 |= R[2] ^ rc32(C[0]);
                rev = true;
            }
        }
    }
    const uint64_t lo = (uint64_t)mism32(acc0) | ((uint64_t)mism32(acc1) << 32);
    const uint64_t hi = mism32(acc2);
    uint64_t any = 0;
    for (uint64_t cm = ls.care; cm; cm &= cm - 1) {
        const int k = __builtin_ctzll(cm);
        any |= k ? ((lo >> k) | (hi << (64 - k))) : lo;
    }
    uint64_t h = ~any & valid;
    if constexpr (kGen) {
        if (rev && ls.even_w) {   // drop self-reverse-complement windows (exact test)
            for (uint64_t t = h; t; t &= t - 1) {
                const int i = __builtin_ctzll(t);
                if (!hit_lane<MG>(c0 + i, P, gt, clo, chi, packed, ss)) h &= ~(1ull << i);
            }
        }
    }
    return h;
}

// 64 hit bits in walk order: bit i = column from + dir * i
template <int MG, bool kGen = true>
__device__ __forceinline__ uint64_t hit_word_dir(int dir, int64_t from, const Mhe<MG>& P, const GenomeTable& gt,
                                                 int64_t clo, int64_t chi, const uint32_t* __restrict__ packed,
                                                 const SeedSpec& ss, const LineSpec& ls) {
    if (dir > 0) return hit_word<MG, kGen>(from, P, gt, clo, chi, packed, ss, ls);
    return __builtin_bitreverse64(hit_word<MG, kGen>(from - 63, P, gt, clo, chi, packed, ss, ls));
}

// One 64-column word of a chain walk.  Walk offsets u >= 0 (column = start + dir * u);
// *last = offset of the last chain hit so far, the word covers offsets u0 .. u0+63.
// Returns true when the chain ends (L consecutive misses after *last),
// with *last its final hit; else *last = the word's last hit.
__device__ __forceinline__ bool scan_word(uint64_t H, int64_t u0, int64_t* last, int L) {
    const int64_t gap = u0 - *last - 1;   // misses since the last hit
    if (H == 0) return true;             // 64 >= L misses
    const int f = __builtin_ctzll(H);
    if (gap + f >= L) return true;
    // bit i of a: offsets i .. i+L-1 of this word all miss (runs into the next word are
    // found there through gap)
    uint64_t a = ~H;
    int len = 1;
    while (2 * len <= L) { a &= a >> len; len *= 2; }
    if (len < L) a &= a >> (L - len);
    if (a) {
        const int r0 = __builtin_ctzll(a);   // > f: a run needs L misses, f < L
        const uint64_t below = H & ((1ull << r0) - 1);
        *last = u0 + (63 - __builtin_clzll(below));
        return true;
    }
    *last = u0 + (63 - __builtin_clzll(H));
    return false;
}

// Chain walk from hit column cur in direction dir, one word (64 columns) per step.
// state 0: the chain ends at the returned column; 1: the chain reaches `stop` (returned:
// a chain hit at or past it); 2: budget spent (returned: the last hit reached).
template <int MG, bool kGen = true>
__device__ int64_t walk_lane(int dir, int64_t cur, int64_t stop, int budget, const Mhe<MG>& P, const GenomeTable& gt,
                             int64_t clo, int64_t chi, const uint32_t* __restrict__ packed, const SeedSpec& ss,
                             const LineSpec& ls, int* state, unsigned* words) {
    int64_t last = 0, u0 = 1;
    for (;;) {
        const int64_t col = cur + dir * last;
        if (dir > 0 ? col >= stop : col <= stop) { *state = 1; return col; }
        if (budget-- <= 0) { *state = 2; return col; }
        ++*words;
        const uint64_t H = hit_word_dir<MG, kGen>(dir, cur + dir * u0, P, gt, clo, chi, packed, ss, ls);
        const bool broke = scan_word(H, u0, &last, ls.L);
        u0 += 64;
        if (broke) {
            const int64_t c = cur + dir * last;
            *state = (dir > 0 ? c >= stop : c <= stop) ? 1 : 0;
            return c;
        }
    }
}

// ---- kernels ------------------------------------------------------------------------

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_key_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                           GenomeTable gt, MatchParams mp, int L,
                                                           uint64_t* __restrict__ lkey, uint32_t* __restrict__ lhash) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    Mhe<MG> Q;
    probe_of<MG, View>(v, probe_info, (uint32_t)k, gt, mp, L, Q);
    const int ref = first_start(Q);
    const uint64_t x = (uint64_t)start_at(Q, ref);
    if (lhash) {   // line_sort's first records and the hashes apart (chain_line_slots)
        lkey[k] = (x << 32) | k;
        lhash[k] = line_hash<MG>(Q, gt.G);
    } else {
        lkey[k] = ((uint64_t)line_hash<MG>(Q, gt.G) << 32) | (x & 0xFFFFFFFFull);
    }
}

constexpr uint64_t kCollideScan = 4096;   // probes scanned after a line-hash collision

// Block-wide append of the items whose want bit is set (kIPT per thread): one atomic per
// workgroup -- a single queue counter hit by every wave serialises in the L2 atomic unit.
constexpr int kLinkIPT = 8;

template <int kIPT>
__device__ __forceinline__ void block_push(uint32_t want, const WalkItem (&it)[kIPT], WalkItem* __restrict__ queue,
                                           unsigned int* __restrict__ qcount) {
    __shared__ uint32_t s_w[kBlock / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t n = (uint32_t)__builtin_popcount(want);
    uint32_t x = n;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    __syncthreads();   // s_w may still be read by the previous call's threads
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const uint32_t c = s_w[w];
            s_w[w] = tot;
            tot += c;
        }
        s_w[kBlock / 64] = tot ? atomicAdd(qcount, tot) : 0u;
    }
    __syncthreads();
    uint32_t o = s_w[kBlock / 64] + s_w[wv] + x - n;
    #pragma unroll
    for (int i = 0; i < kIPT; ++i)
        if ((want >> i) & 1u) queue[o++] = it[i];
}

// Neighbours in line order: same line and gap <= L -> linked without a walk; every other
// probe queues a walk (bridge to the next probe, or its chain's right end).  The walks run
// compacted in chain_walk_short_kernel (no lane of a wave idles behind them).
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_link_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                            GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                            uint8_t* __restrict__ link, WalkItem* __restrict__ queue,
                                                            unsigned int* __restrict__ qcount,
                                                            unsigned int* __restrict__ collide,
                                                            uint32_t* __restrict__ fsl) {
    const int L = ss.L;
    uint32_t want = 0, cbits = 0;
    WalkItem it[kLinkIPT];
    #pragma unroll
    for (int i = 0; i < kLinkIPT; ++i) {
        const uint64_t j = (uint64_t)blockIdx.x * (kBlock * kLinkIPT) + (uint64_t)i * kBlock + threadIdx.x;
        it[i] = WalkItem{(uint32_t)j, 1, 0, INT64_MAX};
        // probe j + 1 is the next lane's probe j: taken by a shuffle (one row load per probe,
        // the rows may be random reads through the line order), loaded only by a wave's last lane
        Mhe<MG> A, B;
        if (j < P) probe_of<MG, View>(v, probe_info, j, gt, mp, L, A);
        else A = Mhe<MG>{};
        B.len = __shfl_down(A.len, 1, 64);
        B.offset = __shfl_down(A.offset, 1, 64);
        B.mersize = __shfl_down(A.mersize, 1, 64);
        #pragma unroll
        for (int g = 0; g < MG; ++g) B.s[g] = __shfl_down(A.s[g], 1, 64);
        if (j >= P) continue;
        if ((threadIdx.x & 63) == 63 && j + 1 < P) probe_of<MG, View>(v, probe_info, j + 1, gt, mp, L, B);
        if (fsl) fsl[j] = (uint32_t)start_at(A, first_start(A));
        bool same = false;
        if (j + 1 < P) same = same_line<MG>(A, B);
        uint8_t lk = 0;
        if (same) {
            const int64_t stop = start_at(B, first_start(B)) - start_at(A, first_start(A)) - L;
            if (stop <= 0) lk = 1;
            else { it[i].kind = 0; it[i].stop = stop; want |= 1u << i; }
        } else {
            want |= 1u << i;
            // a different line with the same line hash (checked below)
            if (collide && j + 1 < P && line_hash<MG>(A, gt.G) == line_hash<MG>(B, gt.G)) cbits |= 1u << i;
        }
        link[j] = lk;
    }
    // a later probe of A's line inside the equal-hash run means two lines interleave (a chain
    // would split in two segments); looked for over kCollideScan probes, a longer run counts
    // as interleaved -- the caller then orders the lines exactly
    while (cbits) {
        const int i = __builtin_ctz(cbits);
        cbits &= cbits - 1;
        const uint64_t j = (uint64_t)blockIdx.x * (kBlock * kLinkIPT) + (uint64_t)i * kBlock + threadIdx.x;
        Mhe<MG> A;
        probe_of<MG, View>(v, probe_info, j, gt, mp, L, A);
        const uint32_t hA = line_hash<MG>(A, gt.G);
        bool hit = j + 2 < P;
        for (uint64_t q = j + 2; q < P && q < j + 2 + kCollideScan; ++q) {
            Mhe<MG> Q;
            probe_of<MG, View>(v, probe_info, q, gt, mp, L, Q);
            if (line_hash<MG>(Q, gt.G) != hA) { hit = false; break; }
            if (same_line<MG>(A, Q)) break;
            if (q + 1 == P) hit = false;
        }
        if (hit) atomicOr(collide, 1u);
    }
    block_push<kLinkIPT>(want, it, queue, qcount);
}

// segment starts (first probe, or the previous probe not linked) walk left to the chain start;
// seg[j] = 1 at segment starts (scanned to segment ids after the walks: the links are final
// after pass 0, the left walks only find where each chain begins)
__global__ __launch_bounds__(kBlock) void chain_left_kernel(uint64_t P, const uint8_t* __restrict__ link,
                                                            WalkItem* __restrict__ queue,
                                                            unsigned int* __restrict__ qcount,
                                                            uint32_t* __restrict__ seg) {
    uint32_t want = 0;
    WalkItem it[kLinkIPT];
    #pragma unroll
    for (int i = 0; i < kLinkIPT; ++i) {
        const uint64_t j = (uint64_t)blockIdx.x * (kBlock * kLinkIPT) + (uint64_t)i * kBlock + threadIdx.x;
        it[i] = WalkItem{(uint32_t)j, 2, 0, INT64_MIN};
        if (j < P) {
            const bool start = j == 0 || !link[j - 1];
            seg[j] = start ? 1u : 0u;
            if (start) want |= 1u << i;
        }
    }
    block_push<kLinkIPT>(want, it, queue, qcount);
}

// Walk order by genome position: record (x >> shift) << 32 | q of queue item q, x = the
// first start of its probe.  A walk reads the packed windows of every component around its
// probe -- about one 128-B line per genome per walk, lines that the walks of nearby probes
// (other lines of the same region: the partial tuples around a substitution, the next chain
// of the diagonal) read too.  In line order those walks are far apart in time and each line
// is fetched again from HBM; sorted by position they run close together and share L2.
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void walk_key_kernel(View v, GenomeTable gt, MatchParams mp, int L,
                                                          const WalkItem* __restrict__ queue,
                                                          const unsigned int* __restrict__ qcount, int shift,
                                                          uint64_t* __restrict__ rec) {
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= *qcount) return;
    Mhe<MG> A;
    probe_of<MG, View>(v, nullptr, queue[q].j, gt, mp, L, A);
    const int64_t x = start_at(A, first_start(A));
    rec[q] = ((uint64_t)(x > 0 ? x : 0) >> shift << 32) | q;
}

// records (j << 32 | i) of the handed-on walks: their line order back (MUMS_DEV_WALK_SORT=2)
__global__ __launch_bounds__(kBlock) void walk_line_key_kernel(const WalkItem* __restrict__ lq,
                                                               const unsigned int* __restrict__ lqcount,
                                                               uint64_t* __restrict__ rec) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= *lqcount) return;
    rec[i] = ((uint64_t)lq[i].j << 32) | i;
}

// Queued walks, one lane per item, up to kWalkBudget 64-column words each (most chain ends
// lie within a few words); the rest go on to chain_walk_kernel's lane groups.
template <int MG, typename View, bool kGen = true>
__global__ __launch_bounds__(kBlock) MUMS_WALK_ATTR void chain_walk_short_kernel(View v, const uint64_t* __restrict__ probe_info,
                                                                  GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                                  const uint32_t* __restrict__ packed,
                                                                  const WalkItem* __restrict__ queue,
                                                                  const unsigned int* __restrict__ qcount,
                                                                  uint8_t* __restrict__ link, int64_t* __restrict__ rcol,
                                                                  int64_t* __restrict__ lcol, WalkItem* __restrict__ lq,
                                                                  unsigned int* __restrict__ lqcount,
                                                                  const uint64_t* __restrict__ order,
                                                                  DevCounters* __restrict__ ctr) {
    const int L = ss.L;
    const LineSpec ls = line_spec(ss, gt);
    const unsigned nq = *qcount;
    const unsigned stride = gridDim.x * kBlock;
    uint32_t my_words = 0, my_items = 0, my_wins = 0;   // (a lane's walks: a few, <= kWalkBudget words each)
    // block-uniform trip count: block_push synchronises the workgroup
    for (unsigned q0 = walk_block() * kBlock; q0 < nq; q0 += stride) {
        const unsigned q = q0 + threadIdx.x;
        uint32_t want = 0;
        WalkItem nx[1] = {WalkItem{}};
        if (q < nq) {
            const WalkItem it = queue[order ? (uint32_t)order[q] : q];
            Mhe<MG> A;
            probe_of<MG, View>(v, probe_info, it.j, gt, mp, L, A);
            const int64_t xa = start_at(A, first_start(A));
            int64_t clo, chi;
            frame_bounds<MG>(A, gt, &clo, &chi);
            const int dir = it.kind == 2 ? -1 : +1;
            int state;
            unsigned nw = 0;
            const int64_t c = walk_lane<MG, kGen>(dir, it.cur, it.stop, kWalkBudget, A, gt, clo, chi, packed, ss, ls, &state,
                                            &nw);
            int npres = 0;
            #pragma unroll
            for (int g = 0; g < MG; ++g) npres += (g < gt.G && A.s[g] != 0) ? 1 : 0;
            my_words += nw;
            my_wins += nw * (uint32_t)npres;
            ++my_items;
            if (state == 2) {
                nx[0] = WalkItem{it.j, it.kind, c, it.stop};
                want = 1;
            } else if (it.kind == 0) {
                link[it.j] = state == 1 ? 1 : 0;
                if (state == 0) rcol[it.j] = xa + c;
            } else if (it.kind == 1) {
                rcol[it.j] = xa + c;
            } else {
                lcol[it.j] = xa + c;
            }
        }
        block_push<1>(want, nx, lq, lqcount);
    }
    if (ctr) {   // words / walks of this wave (the roofline's byte count): one atomic per wave
        #pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            my_words += __shfl_xor(my_words, d, 64);
            my_items += __shfl_xor(my_items, d, 64);
            my_wins += __shfl_xor(my_wins, d, 64);
        }
        if ((threadIdx.x & 63) == 0 && my_items) {
            atomicAdd(&ctr->short_words, (unsigned long long)my_words);
            atomicAdd(&ctr->short_items, (unsigned long long)my_items);
            atomicAdd(&ctr->short_wins, (unsigned long long)my_wins);
        }
    }
}

// chain_walk_short_kernel with lane refill.  Walk lengths are heavy-tailed (about one item
// in five spends the whole budget), so a wave of 64 one-shot lanes nearly always runs
// kWalkBudget steps for items that mostly end after one or two words.  Here each block owns
// a contiguous range of the queue, a lane whose walk has ended takes the next item of that
// range (LDS counter, once kRefillMin lanes of the wave are idle) and every step advances
// each busy lane by one word.  Results per item are the same as chain_walk_short_kernel's
// (same walk, same budget); the handed-on items reach lq in another order, which no later
// step depends on.
#ifndef MUMS_WALK_REFILL_MIN
#define MUMS_WALK_REFILL_MIN 16
#endif
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_walk_refill_kernel(View v, GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                                   const uint32_t* __restrict__ packed,
                                                                   const WalkItem* __restrict__ queue,
                                                                   const unsigned int* __restrict__ qcount,
                                                                   uint8_t* __restrict__ link, int64_t* __restrict__ rcol,
                                                                   int64_t* __restrict__ lcol, WalkItem* __restrict__ lq,
                                                                   unsigned int* __restrict__ lqcount) {
    const int L = ss.L;
    const LineSpec ls = line_spec(ss, gt);
    const unsigned nq = *qcount;
    const unsigned per = (nq + gridDim.x - 1) / gridDim.x;
    const unsigned lo = min(nq, blockIdx.x * per), hi = min(nq, lo + per);
    __shared__ unsigned s_next;
    if (threadIdx.x == 0) s_next = lo;
    __syncthreads();
    if (lo >= hi) return;
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    bool have = false, more = true;   // more: wave-uniform
    WalkItem it{};
    Mhe<MG> A;
    int64_t xa = 0, clo = 0, chi = 0, last = 0, u0 = 1;
    int budget = 0, dir = 1;
    for (;;) {
        const uint64_t idle = __ballot(!have);
        const unsigned n = (unsigned)__popcll(idle);
        if (more && n >= (unsigned)MUMS_WALK_REFILL_MIN) {
            const int lead = __builtin_ctzll(idle);
            unsigned base = 0;
            if (lane == lead) base = atomicAdd(&s_next, n);
            base = __shfl(base, lead);
            if (base + n >= hi) more = false;
            if (!have) {
                const unsigned q = base + (unsigned)__popcll(idle & below);
                if (q < hi) {
                    it = queue[q];
                    probe_of<MG, View>(v, nullptr, it.j, gt, mp, L, A);
                    xa = start_at(A, first_start(A));
                    frame_bounds<MG>(A, gt, &clo, &chi);
                    dir = it.kind == 2 ? -1 : +1;
                    last = 0;
                    u0 = 1;
                    budget = kWalkBudget;
                    have = true;
                }
            }
        }
        if (!__any(have)) {
            if (!more) break;
            continue;
        }
        bool hand_on = false;
        if (have) {   // one step of walk_lane
            const int64_t col = it.cur + dir * last;
            int state = -1;
            int64_t c = col;
            if (dir > 0 ? col >= it.stop : col <= it.stop) state = 1;
            else if (budget-- <= 0) state = 2;
            else {
                const uint64_t H = hit_word_dir<MG>(dir, it.cur + dir * u0, A, gt, clo, chi, packed, ss, ls);
                const bool broke = scan_word(H, u0, &last, L);
                u0 += 64;
                if (broke) {
                    c = it.cur + dir * last;
                    state = (dir > 0 ? c >= it.stop : c <= it.stop) ? 1 : 0;
                }
            }
            if (state >= 0) {
                have = false;
                if (state == 2) {
                    hand_on = true;
                    it.cur = c;
                } else if (it.kind == 0) {
                    link[it.j] = state == 1 ? 1 : 0;
                    if (state == 0) rcol[it.j] = xa + c;
                } else if (it.kind == 1) {
                    rcol[it.j] = xa + c;
                } else {
                    lcol[it.j] = xa + c;
                }
            }
        }
        const uint64_t hm = __ballot(hand_on);
        if (hm) {   // wave-aggregated append to the long-walk queue
            const int lead = __builtin_ctzll(hm);
            unsigned base = 0;
            if (lane == lead) base = atomicAdd(lqcount, (unsigned)__popcll(hm));
            base = __shfl(base, lead);
            if (hand_on) lq[base + (unsigned)__popcll(hm & below)] = it;
        }
    }
}

// Long walks, one group of kWalkGroup lanes per item (grid-stride over the queue; a wave
// walks 64 / kWalkGroup items at once: most queued walks end within a few words, so more
// items in flight hide more load latency than wider steps would).  Each step evaluates the
// kWalkGroup words (64 columns each) after the chain's last hit, one word per lane; the
// chain ends at the first lane whose word holds a run of L misses after a hit, or whose
// first hit lies L or more columns after the previous lane's last hit (the
// maximal chain of hits with gaps <= L).  A ballot finds that lane, shuffles inside the
// group fetch the last hit before the break.
#ifndef MUMS_WALK_GROUP
#define MUMS_WALK_GROUP 16
#endif
constexpr int kWalkGroup = MUMS_WALK_GROUP;
#ifndef MUMS_WALK_HANDOFF
#define MUMS_WALK_HANDOFF 16   // steps of a kWalkGroup-lane walk before it goes to a whole wave (0: never)
#endif
constexpr unsigned kWalkHandoff = MUMS_WALK_HANDOFF;

// maxsteps > 0: a walk still going after maxsteps steps is handed on (from its last hit) to
// xq for the next launch with wider groups -- the few walks of hundreds of steps otherwise
// set the kernel's duration one step at a time.
template <int MG, typename View, int GS, bool kGen = true>
__global__ __launch_bounds__(kBlock) MUMS_WALK_ATTR MUMS_WALK_LEAN_ATTR void chain_walk_kernel(View v, const uint64_t* __restrict__ probe_info,
                                                            GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                            const uint32_t* __restrict__ ord,
                                                            const uint32_t* __restrict__ packed,
                                                            const WalkItem* __restrict__ queue,
                                                            const unsigned int* __restrict__ qcount,
                                                            uint8_t* __restrict__ link, int64_t* __restrict__ rcol,
                                                            int64_t* __restrict__ lcol, unsigned int* __restrict__ dbg,
                                                            DevCounters* __restrict__ ctr, unsigned maxsteps,
                                                            WalkItem* __restrict__ xq, unsigned int* __restrict__ xqcount,
                                                            const uint64_t* __restrict__ order) {
    static_assert(GS >= 2 && GS <= 64 && (GS & (GS - 1)) == 0, "group: power of 2");
    unsigned long long my_words = 0, my_items = 0, my_wins = 0;
    const int lane = threadIdx.x & 63, gl = lane & (GS - 1), gsh = lane & ~(GS - 1);
    const uint64_t gmask = GS == 64 ? ~0ull : ((1ull << GS) - 1);
    const int L = ss.L;
    const LineSpec ls = line_spec(ss, gt);
    const unsigned nq = *qcount;
    const unsigned ngroups = gridDim.x * (kBlock / GS);
    for (unsigned qi = (walk_block() * kBlock + threadIdx.x) / GS; qi < nq; qi += ngroups) {
        const WalkItem it = queue[order ? (uint32_t)order[qi] : qi];
        Mhe<MG> A;
        probe_of<MG, View>(v, probe_info, it.j, gt, mp, L, A);
        const int64_t xa = start_at(A, first_start(A));
        int64_t clo, chi;
        frame_bounds<MG>(A, gt, &clo, &chi);
        const int dir = it.kind == 2 ? -1 : +1;
        const int64_t cur = it.cur;   // walk offsets u from here: column = cur + dir * u
        const int64_t stopu = dir > 0 ? (it.stop == INT64_MAX ? INT64_MAX : it.stop - cur)
                                      : (it.stop == INT64_MIN ? INT64_MAX : cur - it.stop);
        int64_t last = 0, u0 = 1;
        bool reached = last >= stopu;
        bool handed = false;
        unsigned steps = 0;
        while (!reached) {
            if (maxsteps && steps == maxsteps) {   // uniform in the group
                if (gl == 0) xq[atomicAdd(xqcount, 1u)] = WalkItem{it.j, it.kind, cur + dir * last, it.stop};
                handed = true;
                break;
            }
            ++steps;
            const uint64_t H = hit_word_dir<MG, kGen>(dir, cur + dir * (u0 + 64 * (int64_t)gl), A, gt, clo, chi, packed,
                                                ss, ls);
            const int f = H ? __builtin_ctzll(H) : 64;
            const int hb = H ? 63 - __builtin_clzll(H) : -1;
            int rend = -1;   // last hit before a run of L misses inside the word
            if (H) {
                uint64_t a = ~H;
                int len = 1;
                while (2 * len <= L) { a &= a >> len; len *= 2; }
                if (len < L) a &= a >> (L - len);
                if (a) rend = 63 - __builtin_clzll(H & ((1ull << __builtin_ctzll(a)) - 1));
            }
            const int prev_hb = __shfl_up(hb, 1, GS);
            const int64_t miss = gl == 0 ? (u0 - last - 1) + f : (int64_t)(63 - prev_hb) + f;
            const bool brk_in = H == 0 || miss >= L;
            const uint64_t bm = (__ballot(brk_in || rend >= 0) >> gsh) & gmask;
            if (bm) {
                const int k = __builtin_ctzll(bm);
                const int kin = __shfl(brk_in ? 1 : 0, k, GS);
                const int hprev = __shfl(hb, k > 0 ? k - 1 : 0, GS);
                const int rk = __shfl(rend, k, GS);
                if (kin) last = k == 0 ? last : u0 + 64 * (int64_t)(k - 1) + hprev;
                else last = u0 + 64 * (int64_t)k + rk;
                reached = last >= stopu;
                break;
            }
            last = u0 + 64 * (GS - 1) + __shfl(hb, GS - 1, GS);
            u0 += 64 * GS;
            reached = last >= stopu;
        }
        my_words += (unsigned long long)steps * GS;
        ++my_items;
        int npres = 0;
        #pragma unroll
        for (int g = 0; g < MG; ++g) npres += (g < gt.G && A.s[g] != 0) ? 1 : 0;
        my_wins += (unsigned long long)steps * GS * npres;
        if (gl == 0 && dbg) {   // development: walk length histogram (MUMS_DEV_CHAIN_DEBUG)
            atomicAdd(&dbg[0], steps > 1 ? 1u : 0u);
            atomicAdd(&dbg[1], steps > 16 ? 1u : 0u);
            atomicAdd(&dbg[2], steps > 256 ? 1u : 0u);
            atomicMax(&dbg[3], steps);
            atomicAdd(&dbg[4], steps);
        }
        if (gl == 0 && !handed) {
            const int64_t c = cur + dir * last;
            if (it.kind == 0) {
                link[it.j] = reached ? 1 : 0;
                if (!reached) rcol[it.j] = xa + c;
            } else if (it.kind == 1) {
                rcol[it.j] = xa + c;
            } else {
                lcol[it.j] = xa + c;
            }
        }
    }
    if (ctr && gl == 0 && my_items) {   // words / walks of this group (the roofline's byte count)
        atomicAdd(&ctr->walk_words, my_words);
        atomicAdd(&ctr->walk_items, my_items);
        atomicAdd(&ctr->walk_wins, my_wins);
    }
}

// chain of every probe; fk[chain] = its first probe in key order (kbase + the least ord[j]
// of the segment: a segmented min over the wave, one atomicMin per segment and wave)
__global__ __launch_bounds__(kBlock) void chain_seg_kernel(const uint8_t* __restrict__ link,
                                                           const uint32_t* __restrict__ ord,
                                                           const uint32_t* __restrict__ seg_excl, uint64_t P,
                                                           const int64_t* __restrict__ rcol,
                                                           uint32_t* __restrict__ chain_of,
                                                           int64_t* __restrict__ seg_r, uint32_t* __restrict__ fk,
                                                           uint32_t kbase, uint32_t* __restrict__ jl) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint32_t s = 0xFFFFFFFFu, m = 0xFFFFFFFFu;
    if (j < P) {
        const uint32_t f = (j == 0 || !link[j - 1]) ? 1u : 0u;
        s = seg_excl[j] + f - 1u;
        m = ord[j];
        if (chain_of) chain_of[m] = s;
        if (jl) {
            jl[j] = s;
            jl[P + j] = m;
        }
        if (!link[j]) seg_r[s] = rcol[j];
    }
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {   // segments are contiguous: equal s at distance d spans them
        const uint32_t om = __shfl_up(m, d, 64), os = __shfl_up(s, d, 64);
        if (lane >= d && os == s) m = min(m, om);
    }
    const uint32_t ns = __shfl_down(s, 1, 64);
    if (j < P && (lane == 63 || ns != s)) atomicMin(&fk[s], kbase + m);
}

// the extended entry of every chain (ExtendMatch write-back, MatchFinder.h:218-374;
// stored copies have m_mersize 0, MatchHashEntry.cpp:122): pool[s] = {len, offset, starts}
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_entry_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                             GenomeTable gt, MatchParams mp, int L,
                                                             const uint32_t* __restrict__ ord,
                                                             const uint8_t* __restrict__ link,
                                                             const uint32_t* __restrict__ seg_excl,
                                                             const int64_t* __restrict__ lcol,
                                                             const int64_t* __restrict__ seg_r,
                                                             int64_t* __restrict__ pool) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    if (j > 0 && link[j - 1]) return;
    const uint32_t s = seg_excl[j];
    Mhe<MG> A;
    probe_of<MG, View>(v, probe_info, j, gt, mp, L, A);
    const int64_t xa = start_at(A, first_start(A));
    const int64_t cmin = lcol[j] - xa, cmax = seg_r[s] - xa;
    int64_t* e = pool + (uint64_t)s * (uint64_t)(gt.G + 2);
    int64_t w[MG + 2];
    w[0] = cmax - cmin + L;
    w[1] = A.offset;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t sg = A.s[g];
        w[2 + g] = sg > 0 ? sg + cmin : (sg < 0 ? -((-sg) - cmax) : 0);
    }
    if ((gt.G & 1) == 0) {   // 16-B stores (the entry is (G + 2) x 8 B, 16-B aligned for even G)
        #pragma unroll
        for (int q = 0; q < MG + 2; q += 2)
            if (q < gt.G + 2) *reinterpret_cast<int4*>(e + q) = make_int4((int)w[q], (int)(w[q] >> 32), (int)w[q + 1],
                                                                          (int)(w[q + 1] >> 32));
    } else {
        #pragma unroll
        for (int q = 0; q < MG + 2; ++q)
            if (q < gt.G + 2) e[q] = w[q];
    }
}

// ---- line order: (line hash, reference start) by two stable onesweep sorts -------------
// of packed 8-B records (radix_seg.hip): first (x << 32 | k) by x (written by the probe
// producer, chain_line_slots), then (hash << 32 | position after the first sort) by hash;
// ord[j] = the probe at line position j
// The records carry the hash sort's keys, so its four digit histograms are counted here
// (hh: 4 x 256, zeroed) instead of by a histogram read of the records (seg_onesweep_sort
// hist_in).  Grid-stride; in x order most hashes repeat (a line's probes, the main diagonal
// above all): a wave adds the lanes equal to its first lane's hash with one LDS add per digit.
__global__ __launch_bounds__(kBlock) void line_rec2_kernel(const uint32_t* __restrict__ lhash,
                                                           const uint64_t* __restrict__ s1, uint64_t P,
                                                           uint64_t* __restrict__ rec, uint32_t* __restrict__ hh) {
    __shared__ uint32_t h[4][256];
    for (int i = threadIdx.x; i < 4 * 256; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t Pr = (P + kBlock - 1) / kBlock * kBlock;   // uniform trip count (ballots)
    const int lane = threadIdx.x & 63;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < Pr; i += stride) {
        const bool valid = i < P;
        const uint32_t hv = valid ? lhash[(uint32_t)s1[i]] : 0u;
        if (valid) rec[i] = ((uint64_t)hv << 32) | i;
        const uint32_t v0 = __builtin_amdgcn_readfirstlane(hv);
        const uint64_t m = __ballot(valid && hv == v0);
        if (m && lane == __builtin_ctzll(m)) {
            const uint32_t c = (uint32_t)__popcll(m);
            #pragma unroll
            for (int d = 0; d < 4; ++d) atomicAdd(&h[d][(v0 >> (8 * d)) & 0xFFu], c);
        }
        if (valid && hv != v0) {
            #pragma unroll
            for (int d = 0; d < 4; ++d) atomicAdd(&h[d][(hv >> (8 * d)) & 0xFFu], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 256; i += kBlock) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&hh[i], c);
    }
}

__global__ __launch_bounds__(kBlock) void line_ord_kernel(const uint64_t* __restrict__ s1,
                                                          const uint64_t* __restrict__ s2, uint64_t P,
                                                          uint32_t* __restrict__ ord) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < P) ord[j] = (uint32_t)s1[(uint32_t)s2[j]];
}

// the rows in line order as LineRows (match_device.h): a block's kBlock rows are loaded
// element-wise (neighbouring lanes on one row, all loads in flight together) into LDS, then
// each thread packs one row's starts to int32 and checks that they fit and that the
// recomputed offset equals the materialized one (*bad |= 1 otherwise: the caller redoes
// the chains from the 64-bit rows)
template <int MG>
__global__ __launch_bounds__(kBlock) void gather_line_rows_kernel(const int64_t* __restrict__ src,
                                                                  const uint32_t* __restrict__ ord, uint64_t P, int G,
                                                                  int L, int32_t* __restrict__ dst,
                                                                  unsigned int* __restrict__ bad) {
    static_assert(MG % 4 == 0 && MG <= 16, "int4 rows, LDS staging");
    __shared__ int64_t srow[kBlock * (MG + 1)];
    __shared__ uint32_t sk[kBlock];
    const uint64_t j0 = (uint64_t)blockIdx.x * kBlock;
    const uint32_t nj = P - j0 < (uint64_t)kBlock ? (uint32_t)(P - j0) : (uint32_t)kBlock;
    const uint32_t W = (uint32_t)G + 1, ne = nj * W;
    if (threadIdx.x < nj) sk[threadIdx.x] = ord[j0 + threadIdx.x];
    __syncthreads();
    uint32_t r = threadIdx.x / W, c = threadIdx.x - r * W;
    const uint32_t dr = kBlock / W, dc = kBlock % W;
    int64_t x[MG + 1];
    #pragma unroll
    for (int i = 0; i < MG + 1; ++i) {
        const uint32_t e = threadIdx.x + (uint32_t)i * kBlock;
        x[i] = e < ne ? src[(uint64_t)sk[r] * W + c] : 0;
        r += dr;
        c += dc;
        if (c >= W) { c -= W; ++r; }
    }
    #pragma unroll
    for (int i = 0; i < MG + 1; ++i) {
        const uint32_t e = threadIdx.x + (uint32_t)i * kBlock;
        if (e < ne) srow[e] = x[i];
    }
    __syncthreads();
    if (threadIdx.x >= nj) return;
    const int64_t* row = srow + threadIdx.x * W;
    Mhe<MG> Q;
    bool ok = true;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        Q.s[g] = g < G ? row[g] : 0;
        ok = ok && Q.s[g] == (int64_t)(int32_t)Q.s[g];
    }
    ok = ok && probe_offset<MG>(Q, L) == row[G];
    int32_t* out = dst + (j0 + threadIdx.x) * (uint64_t)line_row_stride(G);
    #pragma unroll
    for (int q = 0; q < MG / 4; ++q)
        if (4 * q < G)
            *reinterpret_cast<int4*>(out + 4 * q) =
                make_int4((int32_t)Q.s[4 * q], (int32_t)Q.s[4 * q + 1], (int32_t)Q.s[4 * q + 2], (int32_t)Q.s[4 * q + 3]);
    if (!ok) atomicOr(bad, 1u);
}

// int32 rows (MatProbes::rows32) in line order: row ord[j] -> row j, S / 4 int4 per row
__global__ __launch_bounds__(kBlock) void gather_rows32_kernel(const int32_t* __restrict__ src,
                                                               const uint32_t* __restrict__ ord, uint64_t P,
                                                               uint32_t S, int32_t* __restrict__ dst) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    const int4* a = reinterpret_cast<const int4*>(src + (uint64_t)ord[j] * S);
    int4* b = reinterpret_cast<int4*>(dst + j * S);
    if (S == 8) {
        const int4 x = a[0], y = a[1];
        b[0] = x;
        b[1] = y;
    } else {
        for (uint32_t q = 0; q < S / 4; ++q) b[q] = a[q];
    }
}

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// host: the seed's care set is palindromic and its weight odd (line_spec's bitpar and !even_w)
inline bool seed_bitpar_odd(const SeedSpec& ss) {
    if (ss.pattern == 0 || ss.L <= 0 || ss.L > 64) return false;
    const uint64_t pat = ss.pattern >> __builtin_ctzll(ss.pattern);
    uint64_t rev = 0;
    for (int i = 0; i < 64; ++i) rev |= ((pat >> i) & 1ull) << (63 - i);
    rev >>= (64 - ss.L);
    return rev == pat && (ss.w & 1);
}

// --- chunked FindMatches: chains labelled per slice of the probes ---------------------
// launch_chains on a slice of the probes gives every probe its true chain entry (walks
// read the genomes, not the other probes), but a chain whose probes fall into several
// slices gets one entry per slice.  The replay needs one id per chain (its chain-first
// probe, its rank among the bucket's chains), so the per-slice entries are merged by
// content: hash sort, then the first equal entry of each equal-hash run is the chain.

__global__ __launch_bounds__(kBlock) void add_offset_kernel(uint32_t* __restrict__ a, uint64_t n, uint32_t off) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] += off;
}

__global__ __launch_bounds__(kBlock) void entry_hash_kernel(const int64_t* __restrict__ pool, uint64_t n, int G,
                                                            uint64_t* __restrict__ key) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t* e = pool + i * (uint64_t)(G + 2);
    uint64_t h = 0x243f6a8885a308d3ull;
    for (int g = 0; g < G + 2; ++g) h = mix64(h ^ (uint64_t)e[g] ^ ((uint64_t)g << 58));
    key[i] = h;
}

__device__ __forceinline__ bool same_entry(const int64_t* __restrict__ a, const int64_t* __restrict__ b, int W) {
    for (int g = 0; g < W; ++g)
        if (a[g] != b[g]) return false;
    return true;
}

// sorted position i: rep[i] = first position of its equal-hash run holding an equal
// entry (i itself when none), isrep[i] = rep[i] == i
__global__ __launch_bounds__(kBlock) void entry_rep_kernel(const int64_t* __restrict__ pool, const uint64_t* __restrict__ key,
                                                           const uint32_t* __restrict__ ord, uint64_t n, int G,
                                                           uint32_t* __restrict__ rep, uint32_t* __restrict__ isrep) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = ord[i];
    const uint64_t h = key[c];
    const int W = G + 2;
    const int64_t* ec = pool + (uint64_t)c * W;
    uint64_t r0 = i;
    while (r0 > 0 && key[ord[r0 - 1]] == h) --r0;
    uint64_t r = i;
    for (uint64_t j = r0; j < i; ++j)
        if (same_entry(pool + (uint64_t)ord[j] * W, ec, W)) { r = j; break; }
    rep[i] = (uint32_t)r;
    isrep[i] = r == i ? 1u : 0u;
}

// gmap[local chain] = merged chain id; the merged pool holds each chain's entry once
__global__ __launch_bounds__(kBlock) void entry_map_kernel(const int64_t* __restrict__ pool, const uint32_t* __restrict__ ord,
                                                           const uint32_t* __restrict__ rep, const uint32_t* __restrict__ gid,
                                                           uint64_t n, int G, uint32_t* __restrict__ gmap,
                                                           int64_t* __restrict__ pool_out,
                                                           const uint32_t* __restrict__ fk_loc,
                                                           uint32_t* __restrict__ fk_out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = ord[i], r = rep[i], g = gid[r];
    gmap[c] = g;
    atomicMin(&fk_out[g], fk_loc[c]);   // the merged chain's first probe: the earliest slice's
    if (r == (uint32_t)i) {
        const int W = G + 2;
        for (int w = 0; w < W; ++w) pool_out[(uint64_t)g * W + w] = pool[(uint64_t)c * W + w];
    }
}

__global__ __launch_bounds__(kBlock) void chain_remap_kernel(uint32_t* __restrict__ chain_of, uint64_t P,
                                                             const uint32_t* __restrict__ gmap) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < P) chain_of[k] = gmap[chain_of[k]];
}

}  // namespace

hipError_t launch_add_offset(uint32_t* a, uint64_t n, uint32_t off, hipStream_t st) {
    if (n == 0 || off == 0) return hipSuccess;
    hipLaunchKernelGGL(add_offset_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, a, n, off);
    return hipGetLastError();
}

size_t chain_merge_tmp_bytes(uint64_t n) { return (n + 64) * (8 * 3 + 4 * 5) + 8 * 256; }

hipError_t launch_chain_merge(const int64_t* pool_loc, uint64_t n, int G, uint32_t* chain_of, uint64_t P,
                              int64_t* pool_out, void* d_tmp, void* d_radix_tmp, void* d_scan_tmp, uint32_t* d_nchains,
                              hipStream_t st, const uint32_t* fk_loc, uint32_t* fk_out) {
    if (n == 0) return hipMemsetAsync(d_nchains, 0, 4, st);
    char* p = (char*)d_tmp;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    uint64_t* key = (uint64_t*)carve(n * 8);
    uint64_t* kA = (uint64_t*)carve(n * 8);
    uint64_t* kB = (uint64_t*)carve(n * 8);
    uint32_t* vA = (uint32_t*)carve(n * 4);
    uint32_t* vB = (uint32_t*)carve(n * 4);
    uint32_t* rep = (uint32_t*)carve(n * 4);
    uint32_t* gid = (uint32_t*)carve(n * 4);
    uint32_t* gmap = (uint32_t*)carve(n * 4);
    const unsigned grid = grid_of(n);
    hipLaunchKernelGGL(entry_hash_kernel, dim3(grid), dim3(kBlock), 0, st, pool_loc, n, G, key);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    int buf = 0;
    if ((e = radix_sort<uint64_t>(key, nullptr, n, 64, kA, vA, kB, vB, d_radix_tmp, &buf, st)) != hipSuccess) return e;
    const uint32_t* ord = buf ? vB : vA;
    hipLaunchKernelGGL(entry_rep_kernel, dim3(grid), dim3(kBlock), 0, st, pool_loc, (const uint64_t*)key, ord, n, G, rep,
                       gid);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(gid, n, d_scan_tmp, d_nchains, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(fk_out, 0xFF, n * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(entry_map_kernel, dim3(grid), dim3(kBlock), 0, st, pool_loc, ord, (const uint32_t*)rep,
                       (const uint32_t*)gid, n, G, gmap, pool_out, fk_loc, fk_out);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(chain_remap_kernel, dim3(grid_of(P)), dim3(kBlock), 0, st, chain_of, P, (const uint32_t*)gmap);
    return hipGetLastError();
}

namespace {

}  // namespace

size_t chain_tmp_bytes(uint64_t P, uint32_t Tb, int G) {
    // lkey, sort A/B keys (3 x 8) + vals A/B (2 x 4) + link (1) + rcol, lcol, seg_r (3 x 8)
    // + seg (4) + queues (2 x 24) + padding.  The replay reuses it: per chain <= 76 B, then the
    // big-bucket scratch (count 4 + scan 4 + slot 16 per probe, + 4 per bucket)
    // + the probe rows in line order ((G + 1) x 8)
    return P * (24 + 8 + 1 + 24 + 4 + 2 * sizeof(WalkItem) + 32 + 24 + 8 * (uint64_t)(G + 1)) + (uint64_t)Tb * 4 + 64 * 64 +
           4 * 256 * 4 + 256;   // + the line hashes' digit histograms (line_rec2_kernel)
}

namespace {

// launch_chains' scratch in d_chain_tmp (rows_line only when the rows are gathered there)
struct ChainWs {
    uint64_t *lkey, *kA, *kB;
    uint32_t *vA, *vB;
    uint8_t* link;
    int64_t *rcol, *lcol, *seg_r;
    uint32_t* seg;
    WalkItem *queue, *queue_long;
    unsigned int* qcount;
    int64_t* rows_line;
    uint32_t* bst;   // {0, P}: the one bucket of the line sort
    uint32_t* hh;    // 4 x 256: the line hashes' digit histograms (the hash sort's passes)
};

ChainWs chain_ws(void* d_chain_tmp, uint64_t P, int G, bool with_rows) {
    char* p = (char*)d_chain_tmp;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    ChainWs w;
    w.lkey = (uint64_t*)carve(P * 8);
    w.kA = (uint64_t*)carve(P * 8);
    w.kB = (uint64_t*)carve(P * 8);
    w.vA = (uint32_t*)carve(P * 4);
    w.vB = (uint32_t*)carve(P * 4);
    w.link = (uint8_t*)carve(P);
    w.rcol = (int64_t*)carve(P * 8);
    w.lcol = (int64_t*)carve(P * 8);
    w.seg_r = (int64_t*)carve(P * 8);
    w.seg = (uint32_t*)carve(P * 4);
    w.queue = (WalkItem*)carve(P * sizeof(WalkItem));
    w.queue_long = (WalkItem*)carve(P * sizeof(WalkItem));
    w.qcount = (unsigned int*)carve(64);
    w.bst = (uint32_t*)carve(64);
    w.hh = (uint32_t*)carve(4 * 256 * 4);
    w.rows_line = with_rows ? (int64_t*)carve(P * (uint64_t)(G + 1) * 8) : nullptr;
    return w;
}

// line order of the P probes from the records (x << 32 | k) in w.kA and the line hashes in
// w.vB: ord[j] (in w.vA) = the probe at line position j.  Two stable onesweep sorts of packed
// records (by x on xbits bits, then by hash) instead of eight 8-bit passes over 12-B
// (key, value) pairs.  w.lkey is the second sort's ping-pong buffer.
hipError_t line_sort(const ChainWs& w, uint64_t P, int xbits, void* d_tmp, uint32_t* d_err, hipStream_t st,
                     const uint32_t** ord_out) {
    hipError_t e;
    if ((e = seg_bucket_starts(nullptr, 0, 0, P, w.bst, st)) != hipSuccess) return e;
    int b1 = 0;
    if ((e = seg_onesweep_sort(w.kA, w.kB, P, xbits, 0, w.bst, d_tmp, d_err, &b1, st)) != hipSuccess) return e;
    const uint64_t* s1 = b1 ? w.kB : w.kA;
    uint64_t* r2 = b1 ? w.kA : w.kB;
    const bool fused_hist = kLineHashBits == 32 && !getenv("MUMS_DEV_LINE_GHIST");   // read per call
    if ((e = hipMemsetAsync(w.hh, 0, 4 * 256 * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(line_rec2_kernel, dim3((unsigned)std::min<uint64_t>(grid_of(P), 4096)), dim3(kBlock), 0, st,
                       (const uint32_t*)w.vB, s1, P, r2, w.hh);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    int b2 = 0;
    // the hashes in x order come in runs (a line's probes): run-aware histogram, late publish
    const bool runs = !getenv("MUMS_DEV_LINE_NORUNS");   // read per call (tests toggle it)
    // the last hash pass stores ord[o] = probe of s1[j] directly (MUMS_DEV_LINE_ORD=1, read per
    // call: the records, then line_ord_kernel's gather)
    const bool fused_ord = runs && !getenv("MUMS_DEV_LINE_ORD");
    if ((e = seg_onesweep_sort(r2, w.lkey, P, kLineHashBits, 0, w.bst, d_tmp, d_err, &b2, st, nullptr, 32, false,
                               runs, fused_hist ? w.hh : nullptr, fused_ord ? s1 : nullptr,
                               fused_ord ? w.vA : nullptr)) != hipSuccess)
        return e;
    if (!fused_ord) {
        const uint64_t* s2 = b2 ? w.lkey : r2;
        hipLaunchKernelGGL(line_ord_kernel, dim3(grid_of(P)), dim3(kBlock), 0, st, s1, s2, P, w.vA);
    }
    *ord_out = w.vA;
    return hipGetLastError();
}

int x_bits(const GenomeTable& gt) {
    uint64_t mx = 1;
    for (int g = 0; g < gt.G; ++g) mx = gt.n[g] + 2 > mx ? gt.n[g] + 2 : mx;
    int b = 1;
    while (b < 32 && (1ull << b) < mx) ++b;
    return b;
}

// after the line sort (ord = probe of line position j, vl.rows = the rows in line order):
// links, walks, segment ids, chain_of and the chain entries
template <int MG, typename LV>
hipError_t chains_core(LV vl, const ChainWs& w, const uint32_t* ord, uint64_t P, const GenomeTable& gt,
                       const MatchParams& mp, const SeedSpec& ss, const uint32_t* packed, void* d_scan_tmp,
                       void* d_radix_tmp, uint32_t* chain_of, int64_t* pool, uint32_t* d_nchains, hipStream_t st,
                       void* ctr, hipEvent_t* ev_walk, uint32_t* fk, uint32_t kbase, uint32_t* jl) {
    hipError_t e;
    const unsigned grid = grid_of(P);
    const unsigned walk_grid = 2048, short_grid = 8192;
    unsigned int* qcount = w.qcount;
    unsigned int* qshort = qcount;      // chain_link / chain_left -> chain_walk_short_kernel
    unsigned int* qlong = qcount + 1;   // chain_walk_short_kernel -> chain_walk_kernel
    const bool cdbg = getenv("MUMS_DEV_CHAIN_DEBUG") != nullptr;
    // refilled short-walk lanes (read per call: tests and A/B runs toggle it)
    const bool refill = getenv("MUMS_DEV_WALK_REFILL") && getenv("MUMS_DEV_WALK_REFILL")[0] == '1';
    // the walks without the generic hit-word path when every window is tested by base comparison
    // (palindromic care set, odd weight: hit_word<MG, false>); MUMS_DEV_WALK_GEN=1 keeps it
    const bool lean = seed_bitpar_odd(ss) && !(getenv("MUMS_DEV_WALK_GEN") && getenv("MUMS_DEV_WALK_GEN")[0] == '1');
    // short walks in genome-position order (walk_key_kernel), MUMS_DEV_WALK_SORT=1: measured
    // slower at C3 than the queue's line order, kept for A/B runs
    const char* wsort_env = getenv("MUMS_DEV_WALK_SORT");
    const bool wsort = !refill && wsort_env && (wsort_env[0] == '1' || wsort_env[0] == '2') && P < (1ull << 32);
    const bool wsort_long = wsort && wsort_env[0] == '2';   // and the handed-on walks back in line order
    int pbits = 1;
    while (pbits < 32 && (1ull << pbits) < P) ++pbits;
    // (MUMS_DEV_WALK_SHIFT, read per call: the granule of that order, development A/B)
    const char* wsh_env = getenv("MUMS_DEV_WALK_SHIFT");
    const int wshift = wsh_env ? std::max(0, std::min(31, atoi(wsh_env))) : kWalkSortShift;
    const int wbits = std::max(1, x_bits(gt) - wshift);
    uint32_t* d_err = ctr ? &((DevCounters*)ctr)->err : w.qcount + 14;
    for (int pass = 0; pass < 2; ++pass) {
        if ((e = hipMemsetAsync(qcount, 0, 12, st)) != hipSuccess) return e;
        const unsigned lgrid = (unsigned)((P + kBlock * kLinkIPT - 1) / (kBlock * kLinkIPT));
        if (pass == 0)
            hipLaunchKernelGGL((chain_link_kernel<MG, LV>), dim3(lgrid), dim3(kBlock), 0, st, vl, nullptr, P, gt,
                               mp, ss, w.link, w.queue, qshort, qcount + 12, jl ? jl + 2 * P : nullptr);
        else
            hipLaunchKernelGGL(chain_left_kernel, dim3(lgrid), dim3(kBlock), 0, st, P, (const uint8_t*)w.link, w.queue,
                               qshort, w.seg);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        const uint64_t* order = nullptr;
        if (wsort) {   // the queue length sizes the sort: read back (one small sync per pass)
            unsigned nq = 0;
            if ((e = hipMemcpyAsync(&nq, qshort, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            if (nq > 1) {
                hipLaunchKernelGGL((walk_key_kernel<MG, LV>), dim3(grid_of(nq)), dim3(kBlock), 0, st, vl, gt, mp, ss.L,
                                   (const WalkItem*)w.queue, (const unsigned int*)qshort, wshift, w.kA);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = seg_bucket_starts(nullptr, 0, 0, nq, w.bst + 8, st)) != hipSuccess) return e;
                int ob = 0;
                if ((e = seg_onesweep_sort(w.kA, w.kB, nq, wbits, 0, w.bst + 8, d_radix_tmp, d_err, &ob, st)) !=
                    hipSuccess)
                    return e;
                order = ob ? w.kB : w.kA;
            }
        }
        if (ev_walk) (void)hipEventRecord(ev_walk[3 * pass], st);   // the short walks start
        if (refill)
            hipLaunchKernelGGL((chain_walk_refill_kernel<MG, LV>), dim3(short_grid), dim3(kBlock), 0, st, vl, gt, mp,
                               ss, packed, (const WalkItem*)w.queue, (const unsigned int*)qshort, w.link, w.rcol,
                               w.lcol, w.queue_long, qlong);
        else if (lean)
            hipLaunchKernelGGL((chain_walk_short_kernel<MG, LV, false>), dim3(short_grid), dim3(kBlock), 0, st, vl,
                               nullptr, gt, mp, ss, packed, (const WalkItem*)w.queue, (const unsigned int*)qshort,
                               w.link, w.rcol, w.lcol, w.queue_long, qlong, order, (DevCounters*)ctr);
        else
            hipLaunchKernelGGL((chain_walk_short_kernel<MG, LV>), dim3(short_grid), dim3(kBlock), 0, st, vl, nullptr,
                               gt, mp, ss, packed, (const WalkItem*)w.queue, (const unsigned int*)qshort, w.link,
                               w.rcol, w.lcol, w.queue_long, qlong, order, (DevCounters*)ctr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (cdbg && (e = hipMemsetAsync(qcount + 4, 0, 32, st)) != hipSuccess) return e;
        if (ev_walk) (void)hipEventRecord(ev_walk[3 * pass + 1], st);
        const uint64_t* lorder = nullptr;
        if (wsort_long && order) {
            unsigned nl = 0;
            if ((e = hipMemcpyAsync(&nl, qlong, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            if (nl > 1) {
                uint64_t* ra = order == w.kA ? w.kB : w.kA;   // the short walks' order is consumed
                uint64_t* rb = order == w.kA ? w.kA : w.kB;
                hipLaunchKernelGGL(walk_line_key_kernel, dim3(grid_of(nl)), dim3(kBlock), 0, st,
                                   (const WalkItem*)w.queue_long, (const unsigned int*)qlong, ra);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = seg_bucket_starts(nullptr, 0, 0, nl, w.bst + 8, st)) != hipSuccess) return e;
                int ob = 0;
                if ((e = seg_onesweep_sort(ra, rb, nl, pbits, 0, w.bst + 8, d_radix_tmp, d_err, &ob, st)) !=
                    hipSuccess)
                    return e;
                lorder = ob ? rb : ra;
            }
        }
        // the queue of chain_link / chain_left is consumed: it takes the handed-on walks
#define MUMS_WALK_LAUNCH(GEN)                                                                                     \
    do {                                                                                                             \
        hipLaunchKernelGGL((chain_walk_kernel<MG, LV, kWalkGroup, GEN>), dim3(walk_grid), dim3(kBlock), 0, st, vl,  \
                           nullptr, gt, mp, ss, ord, packed, (const WalkItem*)w.queue_long, (const unsigned int*)qlong, \
                           w.link, w.rcol, w.lcol, cdbg ? qcount + 4 : nullptr, (DevCounters*)ctr, kWalkHandoff,     \
                           w.queue, qcount + 2, lorder);                                                             \
        if ((e = hipGetLastError()) != hipSuccess) return e;                                                         \
        if (kWalkHandoff)                                                                                            \
            hipLaunchKernelGGL((chain_walk_kernel<MG, LV, 64, GEN>), dim3(walk_grid), dim3(kBlock), 0, st, vl, nullptr, \
                               gt, mp, ss, ord, packed, (const WalkItem*)w.queue, (const unsigned int*)(qcount + 2), \
                               w.link, w.rcol, w.lcol, cdbg ? qcount + 4 : nullptr, (DevCounters*)ctr, 0u,           \
                               (WalkItem*)nullptr, (unsigned int*)nullptr, (const uint64_t*)nullptr);               \
    } while (0)
        if (lean) MUMS_WALK_LAUNCH(false);
        else MUMS_WALK_LAUNCH(true);
#undef MUMS_WALK_LAUNCH
        if (ev_walk) (void)hipEventRecord(ev_walk[3 * pass + 2], st);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (cdbg) {   // development: walk queue sizes and the long walks' step histogram
            unsigned hq[9] = {};
            (void)hipMemcpyAsync(hq, qcount, 36, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            fprintf(stderr, "chains: pass %d walks %u, long %u (to whole waves %u) of %lu probes; steps >1: %u >16: %u "
                    ">256: %u max %u total %u\n", pass, hq[0], hq[1], hq[2], (unsigned long)P, hq[4], hq[5], hq[6], hq[7],
                    hq[8]);
        }
    }
    // (the segment-start flags in w.seg: chain_left_kernel)
    if ((e = exclusive_scan_u32(w.seg, P, d_scan_tmp, d_nchains, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(fk, 0xFF, P * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(chain_seg_kernel, dim3(grid), dim3(kBlock), 0, st, w.link, ord, w.seg, P, w.rcol, chain_of,
                       w.seg_r, fk, kbase, jl);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((chain_entry_kernel<MG, LV>), dim3(grid), dim3(kBlock), 0, st, vl, nullptr, P, gt, mp,
                       ss.L, ord, w.link, w.seg, w.lcol, w.seg_r, pool);
    return hipGetLastError();
}

}  // namespace

// the line order: onesweep records when the reference starts fit 32 bits and P < 2^30
// (MUMS_DEV_LINE_RADIX: the 64-bit pair sort), else 64-bit (key, value) radix passes
bool chain_line_records(uint64_t P, const GenomeTable& gt) {
    const bool pairs = getenv("MUMS_DEV_LINE_RADIX") != nullptr;
    uint64_t mx = 0;
    for (int g = 0; g < gt.G; ++g) mx = gt.n[g] > mx ? gt.n[g] : mx;
    return !pairs && P < (1ull << 30) && mx + 2 < (1ull << 32);
}

namespace {

hipError_t line_order(const ChainWs& w, uint64_t P, const GenomeTable& gt, void* d_tmp, void* ctr, hipStream_t st,
                      const uint32_t** ord) {
    if (chain_line_records(P, gt))
        return line_sort(w, P, x_bits(gt), d_tmp, ctr ? &((DevCounters*)ctr)->err : w.qcount + 14, st, ord);
    int buf = 0;
    hipError_t e = radix_sort<uint64_t>(w.lkey, nullptr, P, 64, w.kA, w.vA, w.kB, w.vB, d_tmp, &buf, st);
    *ord = buf ? w.vB : w.vA;
    return e;
}

// exact line order (after an interleaving line-hash collision): by x, then stably by the
// 64-bit line hash (two radix sorts of (key, probe) pairs; rows in key order)
template <int MG>
__global__ __launch_bounds__(kBlock) void line_x_kernel(MatProbes v, uint64_t P, int G, uint64_t* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    Mhe<MG> Q;
    load_probe<MG>(v, (uint32_t)k, G, 0, Q);
    out[k] = (uint64_t)start_at(Q, first_start(Q));
}

template <int MG>
__global__ __launch_bounds__(kBlock) void line_h64_kernel(MatProbes v, const uint32_t* __restrict__ vk, uint64_t P,
                                                          int G, uint64_t* __restrict__ out,
                                                          uint32_t* __restrict__ vcopy) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= P) return;
    Mhe<MG> Q;
    load_probe<MG>(v, vk[i], G, 0, Q);
    out[i] = line_hash64<MG>(Q, G);
    vcopy[i] = vk[i];
}

template <int MG>
hipError_t line_order_exact(MatProbes v, const ChainWs& w, uint64_t P, const GenomeTable& gt, void* d_tmp,
                            hipStream_t st, const uint32_t** ord) {
    hipLaunchKernelGGL((line_x_kernel<MG>), dim3(grid_of(P)), dim3(kBlock), 0, st, v, P, gt.G, w.lkey);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    int b1 = 0;
    if ((e = radix_sort<uint64_t>(w.lkey, nullptr, P, x_bits(gt), w.kA, w.vA, w.kB, w.vB, d_tmp, &b1, st)) != hipSuccess)
        return e;
    hipLaunchKernelGGL((line_h64_kernel<MG>), dim3(grid_of(P)), dim3(kBlock), 0, st, v, b1 ? w.vB : w.vA, P, gt.G,
                       w.lkey, w.seg);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    int b2 = 0;
    if ((e = radix_sort<uint64_t>(w.lkey, w.seg, P, 64, w.kA, w.vA, w.kB, w.vB, d_tmp, &b2, st)) != hipSuccess) return e;
    *ord = b2 ? w.vB : w.vA;
    return hipSuccess;
}

}  // namespace

uint64_t* chain_lkey_slot(void* d_chain_tmp, uint64_t P, int G) { return chain_ws(d_chain_tmp, P, G, true).lkey; }

void chain_line_slots(void* d_chain_tmp, uint64_t P, int G, uint64_t** rec, uint32_t** lhash) {
    const ChainWs w = chain_ws(d_chain_tmp, P, G, true);
    *rec = w.kA;
    *lhash = w.vB;
}

size_t chain_radix_tmp_bytes(uint64_t P) { return std::max(radix_tmp_bytes(P), onesweep_tmp_bytes(P, 0, 32)); }

// Chain labelling of the P probes (key order): chain_of[k] = chain of probe k;
// pool[c] = extended entry of chain c; *d_nchains (device) = number of chains.
template <int MG, typename View>
hipError_t launch_chains(View v, const uint64_t* probe_info, uint64_t P, const GenomeTable& gt, const MatchParams& mp,
                         const SeedSpec& ss, const uint32_t* packed, void* d_chain_tmp, void* d_scan_tmp,
                         void* d_radix_tmp, uint32_t* chain_of, int64_t* pool, uint32_t* d_nchains, hipStream_t st,
                         void* ctr, hipEvent_t* ev_walk, uint32_t* fk, uint32_t kbase, bool lkey_ready,
                         uint32_t* jl) {
    if (P == 0) return hipSuccess;
    if (v.rows32 && !(MG % 4 == 0 && MG <= 16)) return hipErrorInvalidValue;   // int32 rows: G <= 16 only
    const ChainWs w = chain_ws(d_chain_tmp, P, gt.G, true);
    hipError_t e;
    if (!lkey_ready) {   // else written by the materialize pass (chain_lkey_slot)
        const bool recs = chain_line_records(P, gt);
        hipLaunchKernelGGL((chain_key_kernel<MG, View>), dim3(grid_of(P)), dim3(kBlock), 0, st, v, probe_info, P, gt,
                           mp, ss.L, recs ? w.kA : w.lkey, recs ? w.vB : nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const uint32_t* ord = nullptr;
    if ((e = line_order(w, P, gt, d_radix_tmp, ctr, st, &ord)) != hipSuccess) return e;
    // the rows in line order: the link / walk / entry kernels then read row j, not row ord[j];
    // as LineRows (int32 starts, 32 B per probe at G = 8) when every start fits 31 bits
    uint64_t mx = 0;
    for (int g = 0; g < gt.G; ++g) mx = gt.n[g] > mx ? gt.n[g] : mx;
    // test hooks, read per call: "1" the 64-bit rows, "retry" the int32 rows flagged bad once
    const char* wide_sw = getenv("MUMS_DEV_WIDE_LINE_ROWS");
    const bool force_retry = wide_sw && !strcmp(wide_sw, "retry");
    const bool wide_env = wide_sw && !force_retry;
    bool narrow = MG % 4 == 0 && MG <= 16 && !wide_env && mx + 2 < (1ull << 31);
    unsigned int* flags = w.qcount + 12;   // [0] interleaving line-hash collision, [1] a row not narrow
    auto chains_from = [&](const uint32_t* o) -> hipError_t {
        hipError_t r;
        if ((r = hipMemsetAsync(flags, 0, 8, st)) != hipSuccess) return r;
        if constexpr (MG % 4 == 0 && MG <= 16) {
            // the int32 rows are read through the line order (chain_link shares each row with its
            // neighbour lane): 1.3 ms less than gathering them at C3;
            // MUMS_DEV_LINE_GATHER=1 (read per call) gathers them first
            const char* lg = getenv("MUMS_DEV_LINE_GATHER");
            if (v.rows32 && !(lg && lg[0] == '1')) {
                LineRows vl{v.rows32, v.stride32, v.L32, o};
                return chains_core<MG>(vl, w, o, P, gt, mp, ss, packed, d_scan_tmp, d_radix_tmp, chain_of, pool,
                                       d_nchains, st, ctr, ev_walk, fk, kbase, jl);
            }
            if (v.rows32) {   // int32 rows in key order (materialize_dispatch): copied in line order
                hipLaunchKernelGGL(gather_rows32_kernel, dim3(grid_of(P)), dim3(kBlock), 0, st, v.rows32, o, P,
                                   v.stride32, (int32_t*)w.rows_line);
                if ((r = hipGetLastError()) != hipSuccess) return r;
                LineRows vl{(const int32_t*)w.rows_line, v.stride32, v.L32};
                return chains_core<MG>(vl, w, o, P, gt, mp, ss, packed, d_scan_tmp, d_radix_tmp, chain_of, pool, d_nchains, st, ctr,
                                       ev_walk, fk, kbase, jl);
            }
            if (narrow) {
                hipLaunchKernelGGL((gather_line_rows_kernel<MG>), dim3(grid_of(P)), dim3(kBlock), 0, st, v.rows, o, P,
                                   gt.G, ss.L, (int32_t*)w.rows_line, flags + 1);
                if ((r = hipGetLastError()) != hipSuccess) return r;
                LineRows vl{(const int32_t*)w.rows_line, line_row_stride(gt.G), ss.L};
                return chains_core<MG>(vl, w, o, P, gt, mp, ss, packed, d_scan_tmp, d_radix_tmp, chain_of, pool, d_nchains, st, ctr,
                                       ev_walk, fk, kbase, jl);
            }
        }
        if ((r = launch_gather_rows(v.rows, o, P, gt.G, w.rows_line, st)) != hipSuccess) return r;
        MatProbes vl{};
        vl.rows = w.rows_line;
        return chains_core<MG>(vl, w, o, P, gt, mp, ss, packed, d_scan_tmp, d_radix_tmp, chain_of, pool, d_nchains, st, ctr, ev_walk,
                               fk, kbase, jl);
    };
    unsigned hf[2] = {0, 0};
    auto read_flags = [&]() -> hipError_t {
        hipError_t r;
        if ((r = hipMemcpyAsync(hf, flags, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return r;
        return hipStreamSynchronize(st);
    };
    if ((e = chains_from(ord)) != hipSuccess || (e = read_flags()) != hipSuccess) return e;
    if (force_retry && narrow && !v.rows32) hf[1] = 1;
    if (hf[1]) {   // a start or offset the int32 rows do not restate: the 64-bit rows
        narrow = false;
        if ((e = chains_from(ord)) != hipSuccess || (e = read_flags()) != hipSuccess) return e;
    }
    // two lines with equal 32-bit line hashes interleaved (a chain split in two segments):
    // the line order again with the 64-bit hash, and the chains again (rare: colliding
    // multi-probe lines whose x ranges overlap)
    if (!hf[0] && !getenv("MUMS_DEV_LINE_EXACT")) return hipSuccess;
    if (getenv("MUMS_DEV_CHAIN_DEBUG")) fprintf(stderr, "chains: line-hash collision, exact line order\n");
    MatProbes vk = v;
    vk.fs = nullptr;
    if ((e = line_order_exact<MG>(vk, w, P, gt, d_radix_tmp, st, &ord)) != hipSuccess) return e;
    return chains_from(ord);
}

#define MUMS_INST_CHAINS(MG, V)                                                                                   \
    template hipError_t launch_chains<MG, V>(V, const uint64_t*, uint64_t, const GenomeTable&, const MatchParams&, \
                                             const SeedSpec&, const uint32_t*, void*, void*, void*, uint32_t*,     \
                                             int64_t*, uint32_t*, hipStream_t, void*, hipEvent_t*, uint32_t*,    \
                                             uint32_t, bool, uint32_t*);
MUMS_INST_CHAINS(4, MatProbes)
MUMS_INST_CHAINS(8, MatProbes)
MUMS_INST_CHAINS(16, MatProbes)
MUMS_INST_CHAINS(32, MatProbes)
MUMS_INST_CHAINS(64, MatProbes)

}  // namespace mums
