// chunked.hip -- helpers of the chunked mode for more than 2^32 seed-mers per context
// (BASELINE config 5, 2 x 3 Gbp; SURVEY.md 8(e) "chunked SML over 288 GB HBM").
//
// The packed records carry 33-bit global indices (RecViewT<33>): with 2w+1 = 39 key bits
// the top 8 are the MSD digit (implicit in the record's bucket), 31 sit in the record.
// The MSD digits are cut into power-of-two chunks of < 2^30 records; every chunk is
// scattered (seed_scatter_kernel<.., 33, true>), sorted (onesweep, key bits from 33),
// grouped and probed on its own, in key order, so 32-bit stream offsets suffice inside a
// chunk and the probes come out in the reference's AddHashEntry order.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mums_internal.h"

namespace mums {
namespace {

// out[r] = sum of hist[r * T .. r * T + T) (records of MSD digit r)
__global__ __launch_bounds__(256) void digit_totals_kernel(const uint32_t* __restrict__ hist, uint32_t T,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s[256];
    const uint32_t r = blockIdx.x;
    unsigned long long acc = 0;
    for (uint32_t t = threadIdx.x; t < T; t += 256) acc += hist[(uint64_t)r * T + t];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[r] = s[0];
}

}  // namespace

hipError_t launch_digit_totals(const uint32_t* hist, uint32_t ndigits, uint32_t T, unsigned long long* out,
                               hipStream_t st) {
    if (ndigits == 0) return hipSuccess;
    hipLaunchKernelGGL(digit_totals_kernel, dim3(ndigits), dim3(256), 0, st, hist, T, out);
    return hipGetLastError();
}

}  // namespace mums

// ---- MER_REPEAT_LIMIT restarts and start points in the chunked mode ------------------
// MatchFinder::SearchRange's restart (MatchFinder.cpp:253-277) needs every genome's
// SortedMerList: its plan (restart_plan.h) reads SML keys by index, and a record lives iff
// its SML index reaches the start point of its key's phase.  With all chunks resident and
// sorted, the merged stream is one sorted array of N records; a stable partition by genome
// gives the G SMLs as full keys (ck, genome-major, 64-bit slots = global seed-mer indices),
// and a record's SML index is its rank among its genome's records in stream order, counted
// per block of kCrBlk records (per-genome block counts, scanned).
namespace mums {
namespace {

constexpr uint32_t kCrBlk = 4096;   // records per rank block (kBlock threads x 16 rounds)

__device__ __forceinline__ uint64_t cr_key(const CrStream& s, uint64_t j) {
    uint32_t lo = 0, n = s.nd;   // digit of j: digits whose end <= j
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (s.dstart[lo + h + 1] <= j) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return ((uint64_t)lo << s.kb) | ((s.rec[j] >> s.ib) & ((1ull << s.kb) - 1));
}

__device__ __forceinline__ uint64_t cr_idx(const CrStream& s, uint64_t j) { return s.rec[j] & ((1ull << s.ib) - 1); }

// digit (MSD bucket) of stream position j
__device__ __forceinline__ uint32_t cr_digit(const CrStream& s, uint64_t j) {
    uint32_t lo = 0, n = s.nd;
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (s.dstart[lo + h + 1] <= j) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo;
}

// cr_key for a position of a block whose first and last records have digits d0 <= d1: no
// search when they agree (nearly every block: 128 digits over 2e5 blocks at config 3)
__device__ __forceinline__ uint64_t cr_key_in(const CrStream& s, uint64_t j, uint32_t d0, uint32_t d1) {
    uint32_t d = d0;
    if (d1 != d0) {
        uint32_t lo = d0, n = d1 - d0;   // digits in [d0, d1] whose end <= j
        while (n > 0) {
            const uint32_t h = n >> 1;
            if (s.dstart[lo + h + 1] <= j) { lo += h + 1; n -= h + 1; } else n = h;
        }
        d = lo;
    }
    return ((uint64_t)d << s.kb) | ((s.rec[j] >> s.ib) & ((1ull << s.kb) - 1));
}

// cr_key_in from a record already loaded (v = s.rec[j])
__device__ __forceinline__ uint64_t cr_key_val(const CrStream& s, uint64_t v, uint64_t j, uint32_t d0, uint32_t d1) {
    uint32_t d = d0;
    if (d1 != d0) {
        uint32_t lo = d0, n = d1 - d0;
        while (n > 0) {
            const uint32_t h = n >> 1;
            if (s.dstart[lo + h + 1] <= j) { lo += h + 1; n -= h + 1; } else n = h;
        }
        d = lo;
    }
    return ((uint64_t)d << s.kb) | ((v >> s.ib) & ((1ull << s.kb) - 1));
}

// the digits of block b's first and last records into LDS (all threads call it; callers
// barrier before reading sd): thread t tests digit t's range, so the block pays one load
// latency instead of two dependent binary searches over dstart
__device__ __forceinline__ void cr_block_digits(const CrStream& s, uint64_t b, uint32_t* sd) {
    const uint64_t j0 = b * kCrBlk, j1 = (s.N < j0 + kCrBlk ? s.N : j0 + kCrBlk) - 1;
    for (uint32_t t = threadIdx.x; t < s.nd; t += blockDim.x) {
        const uint64_t a = s.dstart[t], e = s.dstart[t + 1];
        if (a <= j0 && j0 < e) sd[0] = t;
        if (a <= j1 && j1 < e) sd[1] = t;
    }
}

// per-block genome counts: gcnt[g * (nblk + 1) + b]
__global__ __launch_bounds__(kBlock) void cr_count_kernel(CrStream s, GenomeTable gt, uint64_t nblk,
                                                          uint32_t* __restrict__ gcnt) {
    __shared__ uint32_t c[kMaxG];
    const uint64_t b = blockIdx.x;
    if (threadIdx.x < kMaxG) c[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < kCrBlk; r += kBlock) {
        const uint64_t j = b * kCrBlk + r;
        if (j < s.N) atomicAdd(&c[genome_of(gt, cr_idx(s, j))], 1u);
    }
    __syncthreads();
    if ((int)threadIdx.x < gt.G) gcnt[(uint64_t)threadIdx.x * (nblk + 1) + b] = c[threadIdx.x];
}

// f(j, g, sml index) for every record of block b, in stream order per genome (stable)
template <typename F>
__device__ __forceinline__ void cr_block_ranks(const CrStream& s, const GenomeTable& gt, uint64_t b,
                                               const uint32_t* __restrict__ gscan, uint64_t nblk, F&& f) {
    __shared__ uint32_t base[kMaxG];
    __shared__ uint32_t wcnt[kBlock / 64][kMaxG];
    const int tid = threadIdx.x, wv = tid >> 6;
    if (tid < gt.G) base[tid] = gscan[(uint64_t)tid * (nblk + 1) + b];
    for (uint32_t r0 = 0; r0 < kCrBlk; r0 += kBlock) {
        for (int i = tid; i < (kBlock / 64) * kMaxG; i += kBlock) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        const uint64_t j = b * kCrBlk + r0 + tid;
        const bool valid = j < s.N;
        const uint32_t g = valid ? (uint32_t)genome_of(gt, cr_idx(s, j)) : 0u;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<6>(g, valid, &tot);
        if (valid && rk == 0) wcnt[wv][g] = tot;
        __syncthreads();
        if (valid) {
            uint32_t o = base[g] + rk;
            for (int w = 0; w < wv; ++w) o += wcnt[w][g];
            f(j, (int)g, (uint64_t)o);
        }
        __syncthreads();
        if (tid < gt.G) {
            uint32_t t = 0;
            for (int w = 0; w < kBlock / 64; ++w) t += wcnt[w][tid];
            base[tid] += t;
        }
        __syncthreads();   // wcnt is read above before the next round zeroes it
    }
}

// the G SortedMerLists as full keys: ck[base_g + sml index] = ckey
// (lbase: the genome-major bases of a stream holding part of every SML -- a sharded rank's
// key range; nullptr: gt.base)
__global__ __launch_bounds__(kBlock) void cr_ck_kernel(CrStream s, GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                       uint64_t nblk, const uint64_t* __restrict__ lbase,
                                                       uint64_t* __restrict__ ck) {
    cr_block_ranks(s, gt, blockIdx.x, gscan, nblk, [&](uint64_t j, int g, uint64_t i) {
        ck[(lbase ? lbase[g] : gt.base[g]) + i] = cr_key(s, j);
    });
}

// the G SortedMerLists as (genome << kbits | ckey, global index) pairs, genome-major
// (ParallelMemHash compat: the SMLs its chunking walks, from the MemHash path's sorted stream);
// sv / ck optional (the chunking reads the keys only; the tie replay and the MER_REPEAT_LIMIT
// plan need the rest)
__global__ __launch_bounds__(kBlock) void cr_partition_kernel(CrStream s, GenomeTable gt,
                                                              const uint32_t* __restrict__ gscan, uint64_t nblk,
                                                              int kbits, uint64_t* __restrict__ sk,
                                                              uint32_t* __restrict__ sv, uint64_t* __restrict__ ck) {
    __shared__ uint32_t sd[2];
    cr_block_digits(s, blockIdx.x, sd);   // (cr_block_ranks barriers before its first callback)
    cr_block_ranks(s, gt, blockIdx.x, gscan, nblk, [&](uint64_t j, int g, uint64_t i) {
        const uint64_t o = gt.base[g] + i, k = cr_key_in(s, j, sd[0], sd[1]);
        sk[o] = ((uint64_t)g << kbits) | k;
        if (sv) sv[o] = (uint32_t)cr_idx(s, j);
        if (ck) ck[o] = k;
    });
}

// ParallelMemHash's chunk-major stream as a stable partition of the sorted stream by chunk:
// a record's chunk is the last chunk whose start in its genome (cs[c * G + g]) is at or
// below its SML index.  The stream is ordered by (ckey, global index), i.e. inside a chunk by
// ckey, then genome, then SML order -- the order of the (chunk, ckey) sort of the SMLs when
// no equal-key run of a genome was reordered into std::sort order (the caller checks).
// Pass 1 counts (chunk, block) records, chunk-major (cnt[c * (nblk + 1) + b]); after an
// exclusive scan pass 2 writes key2 = chunk << kbits | ckey and the index at the scanned
// offset plus the record's stable rank inside its block.
constexpr uint32_t kCpChunks = 2048;   // chunks of the LDS form (more: the caller's radix sort)

__device__ __forceinline__ uint32_t compat_chunk_at(const uint64_t* __restrict__ cs, uint32_t nch, int G, int g,
                                                    uint64_t i) {
    uint32_t lo = 0, n = nch;   // chunks whose start is <= i
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (cs[(uint64_t)(lo + h) * G + g] <= i) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo ? lo - 1 : 0;
}

// (chunk, block) counts without reading the records: block b holds genome g's SML indices
// [gscan[g][b], gscan[g][b + 1]), chunk c takes [cs[c][g], cs[c + 1][g]) of them
__global__ __launch_bounds__(kBlock) void cr_chunk_count_kernel(GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                                uint64_t nblk, const uint64_t* __restrict__ cs,
                                                                uint32_t nch, uint32_t* __restrict__ cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const int G = gt.G;
    const uint64_t b = t / G;
    const int g = (int)(t % G);
    if (b >= nblk) return;
    uint64_t lo = gscan[(uint64_t)g * (nblk + 1) + b];
    const uint64_t hi = gscan[(uint64_t)g * (nblk + 1) + b + 1];
    if (lo >= hi) return;
    uint32_t c = compat_chunk_at(cs, nch, G, g, lo);
    while (lo < hi) {
        const uint64_t ce = c + 1 < nch ? cs[(uint64_t)(c + 1) * G + g] : ~0ull;
        const uint64_t e = ce < hi ? ce : hi;
        if (e > lo) atomicAdd(&cnt[(uint64_t)c * (nblk + 1) + b], (uint32_t)(e - lo));
        lo = e > lo ? e : lo;
        ++c;
    }
}

template <bool kWrite>
__global__ __launch_bounds__(kBlock) void cr_chunk_part_kernel(CrStream s, GenomeTable gt,
                                                               const uint32_t* __restrict__ gscan, uint64_t nblk,
                                                               const uint64_t* __restrict__ cs, uint32_t nch, int kbits,
                                                               uint32_t* __restrict__ cnt, uint64_t* __restrict__ key2,
                                                               uint32_t* __restrict__ idx) {
    __shared__ uint32_t gbase[kMaxG];
    __shared__ uint32_t gw[kBlock / 64][kMaxG];
    __shared__ uint32_t cbase[kCpChunks];
    __shared__ uint32_t cw[kBlock / 64][kCpChunks];   // stamp << 16 | count (no per-round zeroing)
    __shared__ uint32_t sd[2], s_cmin, s_cmax;
    const uint64_t b = blockIdx.x;
    const int tid = threadIdx.x, wv = tid >> 6, G = gt.G;
    if (kWrite) {   // one chunk for the whole block (the common case): its records keep their order
        if (tid == 0) {
            s_cmin = 0xFFFFFFFFu;
            s_cmax = 0;
        }
        cr_block_digits(s, b, sd);
        __syncthreads();
        if (tid < G) {
            const uint64_t lo = gscan[(uint64_t)tid * (nblk + 1) + b], hi = gscan[(uint64_t)tid * (nblk + 1) + b + 1];
            if (lo < hi) {
                atomicMin(&s_cmin, compat_chunk_at(cs, nch, G, tid, lo));
                atomicMax(&s_cmax, compat_chunk_at(cs, nch, G, tid, hi - 1));
            }
        }
        __syncthreads();
        if (s_cmin == s_cmax) {
            const uint32_t c = s_cmin;
            const uint64_t base = cnt[(uint64_t)c * (nblk + 1) + b], j0 = b * kCrBlk;
            for (uint32_t r = tid; r < kCrBlk; r += kBlock) {
                const uint64_t j = j0 + r;
                if (j >= s.N) break;
                key2[base + r] = ((uint64_t)c << kbits) | cr_key_in(s, j, sd[0], sd[1]);
                idx[base + r] = (uint32_t)cr_idx(s, j);
            }
            return;
        }
    }
    if (tid < G) gbase[tid] = gscan[(uint64_t)tid * (nblk + 1) + b];
    for (uint32_t c = tid; c < nch; c += kBlock) {
        cbase[c] = kWrite ? cnt[(uint64_t)c * (nblk + 1) + b] : 0u;
        for (int w = 0; w < kBlock / 64; ++w) cw[w][c] = 0;
    }
    uint32_t stamp = 0;
    for (uint32_t r0 = 0; r0 < kCrBlk; r0 += kBlock) {
        ++stamp;
        for (int i = tid; i < (kBlock / 64) * kMaxG; i += kBlock) (&gw[0][0])[i] = 0;
        __syncthreads();
        const uint64_t j = b * kCrBlk + r0 + tid;
        const bool valid = j < s.N;
        const uint32_t g = valid ? (uint32_t)genome_of(gt, cr_idx(s, j)) : 0u;
        uint32_t gtot;
        const uint32_t grk = wave_match_rank<6>(g, valid, &gtot);
        if (valid && grk == 0) gw[wv][g] = gtot;
        __syncthreads();
        uint32_t c = 0;
        if (valid) {
            uint32_t o = gbase[g] + grk;
            for (int w = 0; w < wv; ++w) o += gw[w][g];
            c = compat_chunk_at(cs, nch, G, (int)g, o);
        }
        uint32_t ctot;
        const uint32_t crk = wave_match_rank<11>(c, valid, &ctot);
        if (valid && crk == 0) {
            if (kWrite) cw[wv][c] = (stamp << 16) | ctot;
            else atomicAdd(&cbase[c], ctot);
        }
        __syncthreads();
        if (kWrite && valid) {
            uint32_t d = cbase[c] + crk;
            for (int w = 0; w < wv; ++w) {
                const uint32_t x = cw[w][c];
                d += (x >> 16) == (stamp & 0xFFFFu) ? (x & 0xFFFFu) : 0u;
            }
            key2[d] = ((uint64_t)c << kbits) | cr_key_in(s, j, sd[0], sd[1]);
            idx[d] = (uint32_t)cr_idx(s, j);
        }
        __syncthreads();
        if (valid && grk == 0) atomicAdd(&gbase[g], gtot);
        if (kWrite && valid && crk == 0) atomicAdd(&cbase[c], ctot);
        __syncthreads();
    }
    if (!kWrite)
        for (uint32_t c = tid; c < nch; c += kBlock) cnt[(uint64_t)c * (nblk + 1) + b] = cbase[c];
}

// masked keys with more than MER_REPEAT_LIMIT records: such a run holds a multiple of 1000,
// so only those positions look for their run's bounds (galloping) -- the first multiple
// of 1000 inside the run reports its key
__device__ __forceinline__ uint64_t cr_run_edge(const CrStream& s, uint64_t m, uint64_t v, int dir) {
    // last position from m in direction dir whose masked key is v
    uint64_t good = m, step = 1;
    for (;;) {
        const bool in = dir < 0 ? good >= step : good + step < s.N;
        if (!in) break;
        const uint64_t q = dir < 0 ? good - step : good + step;
        if ((cr_key(s, q) >> 1) != v) break;
        good = q;
        step <<= 1;
    }
    uint64_t lo = dir < 0 ? (good >= step ? good - step + 1 : 0) : good, hi = dir < 0 ? good : std::min(good + step, s.N);
    if (dir < 0) {   // first position in [lo, good] with key v
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if ((cr_key(s, mid) >> 1) == v) hi = mid; else lo = mid + 1;
        }
        return lo;
    }
    while (hi - lo > 1) {   // last position in [good, hi) with key v
        const uint64_t mid = lo + (hi - lo) / 2;
        if ((cr_key(s, mid) >> 1) == v) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void cr_cand_kernel(CrStream s, uint64_t* __restrict__ list,
                                                         unsigned long long* __restrict__ cnt, uint64_t cap) {
    const uint64_t m = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * restart::kRepeatLimit;
    if (m >= s.N) return;
    const uint64_t v = cr_key(s, m) >> 1;
    const uint64_t a = cr_run_edge(s, m, v, -1);
    if (m >= a + restart::kRepeatLimit) return;   // an earlier multiple of 1000 lies in the run
    const uint64_t b = cr_run_edge(s, m, v, +1);
    if (b - a + 1 <= restart::kRepeatLimit) return;
    const unsigned long long k = atomicAdd(cnt, 1ull);
    if (k < cap) list[k] = v;
}

// ---- ParallelMemHash compat: chunk starts from the sorted stream (no genome-major SMLs) ----
// compat_breaks_kernel / compat_find_kernel / compat_split_kernel (compat.hip) read the SMLs
// genome-major.  When no break walks back (the longest SML's record at k * CHUNK_SIZE starts
// its masked-key group, the common case), chunk k starts at k * CHUNK_SIZE there, and the rest
// needs few SML reads: the break mer b_k = SML_mx[k * CHUNK], the check on SML_mx[k * CHUNK - 1],
// and for FindMer in SML g only lb = #records of g with key < b_k and ub = #records <= b_k --
// a bsearch over a sorted list compares SML_g[mid] with b_k, i.e. mid with lb and ub.  An SML
// element is a select (gscan's blocks, then a block scan); lb / ub are stream bounds of b_k
// and the genomes' ranks there.  One workgroup per chunk start.  flags[0]: 1 a break walks
// back, 2 a split the bounds cannot decide; the caller then builds the SMLs.

// records of genome g in [j0, j) of block b, for every genome (cnt[kMaxG] in LDS, zeroed by
// the caller, barrier after)
__device__ __forceinline__ void cf_block_counts(const CrStream& s, const GenomeTable& gt, uint64_t j0, uint64_t j,
                                                uint32_t* cnt) {
    for (uint64_t x = j0 + threadIdx.x; x < j; x += kBlock) atomicAdd(&cnt[genome_of(gt, cr_idx(s, x))], 1u);
}

// stream position of SML_g[r] (all threads; result in *out after the last barrier)
__device__ __forceinline__ void cf_select(const CrStream& s, const GenomeTable& gt, const uint32_t* __restrict__ gscan,
                                          uint64_t nblk, int g, uint64_t r, uint32_t* s_cnt, uint64_t* s_b,
                                          uint64_t* out) {
    const uint32_t* gs = gscan + (uint64_t)g * (nblk + 1);
    if (threadIdx.x == 0) {   // last block b with gs[b] <= r
        uint64_t lo = 0, n = nblk;
        while (n > 0) {
            const uint64_t h = n >> 1;
            if (gs[lo + h + 1] <= r) { lo += h + 1; n -= h + 1; } else n = h;
        }
        *s_b = lo;
    }
    __syncthreads();
    const uint64_t b = *s_b;
    const uint64_t j0 = b * kCrBlk, j1 = s.N < j0 + kCrBlk ? s.N : j0 + kCrBlk;
    const uint32_t want = (uint32_t)(r - gs[b]);
    // thread t's 16 consecutive records: count, block scan, the owner finds the record
    constexpr uint32_t kPer = kCrBlk / kBlock;
    const uint64_t a = j0 + (uint64_t)threadIdx.x * kPer;
    uint32_t c = 0;
    for (uint32_t u = 0; u < kPer; ++u)
        if (a + u < j1) c += genome_of(gt, cr_idx(s, a + u)) == g ? 1u : 0u;
    s_cnt[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x < 64) {   // exclusive scan of the 256 counts by one wave, 4 per lane
        uint32_t v0 = s_cnt[4 * threadIdx.x], v1 = s_cnt[4 * threadIdx.x + 1], v2 = s_cnt[4 * threadIdx.x + 2],
                 v3 = s_cnt[4 * threadIdx.x + 3];
        const uint32_t t4 = v0 + v1 + v2 + v3;
        uint32_t inc = t4;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if ((int)threadIdx.x >= d) inc += t;
        }
        const uint32_t ex = inc - t4;
        s_cnt[4 * threadIdx.x] = ex;
        s_cnt[4 * threadIdx.x + 1] = ex + v0;
        s_cnt[4 * threadIdx.x + 2] = ex + v0 + v1;
        s_cnt[4 * threadIdx.x + 3] = ex + v0 + v1 + v2;
    }
    __syncthreads();
    const uint32_t e0 = s_cnt[threadIdx.x];
    if (want >= e0 && want < e0 + c) {
        uint32_t k = e0;
        for (uint32_t u = 0; u < kPer; ++u)
            if (a + u < j1 && genome_of(gt, cr_idx(s, a + u)) == g) {
                if (k == want) { *out = a + u; break; }
                ++k;
            }
    }
    __syncthreads();
}

// first stream position whose key is >= q
__device__ __forceinline__ uint64_t cf_lower(const CrStream& s, uint64_t q) {
    const uint64_t d = q >> s.kb;
    if (d >= s.nd) return s.N;
    const uint64_t kq = q & ((1ull << s.kb) - 1);
    uint64_t lo = s.dstart[d], n = s.dstart[d + 1] - lo;
    while (n > 0) {
        const uint64_t h = n >> 1;
        if (((s.rec[lo + h] >> s.ib) & ((1ull << s.kb) - 1)) < kq) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void compat_fast_chunks_kernel(CrStream s, GenomeTable gt,
                                                                    const uint32_t* __restrict__ gscan, uint64_t nblk,
                                                                    int mx, uint64_t chunk, int L,
                                                                    uint64_t* __restrict__ cs,
                                                                    uint32_t* __restrict__ flags) {
    __shared__ uint32_t s_cnt[kBlock];
    __shared__ uint32_t c_lo[kMaxG], c_hi[kMaxG];
    __shared__ uint64_t s_b, s_pos[2], s_P[2], s_und[kMaxG];
    __shared__ uint32_t s_nund;
    const uint32_t k = blockIdx.x + 1;
    const int G = gt.G;
    const uint64_t i = (uint64_t)k * chunk;
    cf_select(s, gt, gscan, nblk, mx, i, s_cnt, &s_b, &s_pos[0]);
    cf_select(s, gt, gscan, nblk, mx, i - 1, s_cnt, &s_b, &s_pos[1]);
    const uint64_t q = cr_key(s, s_pos[0]);
    if ((cr_key(s, s_pos[1]) >> 1) == (q >> 1)) {   // the break walks back: the caller's SML path
        if (threadIdx.x == 0) atomicOr(&flags[0], 1u);
        return;
    }
    if (threadIdx.x == 0) {
        s_P[0] = cf_lower(s, q);
        s_P[1] = cf_lower(s, q + 1);
    }
    if (threadIdx.x < kMaxG) {
        c_lo[threadIdx.x] = 0;
        c_hi[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) s_nund = 0;
    __syncthreads();
    const uint64_t P0 = s_P[0], P1 = s_P[1];
    const uint64_t b0 = P0 / kCrBlk, b1 = P1 / kCrBlk;
    cf_block_counts(s, gt, b0 * kCrBlk, P0, c_lo);
    cf_block_counts(s, gt, b1 * kCrBlk, P1, c_hi);
    __syncthreads();
    const int g = threadIdx.x;
    if (g < G && g != mx) {
    const uint64_t lb = (b0 < nblk ? gscan[(uint64_t)g * (nblk + 1) + b0] : gscan[(uint64_t)g * (nblk + 1) + nblk]) + c_lo[g];
    const uint64_t ub = (b1 < nblk ? gscan[(uint64_t)g * (nblk + 1) + b1] : gscan[(uint64_t)g * (nblk + 1) + nblk]) + c_hi[g];
    // compat_find_kernel's bsearch with SML_g[mid] <, ==, > q read as mid < lb, < ub, >= ub
    const uint64_t n = gt.n[g];
    uint64_t cur = 0;
    bool found = false;
    if (n != 0 && n >= (uint64_t)L) {
        uint64_t start = 0, end = n - (uint64_t)L;
        for (;;) {
            const uint64_t mid = (start + end) / 2;
            cur = mid;
            if (mid >= lb && mid < ub) break;
            if (mid < lb && mid < end) start = mid + 1;
            else if (mid >= ub && start < mid) end = mid - 1;
            else break;
        }
        found = cur >= lb && cur < ub;
        if (found) cur = (q == 0) ? 0 : cur + 1;
    }
    cs[(uint64_t)k * G + g] = cur;
    // compat_split_kernel's check SML_g[p - 1] == SML_g[p] at p = cur
    const uint64_t p = cur;
    if (p != 0 && p < gt.m[g]) {
        if (found) {
            if (p < ub) atomicOr(&flags[0], 2u);   // SML_g[p - 1] == q; SML_g[p] == q iff p < ub
        } else if (p != lb) {                      // (p == lb: SML_g[p - 1] < q < SML_g[p])
            s_und[atomicAdd(&s_nund, 1u)] = ((uint64_t)g << 56) | p;   // both on one side of q
        }
    }
    }
    if (g == mx) cs[(uint64_t)k * G + g] = i;
    __syncthreads();
    // the undecided ones: read both SML elements
    const uint32_t nu = s_nund;
    for (uint32_t u = 0; u < nu; ++u) {
        const int gu = (int)(s_und[u] >> 56);
        const uint64_t pu = s_und[u] & ((1ull << 56) - 1);
        cf_select(s, gt, gscan, nblk, gu, pu - 1, s_cnt, &s_b, &s_pos[0]);
        cf_select(s, gt, gscan, nblk, gu, pu, s_cnt, &s_b, &s_pos[1]);
        if (threadIdx.x == 0 && cr_key(s, s_pos[0]) == cr_key(s, s_pos[1])) atomicOr(&flags[0], 2u);
    }
}

// ---- ParallelMemHash compat: the chunk-major records straight from the sorted stream -----
// The chunk-major stream is the stable partition of the sorted stream by chunk (above).  A
// block boundary of the stream, R_g records of every genome g before it, is closed when no
// record before it has a higher chunk than one after it: max_g chunk(R_g - 1) <= min_g
// chunk(R_g).  Between two closed boundaries the records fill exactly their own position
// range.  Nearly every block has both boundaries closed and one chunk: its records stay in
// stream order.  The rest form units -- a block holding a chunk start, or a run of blocks
// whose inner boundaries are open (a chunk start's equal-key records split by a block edge:
// the longest genome's record opens chunk k, the others' close chunk k - 1) -- partitioned by
// chunk inside the unit.  compat_recs_kernel's packed records then come out of one pass over
// the stream, without the key2 / index arrays of the partition.  A unit above kCdUnit blocks
// or kCdSpan chunks, a group-key clash or a masked-key run above MER_REPEAT_LIMIT (a chunk
// might be cut: compat_truncate needs key2) set a flag bit; the caller then takes the
// partition + compat_recs path.
constexpr uint32_t kCdSpan = 32;   // chunks inside one unit
constexpr uint32_t kCdUnit = 64;   // blocks per unit

struct CdWs {   // workspace, nblk = cr_blocks(N)
    uint64_t* bedge;    // 2 nblk: key2 of block b's first and last output record
    uint32_t* pmax1;    // nblk + 1: 1 + highest chunk before boundary b (0: none)
    uint32_t* qmin;     // nblk + 1: lowest chunk after boundary b (~0: none)
    uint32_t* cfirst;   // nblk: block b's chunk range over its own records
    uint32_t* clast;
    uint32_t* units;    // 2 nblk: (first block, end block) of every unit
};

__host__ __device__ inline CdWs cd_ws(void* p, uint64_t nblk) {
    CdWs w;
    uint64_t* e = (uint64_t*)p;
    w.bedge = e;
    uint32_t* u = (uint32_t*)(e + 2 * nblk);
    w.pmax1 = u;
    w.qmin = u + (nblk + 1);
    w.cfirst = u + 2 * (nblk + 1);
    w.clast = w.cfirst + nblk;
    w.units = w.clast + nblk;
    return w;
}

// thread (b, g), b <= nblk: genome g's side of boundary b and of block b's chunk range
__global__ __launch_bounds__(kBlock) void cd_bounds_kernel(GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                           uint64_t nblk, const uint64_t* __restrict__ cs, uint32_t nch,
                                                           CdWs w) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const int G = gt.G;
    const uint64_t b = t / G;
    const int g = (int)(t % G);
    if (b > nblk) return;
    const uint32_t* gs = gscan + (uint64_t)g * (nblk + 1);
    const uint64_t R = gs[b], m = gs[nblk];
    if (R > 0) atomicMax(&w.pmax1[b], compat_chunk_at(cs, nch, G, g, R - 1) + 1u);
    if (R < m) {
        const uint32_t q = compat_chunk_at(cs, nch, G, g, R);
        atomicMin(&w.qmin[b], q);
        if (b < nblk && gs[b + 1] > R) {   // genome g has records in block b
            atomicMin(&w.cfirst[b], q);
            atomicMax(&w.clast[b], compat_chunk_at(cs, nch, G, g, gs[b + 1] - 1));
        }
    }
}

__device__ __forceinline__ bool cd_open(const CdWs& w, uint64_t b) {
    const uint32_t p1 = w.pmax1[b], q = w.qmin[b];
    return p1 != 0u && q != 0xFFFFFFFFu && p1 - 1u > q;
}

__device__ __forceinline__ uint64_t cd_rec(uint64_t k, int kbits, uint64_t idx) {
    return (compat_gid(k, kbits) << 33) | ((k & 1ull) << 32) | idx;
}

__device__ __forceinline__ bool cd_clash(uint64_t kp, uint64_t k, int kbits) {
    return (kp >> 1) != (k >> 1) && compat_gid(kp, kbits) == compat_gid(k, kbits);
}

// one workgroup per stream block: single-chunk blocks between closed boundaries written in
// stream order; a unit's first block lists the unit (flags[1] of them) for cd_unit_kernel
__global__ __launch_bounds__(kBlock) void cd_direct_kernel(CrStream s, uint64_t nblk, int kbits, CdWs w,
                                                           uint64_t* __restrict__ rec, uint32_t* __restrict__ flags) {
    __shared__ uint32_t sd[2];
    const uint64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const uint64_t j0 = b * kCrBlk, j1 = s.N < j0 + kCrBlk ? s.N : j0 + kCrBlk;
    cr_block_digits(s, b, sd);
    __syncthreads();
    // MER_REPEAT_LIMIT screen, inside the block: a masked-key run of more than 1000 records
    // holds two positions 500 apart of one block -- two multiples of 500, or the block's first
    // record and the one 500 on, or its last and the one 500 before (of a run crossing a block
    // edge, 501 or more records lie on one side).  Runs of 501-1000 may flag too (fallback).
    if (tid < 16) {
        uint64_t x = ~0ull;
        if (tid == 0) x = j0;
        else if (tid == 1) x = j1 >= j0 + 501 ? j1 - 501 : ~0ull;
        else x = ((j0 + 499) / 500 + (uint64_t)(tid - 2)) * 500;
        if (x >= j0 && x + 500 < j1 &&
            (cr_key_in(s, x, sd[0], sd[1]) >> 1) == (cr_key_in(s, x + 500, sd[0], sd[1]) >> 1))
            atomicOr(&flags[0], 4u);
    }
    if (cd_open(w, b)) return;   // inside a unit an earlier block heads
    const uint32_t c0 = w.cfirst[b], c1 = w.clast[b];
    if (c0 != c1 || cd_open(w, b + 1)) {
        if (tid == 0) {
            uint64_t e = b + 1;
            uint32_t lo = c0, hi = c1;
            while (e < nblk && cd_open(w, e) && e - b < kCdUnit) {
                lo = min(lo, w.cfirst[e]);
                hi = max(hi, w.clast[e]);
                ++e;
            }
            if (e < nblk && cd_open(w, e)) atomicOr(&flags[0], 1u);
            else if (hi - lo >= kCdSpan) atomicOr(&flags[0], 8u);
            else {
                const uint32_t u = atomicAdd(&flags[1], 1u);
                w.units[2 * u] = (uint32_t)b;
                w.units[2 * u + 1] = (uint32_t)e;
            }
        }
        return;
    }
    const uint64_t ch = (uint64_t)c0 << kbits;
    const uint32_t d0 = sd[0], d1 = sd[1];
    const uint64_t* __restrict__ src = s.rec;
    bool clash = false;
    // 4 records per thread per batch, loaded before any is stored; the predecessor of a
    // record (the clash check) from the lane below, lane 0 loads it
    constexpr int kU = 4;
    const int lane = tid & 63;
    for (uint64_t r0 = j0; r0 < j1; r0 += kU * kBlock) {
        uint64_t v[kU], vp[kU];
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t j = r0 + (uint64_t)u * kBlock + tid;
            v[u] = j < j1 ? src[j] : 0ull;
            vp[u] = (lane == 0 && j > j0 && j < j1) ? src[j - 1] : 0ull;
        }
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t j = r0 + (uint64_t)u * kBlock + tid;
            const uint64_t up = (uint64_t)__shfl_up((unsigned long long)v[u], 1, 64);
            if (j >= j1) continue;
            const uint64_t k = ch | cr_key_val(s, v[u], j, d0, d1);
            rec[j] = cd_rec(k, kbits, v[u] & ((1ull << s.ib) - 1));
            if (j > j0) clash |= cd_clash(ch | cr_key_val(s, lane ? up : vp[u], j - 1, d0, d1), k, kbits);
            if (j == j0) w.bedge[2 * b] = k;
            if (j + 1 == j1) w.bedge[2 * b + 1] = k;
        }
    }
    if (clash) atomicOr(&flags[0], 2u);
}

// the listed units (grid-stride): chunks from the genome ranks (kept per record in sc), a
// stable partition by chunk over the unit, key2 by output position in k2 for the clash check
__global__ __launch_bounds__(kBlock) void cd_unit_kernel(CrStream s, GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                         uint64_t nblk, const uint64_t* __restrict__ cs, uint32_t nch,
                                                         int kbits, CdWs w, uint64_t* __restrict__ rec,
                                                         uint64_t* __restrict__ k2, uint8_t* __restrict__ sc,
                                                         uint32_t* __restrict__ flags) {
    __shared__ uint32_t cpre[kCdSpan];
    __shared__ uint32_t wc[kBlock / 64][kCdSpan];
    __shared__ uint32_t sd[2], s_c0;
    const int tid = threadIdx.x, wv = tid >> 6, G = gt.G;
    const uint32_t nu = flags[1];
    for (uint32_t li = blockIdx.x; li < nu; li += gridDim.x) {
        const uint64_t b0 = w.units[2 * li], b1 = w.units[2 * li + 1];
        const uint64_t u0 = b0 * kCrBlk, u1 = s.N < b1 * kCrBlk ? s.N : b1 * kCrBlk;
        __syncthreads();   // the previous unit's LDS reads are done
        if (tid < (int)kCdSpan) cpre[tid] = 0;
        if (tid == 0) {
            uint32_t c0 = w.cfirst[b0];
            for (uint64_t b = b0 + 1; b < b1; ++b) c0 = min(c0, w.cfirst[b]);
            s_c0 = c0;
        }
        __syncthreads();
        const uint32_t c0 = s_c0;
        for (uint64_t b = b0; b < b1; ++b)
            cr_block_ranks(s, gt, b, gscan, nblk, [&](uint64_t j, int g, uint64_t o) {
                const uint32_t c = compat_chunk_at(cs, nch, G, g, o) - c0;
                sc[j] = (uint8_t)c;
                atomicAdd(&cpre[c], 1u);
            });
        __syncthreads();
        if (tid == 0) {
            uint32_t a = 0;
            for (uint32_t c = 0; c < kCdSpan; ++c) {
                const uint32_t x = cpre[c];
                cpre[c] = a;
                a += x;
            }
        }
        for (uint64_t b = b0; b < b1; ++b) {
            __syncthreads();   // (sd of the previous block read)
            cr_block_digits(s, b, sd);
            const uint64_t j0 = b * kCrBlk, j1 = s.N < j0 + kCrBlk ? s.N : j0 + kCrBlk;
            for (uint64_t r0 = j0; r0 < j1; r0 += kBlock) {
                for (int i = tid; i < (kBlock / 64) * (int)kCdSpan; i += kBlock) (&wc[0][0])[i] = 0;
                __syncthreads();
                const uint64_t j = r0 + tid;
                const bool valid = j < j1;
                const uint32_t c = valid ? sc[j] : 0u;
                uint32_t tot;
                const uint32_t rk = wave_match_rank<5>(c, valid, &tot);
                if (valid && rk == 0) wc[wv][c] = tot;
                __syncthreads();
                if (valid) {
                    uint32_t d = cpre[c] + rk;
                    for (int x = 0; x < wv; ++x) d += wc[x][c];
                    const uint64_t k = ((uint64_t)(c0 + c) << kbits) | cr_key_in(s, j, sd[0], sd[1]);
                    k2[u0 + d] = k;
                    rec[u0 + d] = cd_rec(k, kbits, cr_idx(s, j));
                }
                __syncthreads();
                if (valid && rk == 0) atomicAdd(&cpre[c], tot);
            }
        }
        __syncthreads();   // (k2 of the whole unit written: same workgroup, global memory)
        bool clash = false;
        for (uint64_t p = u0 + 1 + tid; p < u1; p += kBlock) clash |= cd_clash(k2[p - 1], k2[p], kbits);
        if (clash) atomicOr(&flags[0], 2u);
        for (uint64_t b = b0 + tid; b < b1; b += kBlock) {
            const uint64_t j0 = b * kCrBlk, j1 = s.N < j0 + kCrBlk ? s.N : j0 + kCrBlk;
            w.bedge[2 * b] = k2[j0];
            w.bedge[2 * b + 1] = k2[j1 - 1];
        }
    }
}

// the clash check across block edges
__global__ __launch_bounds__(kBlock) void cd_edges_kernel(uint64_t nblk, int kbits, CdWs w,
                                                          uint32_t* __restrict__ flags) {
    const uint64_t b = (uint64_t)blockIdx.x * kBlock + threadIdx.x + 1;
    if (b >= nblk) return;
    if (cd_clash(w.bedge[2 * b - 1], w.bedge[2 * b], kbits)) atomicOr(&flags[0], 2u);
}

// live[j - lo] for the records [lo, hi) of one chunk: SML index >= its phase's start point
__global__ __launch_bounds__(kBlock) void cr_live_kernel(CrStream s, GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                         uint64_t nblk, uint64_t b0, uint64_t lo, uint64_t hi,
                                                         const uint64_t* __restrict__ rkey, uint64_t R,
                                                         const uint64_t* __restrict__ rS,
                                                         const uint64_t* __restrict__ S0, const uint64_t* __restrict__ goff,
                                                         uint32_t* __restrict__ live) {
    const int G = gt.G;
    cr_block_ranks(s, gt, b0 + blockIdx.x, gscan, nblk, [&](uint64_t j, int g, uint64_t i) {
        if (j < lo || j >= hi) return;
        if (goff) i += goff[g];   // a sharded rank: SML indices below its key range
        const uint64_t v = cr_key(s, j) >> 1;
        uint64_t a = 0, n = R;   // phase = restart keys <= v
        while (n > 0) {
            const uint64_t h = n >> 1;
            if (rkey[a + h] <= v) { a += h + 1; n -= h + 1; } else n = h;
        }
        const uint64_t sp = a == 0 ? S0[g] : rS[(a - 1) * (uint64_t)G + g];
        live[j - lo] = i >= sp ? 1u : 0u;
    });
}

// straddled runs: start point s of genome g inside a run of equal keys -> {g, lo, hi}
__global__ __launch_bounds__(kBlock) void cr_runs_kernel(const uint64_t* __restrict__ ck, GenomeTable gt,
                                                         const uint64_t* __restrict__ sp, uint64_t rows,
                                                         uint64_t* __restrict__ runs, unsigned long long* __restrict__ nr,
                                                         uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const int G = gt.G;
    if (i >= rows * (uint64_t)G) return;
    const int g = (int)(i % (uint64_t)G);
    const uint64_t s = sp[i], m = gt.m[g];
    if (s == 0 || s >= m) return;
    const uint64_t* a = ck + gt.base[g];
    const uint64_t k = a[s];
    if (a[s - 1] != k) return;
    uint64_t lo = s - 1, hi = s + 1;
    while (lo > 0 && a[lo - 1] == k) --lo;
    while (hi < m && a[hi] == k) ++hi;
    const unsigned long long q = atomicAdd(nr, 1ull);
    if (q < cap) {
        runs[3 * q] = (uint64_t)g;
        runs[3 * q + 1] = lo;
        runs[3 * q + 2] = hi;
    }
}

// A sharded rank's straddled runs: it holds SML indices [goff[g], goff[g] + gn[g]) of genome
// g at ck[lbase[g] ..]; a start point strictly inside that range (its predecessor is held
// too, so a run of equal full keys can straddle it) -> {g, lo, hi} in global SML indices
__global__ __launch_bounds__(kBlock) void cr_druns_kernel(const uint64_t* __restrict__ ck, int G,
                                                          const uint64_t* __restrict__ lbase,
                                                          const uint64_t* __restrict__ goff,
                                                          const uint64_t* __restrict__ gn,
                                                          const uint64_t* __restrict__ sp, uint64_t rows,
                                                          uint64_t* __restrict__ runs,
                                                          unsigned long long* __restrict__ nr, uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= rows * (uint64_t)G) return;
    const int g = (int)(i % (uint64_t)G);
    const uint64_t o = goff[g], n = gn[g], s = sp[i];
    if (s <= o || s - o >= n) return;
    const uint64_t* a = ck + lbase[g];
    const uint64_t ls = s - o, k = a[ls];
    if (a[ls - 1] != k) return;
    uint64_t lo = ls - 1, hi = ls + 1;
    while (lo > 0 && a[lo - 1] == k) --lo;
    while (hi < n && a[hi] == k) ++hi;
    const unsigned long long q = atomicAdd(nr, 1ull);
    if (q < cap) {
        runs[3 * q] = (uint64_t)g;
        runs[3 * q + 1] = o + lo;
        runs[3 * q + 2] = o + hi;
    }
}

// A sharded rank's straddled run q (genome g, global slots [lo, hi)): its records, in stream
// order, take the ids of the std::sort order, V[vofs[q] + r] (positions in the genome),
// computed on the rank that replayed genome g's sort; one lane per run
__global__ void cr_dtie_write_kernel(CrStream s, GenomeTable gt, const uint64_t* __restrict__ runs, uint64_t nrun,
                                     const uint64_t* __restrict__ ck, const uint64_t* __restrict__ lbase,
                                     const uint64_t* __restrict__ goff, const uint32_t* __restrict__ V,
                                     const uint64_t* __restrict__ vofs, uint64_t* __restrict__ rec) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrun) return;
    const int g = (int)runs[3 * q];
    const uint64_t lo = runs[3 * q + 1], hi = runs[3 * q + 2];
    const uint64_t key = ck[lbase[g] + (lo - goff[g])];
    uint64_t a = 0, n = s.N;   // first stream record with key >= key
    while (n > 0) {
        const uint64_t h = n >> 1;
        if (cr_key(s, a + h) < key) { a += h + 1; n -= h + 1; } else n = h;
    }
    const uint32_t* v = V + vofs[q];
    uint64_t r = 0;
    for (uint64_t j = a; j < s.N && r < hi - lo && cr_key(s, j) == key; ++j) {
        if (genome_of(gt, cr_idx(s, j)) != g) continue;
        rec[j] = (rec[j] & ~((1ull << s.ib) - 1)) | (gt.base[g] + v[r]);
        ++r;
    }
}

// LogProgress on genome-major SMLs (the pair path's restart workspace): the masked key of
// SML index e of genome g for every query g << 56 | e
__global__ __launch_bounds__(kBlock) void cr_ck_query_kernel(const uint64_t* __restrict__ ck, GenomeTable gt,
                                                             const uint64_t* __restrict__ q, uint64_t nq,
                                                             uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq) return;
    const int g = (int)(q[i] >> 56);
    out[i] = ck[gt.base[g] + (q[i] & ((1ull << 56) - 1))] >> 1;
}

// Repeat tolerance (every run of equal keys in std::sort order): every record of genome g in
// a flagged run (the tie replay's scanned slot flags ts) takes the id at its SML slot, V[i]
// (positions in the genome).  Ids move only inside genome g, so gscan stays valid.
__global__ __launch_bounds__(kBlock) void cr_tie_all_kernel(CrStream s, GenomeTable gt,
                                                            const uint32_t* __restrict__ gscan, uint64_t nblk, int g,
                                                            const uint32_t* __restrict__ ts,
                                                            const uint32_t* __restrict__ V, uint64_t* rec) {
    cr_block_ranks(s, gt, blockIdx.x, gscan, nblk, [&](uint64_t j, int gg, uint64_t i) {
        if (gg != g || ts[i + 1] == ts[i]) return;
        rec[j] = (rec[j] & ~((1ull << s.ib) - 1)) | (gt.base[g] + V[i]);
    });
}

// Sharded repeat tolerance: a rank's pair flags of its SML parts (slot i of genome g flags the
// pair i, i + 1 of equal full keys; runs never straddle two ranks' key ranges), written at
// out[gofs[g] + i], and the id rewrite from the replayed order: V[vofs[g] + i] (~0: a slot
// outside every run keeps its id)
__global__ __launch_bounds__(kBlock) void cr_pair_flags_kernel(const uint64_t* __restrict__ ck, int G,
                                                               const uint64_t* __restrict__ lbase,
                                                               const uint64_t* __restrict__ gofs,
                                                               uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    int g = 0;
    for (int k = 1; k < G; ++k) g += (j >= lbase[k]) ? 1 : 0;
    const uint64_t i = j - lbase[g];
    out[gofs[g] + i] = (j + 1 < lbase[g + 1] && ck[j] == ck[j + 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void cr_tie_vals_kernel(CrStream s, GenomeTable gt,
                                                             const uint32_t* __restrict__ gscan, uint64_t nblk,
                                                             const uint64_t* __restrict__ vofs,
                                                             const uint32_t* __restrict__ V, uint64_t* rec) {
    cr_block_ranks(s, gt, blockIdx.x, gscan, nblk, [&](uint64_t j, int g, uint64_t i) {
        const uint32_t v = V[vofs[g] + i];
        if (v != 0xFFFFFFFFu) rec[j] = (rec[j] & ~((1ull << s.ib) - 1)) | (gt.base[g] + v);
    });
}

// K[pos] = key of genome g's seed-mer pos (the tie replay's position order)
__global__ __launch_bounds__(kBlock) void cr_kpos_kernel(CrStream s, GenomeTable gt, int g, uint64_t* __restrict__ K) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= s.N) return;
    const uint64_t gi = cr_idx(s, j);
    if (genome_of(gt, gi) != g) return;
    K[gi - gt.base[g]] = cr_key(s, j);
}

// the records of a straddled run of genome g (slots [lo, hi), key ck) take the ids of the
// std::sort order (V: positions at the slots); one lane per run
__global__ void cr_tie_write_kernel(CrStream s, GenomeTable gt, int g, const uint64_t* __restrict__ runs, uint64_t nrun,
                                    const uint64_t* __restrict__ ck, const uint32_t* __restrict__ V,
                                    uint64_t* __restrict__ rec) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrun || (int)runs[3 * q] != g) return;
    const uint64_t lo = runs[3 * q + 1], hi = runs[3 * q + 2];
    const uint64_t key = ck[gt.base[g] + lo];
    uint64_t a = 0, n = s.N;   // first stream record with key >= key
    while (n > 0) {
        const uint64_t h = n >> 1;
        if (cr_key(s, a + h) < key) { a += h + 1; n -= h + 1; } else n = h;
    }
    uint64_t r = 0;
    for (uint64_t j = a; j < s.N && r < hi - lo && cr_key(s, j) == key; ++j) {
        if (genome_of(gt, cr_idx(s, j)) != g) continue;
        const uint64_t gi = gt.base[g] + V[lo + r];
        rec[j] = (rec[j] & ~((1ull << s.ib) - 1)) | gi;
        ++r;
    }
}

// LogProgress: the masked key of the e-th record of genome g in stream order (= its SML
// index e) for every query q = g << 56 | e: the block holding it from the genome's block
// prefix counts, then a walk over that block's records
__global__ __launch_bounds__(kBlock) void cr_query_kernel(CrStream s, GenomeTable gt, const uint32_t* __restrict__ gscan,
                                                          uint64_t nblk, const uint64_t* __restrict__ q, uint64_t nq,
                                                          uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq) return;
    const int g = (int)(q[i] >> 56);
    const uint64_t e = q[i] & ((1ull << 56) - 1);
    const uint32_t* c = gscan + (uint64_t)g * (nblk + 1);   // exclusive prefix counts per block
    uint64_t lo = 0, n = nblk;                              // last block b with c[b] <= e
    while (n > 0) {
        const uint64_t h = n >> 1;
        if (c[lo + h] <= e) { lo += h + 1; n -= h + 1; } else n = h;
    }
    const uint64_t b = lo - 1;
    uint64_t r = e - c[b];
    uint64_t key = ~0ull;
    for (uint64_t j = b * kCrBlk; j < s.N && j < (b + 1) * kCrBlk; ++j) {
        if (genome_of(gt, cr_idx(s, j)) != g) continue;
        if (r == 0) { key = cr_key(s, j) >> 1; break; }
        --r;
    }
    out[i] = key;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void cr_compact_kernel(const T* __restrict__ src, const uint32_t* __restrict__ live,
                                                            const uint32_t* __restrict__ pos, uint64_t n,
                                                            T* __restrict__ dst) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < n && live[j]) dst[pos[j]] = src[j];
}

inline dim3 cr_grid(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace

uint64_t cr_blocks(uint64_t N) { return (N + kCrBlk - 1) / kCrBlk; }

hipError_t launch_cr_counts(const CrStream& s, const GenomeTable& gt, uint32_t* gcnt, void* d_scan_tmp,
                            hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    hipError_t e = hipMemsetAsync(gcnt, 0, (size_t)gt.G * (nblk + 1) * 4, st);
    if (e != hipSuccess || nblk == 0) return e;
    hipLaunchKernelGGL(cr_count_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, nblk, gcnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    for (int g = 0; g < gt.G; ++g)
        if ((e = exclusive_scan_u32(gcnt + (uint64_t)g * (nblk + 1), nblk + 1, d_scan_tmp, nullptr, st)) != hipSuccess)
            return e;
    return hipSuccess;
}

hipError_t launch_cr_partition(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int kbits, uint64_t* sk,
                               uint32_t* sv, uint64_t* ck, hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_partition_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, gscan, nblk, kbits, sk,
                       sv, ck);
    return hipGetLastError();
}

size_t cr_chunk_part_cnt_words(uint64_t N, uint32_t nch) { return (size_t)nch * (cr_blocks(N) + 1); }

bool cr_chunk_part_fits(uint64_t N, uint32_t nch) {
    return nch <= kCpChunks && cr_chunk_part_cnt_words(N, nch) < (1ull << 31);
}

hipError_t launch_cr_chunk_part(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* cs,
                                uint32_t nch, int kbits, uint32_t* cnt, void* d_scan_tmp, uint64_t* key2, uint32_t* idx,
                                hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    if (nblk == 0) return hipSuccess;
    if (!cr_chunk_part_fits(s.N, nch)) return hipErrorInvalidValue;
    const size_t words = cr_chunk_part_cnt_words(s.N, nch);
    hipError_t e = hipMemsetAsync(cnt, 0, words * 4, st);
    if (e != hipSuccess) return e;
    const uint64_t pairs = nblk * (uint64_t)gt.G;
    hipLaunchKernelGGL(cr_chunk_count_kernel, dim3((unsigned)((pairs + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, gt,
                       gscan, nblk, cs, nch, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(cnt, words, d_scan_tmp, nullptr, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(cr_chunk_part_kernel<true>, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, gscan, nblk, cs,
                       nch, kbits, cnt, key2, idx);
    return hipGetLastError();
}

hipError_t launch_compat_fast_chunks(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int mx,
                                    uint64_t chunk, int L, uint32_t nch, uint64_t* cs, uint32_t* flags, hipStream_t st) {
    hipError_t e = hipMemsetAsync(flags, 0, 4, st);
    if (e != hipSuccess || nch <= 1) return e;
    hipLaunchKernelGGL(compat_fast_chunks_kernel, dim3(nch - 1), dim3(kBlock), 0, st, s, gt, gscan, cr_blocks(s.N), mx,
                       chunk, L, cs, flags);
    return hipGetLastError();
}

size_t cr_direct_ws_bytes(uint64_t N) {
    const uint64_t nblk = cr_blocks(N);
    return (size_t)nblk * 16 + (size_t)(6 * nblk + 2) * 4 + 64;
}

hipError_t launch_cr_compat_direct(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* cs,
                                   uint32_t nch, int kbits, uint64_t* rec, uint64_t* k2, uint8_t* sc, void* ws,
                                   uint32_t* flags, hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    hipError_t e = hipMemsetAsync(flags, 0, 8, st);
    if (e != hipSuccess || nblk == 0) return e;
    const CdWs w = cd_ws(ws, nblk);
    // pmax1 = 0, qmin = ~0, cfirst = ~0, clast = 0
    if ((e = hipMemsetAsync(w.pmax1, 0, (nblk + 1) * 4, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.qmin, 0xFF, (2 * nblk + 1) * 4, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.clast, 0, nblk * 4, st)) != hipSuccess) return e;
    const uint64_t pairs = (nblk + 1) * (uint64_t)gt.G;
    hipLaunchKernelGGL(cd_bounds_kernel, dim3((unsigned)((pairs + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, gt, gscan,
                       nblk, cs, nch, w);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(cd_direct_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, nblk, kbits, w, rec, flags);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const unsigned ugrid = (unsigned)std::min<uint64_t>(nblk, 1024);
    hipLaunchKernelGGL(cd_unit_kernel, dim3(ugrid), dim3(kBlock), 0, st, s, gt, gscan, nblk, cs, nch, kbits, w, rec,
                       k2, sc, flags);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (nblk > 1)
        hipLaunchKernelGGL(cd_edges_kernel, dim3((unsigned)((nblk - 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, nblk,
                           kbits, w, flags);
    return hipGetLastError();
}

hipError_t launch_cr_ck(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, uint64_t* ck, hipStream_t st,
                        const uint64_t* lbase) {
    const uint64_t nblk = cr_blocks(s.N);
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_ck_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, gscan, nblk, lbase, ck);
    return hipGetLastError();
}

hipError_t launch_cr_cands(const CrStream& s, uint64_t* list, unsigned long long* cnt, uint64_t cap, hipStream_t st) {
    hipError_t e = hipMemsetAsync(cnt, 0, 8, st);
    if (e != hipSuccess || s.N == 0) return e;
    hipLaunchKernelGGL(cr_cand_kernel, cr_grid((s.N + restart::kRepeatLimit - 1) / restart::kRepeatLimit), dim3(kBlock),
                       0, st, s, list, cnt, cap);
    return hipGetLastError();
}

hipError_t launch_cr_runs(const uint64_t* ck, const GenomeTable& gt, const uint64_t* sp, uint64_t rows, uint64_t* runs,
                          unsigned long long* nr, uint64_t cap, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_runs_kernel, cr_grid(rows * (uint64_t)gt.G), dim3(kBlock), 0, st, ck, gt, sp, rows, runs, nr,
                       cap);
    return hipGetLastError();
}

hipError_t launch_cr_druns(const uint64_t* ck, int G, const uint64_t* lbase, const uint64_t* goff, const uint64_t* gn,
                           const uint64_t* sp, uint64_t rows, uint64_t* runs, unsigned long long* nr, uint64_t cap,
                           hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_druns_kernel, cr_grid(rows * (uint64_t)G), dim3(kBlock), 0, st, ck, G, lbase, goff, gn, sp,
                       rows, runs, nr, cap);
    return hipGetLastError();
}

hipError_t launch_cr_dtie_write(const CrStream& s, const GenomeTable& gt, const uint64_t* runs, uint64_t nrun,
                                const uint64_t* ck, const uint64_t* lbase, const uint64_t* goff, const uint32_t* V,
                                const uint64_t* vofs, uint64_t* rec, hipStream_t st) {
    if (nrun == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_dtie_write_kernel, dim3((unsigned)((nrun + 63) / 64)), dim3(64), 0, st, s, gt, runs, nrun,
                       ck, lbase, goff, V, vofs, rec);
    return hipGetLastError();
}

hipError_t launch_cr_tie_all(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int g, const uint32_t* ts,
                             const uint32_t* V, uint64_t* rec, hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_tie_all_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, gscan, nblk, g, ts, V, rec);
    return hipGetLastError();
}

hipError_t launch_cr_pair_flags(const uint64_t* ck, int G, const uint64_t* lbase, const uint64_t* gofs, uint64_t n,
                                uint32_t* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_pair_flags_kernel, cr_grid(n), dim3(kBlock), 0, st, ck, G, lbase, gofs, n, out);
    return hipGetLastError();
}

hipError_t launch_cr_tie_vals(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* vofs,
                              const uint32_t* V, uint64_t* rec, hipStream_t st) {
    const uint64_t nblk = cr_blocks(s.N);
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_tie_vals_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, s, gt, gscan, nblk, vofs, V, rec);
    return hipGetLastError();
}

hipError_t launch_cr_kpos(const CrStream& s, const GenomeTable& gt, int g, uint64_t* K, hipStream_t st) {
    if (s.N == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_kpos_kernel, cr_grid(s.N), dim3(kBlock), 0, st, s, gt, g, K);
    return hipGetLastError();
}

hipError_t launch_cr_ck_query(const uint64_t* ck, const GenomeTable& gt, const uint64_t* q, uint64_t nq, uint64_t* out,
                              hipStream_t st) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_ck_query_kernel, cr_grid(nq), dim3(kBlock), 0, st, ck, gt, q, nq, out);
    return hipGetLastError();
}

hipError_t launch_cr_query(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* q, uint64_t nq,
                           uint64_t* out, hipStream_t st) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_query_kernel, cr_grid(nq), dim3(kBlock), 0, st, s, gt, gscan, cr_blocks(s.N), q, nq, out);
    return hipGetLastError();
}

hipError_t launch_cr_tie_write(const CrStream& s, const GenomeTable& gt, int g, const uint64_t* runs, uint64_t nrun,
                               const uint64_t* ck, const uint32_t* V, uint64_t* rec, hipStream_t st) {
    if (nrun == 0) return hipSuccess;
    hipLaunchKernelGGL(cr_tie_write_kernel, dim3((unsigned)((nrun + 63) / 64)), dim3(64), 0, st, s, gt, g, runs, nrun,
                       ck, V, rec);
    return hipGetLastError();
}

// live records of chunk [lo, hi) compacted (order kept) into dst; *d_total = how many;
// bucket starts (chunk-relative, nb + 1) mapped through the scan into dst_bstart
hipError_t launch_cr_live_compact(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, uint64_t lo,
                                  uint64_t hi, const uint64_t* rkey, uint64_t R, const uint64_t* rS, const uint64_t* S0,
                                  uint32_t* live, uint32_t* pos, void* d_scan_tmp, uint64_t* dst,
                                  const uint32_t* bstart, uint32_t nb, uint32_t* dst_bstart, uint32_t* d_total,
                                  hipStream_t st, const uint64_t* goff) {
    const uint64_t n = hi - lo;
    const uint64_t nblk = cr_blocks(s.N);
    const uint64_t b0 = lo / kCrBlk, b1 = (hi + kCrBlk - 1) / kCrBlk;
    hipError_t e = hipMemsetAsync(live + n, 0, 4, st);
    if (e != hipSuccess) return e;
    if (n) {
        hipLaunchKernelGGL(cr_live_kernel, dim3((unsigned)(b1 - b0)), dim3(kBlock), 0, st, s, gt, gscan, nblk, b0, lo,
                           hi, rkey, R, rS, S0, goff, live);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = hipMemcpyAsync(pos, live, (n + 1) * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(pos, n + 1, d_scan_tmp, d_total, st)) != hipSuccess) return e;
    if (n) {
        hipLaunchKernelGGL(cr_compact_kernel<uint64_t>, cr_grid(n), dim3(kBlock), 0, st, s.rec + lo, live, pos, n, dst);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return launch_map_starts(bstart, nb, pos, dst_bstart, st);
}

}  // namespace mums
