// match_device.h -- MatchHashEntry arithmetic on gfx950 registers (rows A8-A10).
//
// A match lives in registers as {len, offset, mersize, s[MG]} with MG a
// compile-time bound (all loops fully unrolled: no runtime-indexed register
// arrays, which would spill to scratch).  Genomes G..MG-1 hold 0 (NO_MATCH),
// which is neutral for every function below.
#pragma once

#include <type_traits>

#include "mums_internal.h"
#include "seed_device.h"

namespace mums {

template <int MG>
struct Mhe {
    int64_t len;
    int64_t offset;
    int64_t mersize;  // L for probes (MemHash.cpp:172), 0 for stored entries (MatchHashEntry.cpp:122)
    int64_t s[MG];    // signed 1-based starts, 0 = NO_MATCH
};

// FirstStart (HybridAbstractMatch.h:121-129)
template <int MG>
__device__ __forceinline__ int first_start(const Mhe<MG>& m) {
    int f = MG;
    #pragma unroll
    for (int g = MG - 1; g >= 0; --g) f = (m.s[g] != 0) ? g : f;
    return f;
}

template <int MG>
__device__ __forceinline__ int64_t start_at(const Mhe<MG>& m, int i) {
    int64_t v = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) v = (g == i) ? m.s[g] : v;
    return v;
}

// Contains: does a contain b (MatchHashEntry.cpp:164-200)
template <int MG>
__device__ __forceinline__ bool mhe_contains(const Mhe<MG>& a, const Mhe<MG>& b) {
    if (a.offset != b.offset) return false;
    const int i = first_start(b);
    const int64_t ai = start_at(a, i), bi = start_at(b, i);
    if (ai == 0) return false;
    const int64_t diff = bi - ai;
    if (diff < 0 || (uint64_t)a.len < (uint64_t)(b.len + diff)) return false;
    const int64_t diff_rc = b.len - a.len + diff;
    bool ok = true;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        if (g <= i) continue;
        const int64_t di = b.s[g] - a.s[g];
        if (b.s[g] == 0 && a.s[g] == 0) continue;
        if (b.s[g] < 0 && diff_rc == di) continue;
        if (diff != di) ok = false;
    }
    return ok;
}

// strict_start_lessthan_ptr (MatchHashEntry.cpp:48-69)
template <int MG>
__device__ __forceinline__ bool mhe_strict_lt(const Mhe<MG>& a, const Mhe<MG>& b) {
    const int start_diff = first_start(a) - first_start(b);
    if (start_diff == 0) {
        int res = -1;  // -1 undecided, 0 false, 1 true
        #pragma unroll
        for (int g = 0; g < MG; ++g) {
            int64_t as = a.s[g], bs = b.s[g];
            if (as < 0) as = -as + a.len - a.mersize;
            if (bs < 0) bs = -bs + b.len - b.mersize;
            const int64_t d = as - bs;
            if (res < 0 && d != 0) res = d < 0 ? 1 : 0;
        }
        if (res >= 0) return res == 1;
    }
    return start_diff < 0;
}

// MheCompare (MatchHashEntry.h:121-143)
template <int MG>
__device__ __forceinline__ bool mhe_less(const Mhe<MG>& a, const Mhe<MG>& b) {
    const int fa = first_start(a), fb = first_start(b);
    if (fa > fb) return true;
    if (fa != fb) return false;
    int res = -1;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const bool az = a.s[g] == 0, bz = b.s[g] == 0;
        if (res < 0 && az && !bz) res = 1;
        if (res < 0 && !az && bz) res = 0;
    }
    if (res >= 0) return res == 1;
    if (mhe_contains(a, b) || mhe_contains(b, a)) return false;
    return mhe_strict_lt(a, b);
}

// stored entry layout in the pool: int64 [len, offset, s_0 .. s_{G-1}]
template <int MG>
__device__ __forceinline__ void load_entry(const int64_t* __restrict__ pool, uint32_t id, int G, Mhe<MG>& e) {
    const int64_t* p = pool + (uint64_t)id * (uint64_t)(G + 2);
    e.len = p[0];
    e.offset = p[1];
    e.mersize = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) e.s[g] = (g < G) ? p[2 + g] : 0;
}

// std::lower_bound over table ids[0..t) (libstdc++: half = len >> 1, middle = first + half)
template <int MG>
__device__ __forceinline__ uint32_t lower_bound_tbl(const uint32_t* tbl, uint32_t t, const int64_t* __restrict__ pool,
                                                   int G, const Mhe<MG>& val) {
    uint32_t first = 0, len = t;
    Mhe<MG> e;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        load_entry(pool, tbl[mid], G, e);
        if (mhe_less(e, val)) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

// Build the seed probe of a masked-key group whose first record in the sorted
// stream is h (records of the group lie in [h, end)).
// MemHash::EnumerateMatches (MemHash.cpp:139-162) acceptance with enum_tol <= 1,
// HashMatch (:167-187) / MaskedMemHash::HashMatch (MaskedMemHash.cpp:38-63),
// SetDirection (:189-203), CalculateOffset (MatchHashEntry.cpp:141-160).
// Returns false when the group yields no AddHashEntry call.
// *gsize receives the group size (counted up to kRepeatLimit + 1).
template <int MG, typename View>
__device__ __forceinline__ bool build_probe(const View& v, uint64_t h, uint64_t end, const GenomeTable& gt,
                                            const MatchParams& mp, int L, Mhe<MG>& P, uint32_t* gsize) {
    const uint64_t k0 = v.gkey(h);
    const uint32_t maxc = (uint32_t)gt.G * (mp.repeat_tol + 1u);
    uint32_t tally[MG];
    int64_t pos1[MG];
    uint32_t par[MG];
    #pragma unroll
    for (int g = 0; g < MG; ++g) { tally[g] = 0; pos1[g] = 0; par[g] = 0; }
    uint32_t cnt = 0, nh = 0;
    bool reject = false;
    for (uint64_t i = h; i < end; ++i) {
        if (v.gkey(i) != k0) break;
        ++cnt;
        if (cnt > maxc) {
            // some genome exceeds repeat_tol+1 occurrences: rejected.  Keep
            // counting only to report groups above MER_REPEAT_LIMIT.
            reject = true;
            if (cnt > (uint32_t)kRepeatLimit) break;
            continue;
        }
        if (reject) continue;
        const uint64_t gi = v.gidx(i);
        const int g = genome_of(gt, gi);
        const int64_t p = (int64_t)(gi - gt.base[g]);
        const uint32_t pb = v.par(i);
        #pragma unroll
        for (int q = 0; q < MG; ++q) {
            if (q != g) continue;
            if (tally[q] < mp.enum_tol) { pos1[q] = p + 1; par[q] = pb; ++nh; }
            if (tally[q] > mp.repeat_tol) reject = true;
            ++tally[q];
        }
    }
    *gsize = cnt;
    if (reject || cnt < 2 || nh < 2) return false;
    P.len = L;
    P.mersize = L;
    #pragma unroll
    for (int g = 0; g < MG; ++g) P.s[g] = pos1[g];
    const int ref = first_start(P);
    uint32_t ref_par = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) ref_par = (g == ref) ? par[g] : ref_par;
    #pragma unroll
    for (int g = 0; g < MG; ++g)
        if (g > ref && P.s[g] != 0 && par[g] != ref_par) P.s[g] = -P.s[g];
    const int64_t sref = start_at(P, ref);
    int64_t off = 0;
    uint64_t match_number = 0;
    int mult = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        if (g > ref && P.s[g] != 0) off += P.s[g] - sref - (P.s[g] < 0 ? (int64_t)L : 0);
        if (g < gt.G) {
            match_number = (match_number << 1) | (P.s[g] != 0 ? 1ull : 0ull);
            mult += P.s[g] != 0;
        }
    }
    P.offset = off;
    if (mp.masked) return mp.seq_mask == 0 || match_number == mp.seq_mask;
    return mult >= 2;
}

// genome of a global seed-mer index, unrolled to MG so the bases stay in SGPRs
template <int MG>
__device__ __forceinline__ int genome_of_mg(const GenomeTable& gt, uint64_t i) {
    int g = 0;
    #pragma unroll
    for (int k = 1; k < MG; ++k) g += (k < gt.G && i >= gt.base[k]) ? 1 : 0;
    return g;
}

// genome presence bits of a probe (bit g = genome g): 32 bits up to 32 genomes, else 64
template <int MG>
using MaskT = typename std::conditional<(MG > 32), uint64_t, uint32_t>::type;

// MaskedMemHash's match number (MaskedMemHash.cpp:51-58): genome 0 is the top of G bits
template <typename M>
__device__ __forceinline__ uint64_t match_number_of(M mask, uint32_t G) {
    if constexpr (sizeof(M) == 8) return __builtin_bitreverse64(mask) >> (64 - G);
    else return (uint64_t)(__builtin_bitreverse32(mask) >> (32 - G));
}

// Fast path of build_probe for the MemHash defaults repeat_tol = 0, enum_tol = 1
// (MemHash.h:31-32): accept iff >= 2 records and no genome twice; the probe offset
// (CalculateOffset, MatchHashEntry.cpp:141-160, after SetDirection) is summed
// directly without materialising the starts.  An accepted group has <= G records,
// so G+1 records are fetched as ONE batch of independent loads (no dependent load
// chain); only groups larger than G fall back to a counting walk (for the
// MER_REPEAT_LIMIT report).  Same results as build_probe.
// r[k] = record h + k for k <= G and h + k < end, else {~0, 0, 0} (the batch); v is only
// read past the batch, by the counting walk of an oversize group.
template <int MG, typename View>
__device__ __forceinline__ bool probe_offset_batch(const RecFields (&r)[MG + 1], const View& v, uint64_t h,
                                                   uint64_t end, const GenomeTable& gt, const MatchParams& mp, int L,
                                                   int64_t* offset, uint32_t* gsize) {
    const uint32_t G = (uint32_t)gt.G;
    const uint64_t k0 = r[0].gk;
    uint32_t cnt = 0;
    bool run = true;
    #pragma unroll
    for (int k = 0; k <= MG; ++k) {
        run = run && (r[k].gk == k0);
        cnt += run ? 1u : 0u;
    }
    if (cnt > G) {   // pigeonhole: some genome twice -> rejected; count on for the report
        uint64_t i = h + cnt;
        while (i < end && cnt <= (uint32_t)kRepeatLimit && v.gkey(i) == k0) { ++cnt; ++i; }
        *gsize = cnt;
        return false;
    }
    *gsize = cnt;
    if (cnt < 2) return false;
    MaskT<MG> mask = 0;
    bool dup = false;
    int gref = 64;
    int64_t sref = 0;
    uint32_t pref = 0;
    int gk[MG + 1];
    #pragma unroll
    for (int k = 0; k <= MG; ++k) {
        gk[k] = genome_of_mg<MG>(gt, r[k].idx);
        if ((uint32_t)k < cnt) {
            const int g = gk[k];
            dup = dup || ((mask >> g) & 1u);
            mask |= (MaskT<MG>)1 << g;
            if (g < gref) {
                gref = g;
                sref = (int64_t)(r[k].idx - gt.base[g]) + 1;
                pref = r[k].par;
            }
        }
    }
    if (dup) return false;
    int64_t off = 0;
    #pragma unroll
    for (int k = 0; k <= MG; ++k) {
        if ((uint32_t)k < cnt && gk[k] != gref) {
            const int64_t s = (int64_t)(r[k].idx - gt.base[gk[k]]) + 1;
            off += (r[k].par != pref) ? (-s - sref - (int64_t)L) : (s - sref);
        }
    }
    *offset = off;
    if (mp.masked) {
        const uint64_t match_number = match_number_of(mask, G);
        return mp.seq_mask == 0 || match_number == mp.seq_mask;
    }
    return true;
}

template <int MG, typename View>
__device__ __forceinline__ bool probe_offset_fast(const View& v, uint64_t h, uint64_t end, const GenomeTable& gt,
                                                  const MatchParams& mp, int L, int64_t* offset, uint32_t* gsize) {
    RecFields r[MG + 1];
    #pragma unroll
    for (int k = 0; k <= MG; ++k)
        r[k] = ((uint32_t)k <= (uint32_t)gt.G && h + k < end) ? v.get(h + k) : RecFields{~0ull, 0u, 0u};
    return probe_offset_batch<MG, View>(r, v, h, end, gt, mp, L, offset, gsize);
}

// ((offset % T) + T) % T without a 64-bit division: quotient from a double reciprocal
// (exact to within one for |offset| < 2^52), then one correction step.
__device__ __forceinline__ uint32_t bucket_of_fast(int64_t offset, uint32_t table_size, double inv_t) {
    const int64_t T = (int64_t)table_size;
    const int64_t q = (int64_t)floor((double)offset * inv_t);
    int64_t r = offset - q * T;
    r = r < 0 ? r + T : r;
    r = r >= T ? r - T : r;
    return (uint32_t)r;
}

// Default-tolerance probe (repeat_tol 0, enum_tol 1) from the raw packed records
// x[k] = record h + k (k <= G, inside the bucket; others = ~0), branch-free: the same
// results as probe_offset_fast.  gsize_batch = equal-key run length inside the batch
// (the caller walks on when it exceeds G).  Genome and base of each record come from
// one unrolled compare/select pass over the (32-bit) genome bases.
// The coarse genome lookup of GenomeTable (gl_*) staged in LDS by the calling kernel: a
// record's genome and base from two LDS reads instead of G - 1 compares and selects.
typedef __attribute__((address_space(3))) const uint8_t lds_u8c;
typedef __attribute__((address_space(3))) const uint32_t lds_u32c;
struct GLook {
    lds_u8c* tab;     // gl[], gl_n entries
    lds_u32c* base;   // base[0 .. kMaxG] as uint32 (N < 2^32)
    uint32_t shift, last;
};
__device__ __forceinline__ void glook(const GLook& l, uint32_t idx, uint32_t* g, uint32_t* b) {
    const uint32_t s = min(idx >> l.shift, l.last);   // (padding records: idx ~0)
    const uint32_t t = l.tab[s];
    const uint32_t b0 = l.base[t], b1 = l.base[t + 1];
    const bool ge = idx >= b1;
    *g = t + (ge ? 1u : 0u);
    *b = ge ? b1 : b0;
}

template <int MG, int IB = 32, bool kGl = false>
__device__ __forceinline__ bool probe_fast_raw(const uint64_t (&x)[MG + 1], const GenomeTable& gt,
                                               const MatchParams& mp, int L, int64_t* offset, uint32_t* gsize,
                                               const GLook* glk = nullptr) {
    const uint32_t G = (uint32_t)gt.G;
    const uint32_t k0 = (uint32_t)(x[0] >> (IB + 1));
    uint32_t cnt = 0;
    bool run = true;
    #pragma unroll
    for (int k = 0; k <= MG; ++k) {
        run = run && ((uint32_t)(x[k] >> (IB + 1)) == k0) && (x[k] != ~0ull);
        cnt += run ? 1u : 0u;
    }
    *gsize = cnt;
    MaskT<MG> mask = 0;
    uint32_t gref = 64, pref = 0;
    // 32-bit starts and bases for 32-bit record indices; 64-bit in the chunked mode
    using IdxT = typename std::conditional<(IB > 32), uint64_t, uint32_t>::type;
    IdxT sref = 0;
    bool dup = false;
    // record MG only bounds the run: an accepted probe has cnt <= G <= MG records, so it is
    // never a member (cnt = MG + 1 is rejected below whatever mask, dup and off hold)
    uint32_t gk[MG];
    IdxT sk[MG];
    #pragma unroll
    for (int k = 0; k < MG; ++k) {
        const IdxT idx = (IdxT)(x[k] & ((1ull << IB) - 1));
        uint32_t g = 0;
        IdxT b = 0;
        if constexpr (kGl && IB == 32) {
            uint32_t bb;
            glook(*glk, (uint32_t)idx, &g, &bb);
            b = bb;
        } else {
            #pragma unroll
            for (int j = 1; j < MG; ++j) {
                const IdxT bj = (IdxT)gt.base[j];
                const bool ge = (uint32_t)j < G && idx >= bj;
                g = ge ? (uint32_t)j : g;
                b = ge ? bj : b;
            }
        }
        gk[k] = g;
        sk[k] = idx - b + 1u;   // 1-based start in genome g
        const bool in = (uint32_t)k < cnt;
        dup = dup || (in && ((mask >> g) & 1u));
        mask |= in ? ((MaskT<MG>)1 << g) : (MaskT<MG>)0;
        const bool better = in && g < gref;
        gref = better ? g : gref;
        sref = better ? sk[k] : sref;
        pref = better ? (uint32_t)(x[k] >> IB) & 1u : pref;
    }
    int64_t off = 0;
    #pragma unroll
    for (int k = 0; k < MG; ++k) {
        const bool use = (uint32_t)k < cnt && gk[k] != gref;
        const int64_t sv = (int64_t)sk[k], sr = (int64_t)sref;
        const int64_t term = (((uint32_t)(x[k] >> IB) & 1u) != pref) ? (-sv - sr - (int64_t)L) : (sv - sr);
        off += use ? term : 0;
    }
    *offset = off;
    const bool accept = cnt >= 2 && cnt <= G && !dup;
    if (mp.masked) {
        const uint64_t match_number = match_number_of(mask, G);
        return accept && (mp.seq_mask == 0 || match_number == mp.seq_mask);
    }
    return accept;
}

// The probe (starts after SetDirection, CalculateOffset) of an accepted default-tolerance
// group of cnt (<= G) records x[0 .. cnt) -- packed records (key << IB+1 | parity << IB | index);
// the parity bit is part of the sort key, so the reference genome (the smallest present) is
// found, not assumed first.  All loads are the caller's one batch; the same row as build_probe.
template <int MG, int IB = 32, bool kGl = false>
__device__ __forceinline__ void probe_row_fast(const uint64_t (&x)[MG], uint32_t cnt, const GenomeTable& gt, int L,
                                               Mhe<MG>& P, const GLook* glk = nullptr) {
    using IdxT = typename std::conditional<(IB > 32), uint64_t, uint32_t>::type;
    const uint32_t G = (uint32_t)gt.G;
    int64_t st[MG];
    uint32_t gk[MG], pk[MG];
    #pragma unroll
    for (int k = 0; k < MG; ++k) {
        const IdxT idx = (IdxT)(x[k] & ((1ull << IB) - 1));
        uint32_t g = 0;
        IdxT b = 0;
        if constexpr (kGl && IB == 32) {
            uint32_t bb;
            glook(*glk, (uint32_t)idx, &g, &bb);
            b = bb;
        } else {
            #pragma unroll
            for (int j = 1; j < MG; ++j) {
                const IdxT bj = (IdxT)gt.base[j];
                const bool ge = (uint32_t)j < G && idx >= bj;
                g = ge ? (uint32_t)j : g;
                b = ge ? bj : b;
            }
        }
        gk[k] = (uint32_t)k < cnt ? g : 0xFFu;
        pk[k] = (uint32_t)(x[k] >> IB) & 1u;
        st[k] = (int64_t)(idx - b) + 1;
    }
    uint32_t gref = 0xFFu, ref_par = 0;
    int64_t sref = 0;
    #pragma unroll
    for (int k = 0; k < MG; ++k) {
        const bool better = gk[k] < gref;   // (records past cnt carry 0xFF)
        gref = better ? gk[k] : gref;
        ref_par = better ? pk[k] : ref_par;
        sref = better ? st[k] : sref;
    }
    int64_t off = 0;
    #pragma unroll
    for (int k = 0; k < MG; ++k) {
        const bool other = gk[k] != gref && gk[k] != 0xFFu;
        const bool rev = other && pk[k] != ref_par;
        st[k] = rev ? -st[k] : st[k];
        off += other ? (st[k] - sref - (rev ? (int64_t)L : 0)) : 0;
    }
    P.len = L;
    P.mersize = L;
    P.offset = off;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        int64_t v = 0;
        #pragma unroll
        for (int k = 0; k < MG; ++k) v = gk[k] == (uint32_t)g ? st[k] : v;
        P.s[g] = v;
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

// line invariants: reference start x = s_ref (> 0); per other component the
// diagonal s_g - s_ref (forward) or |s_g| + s_ref (reverse).  kLineHashBits of them key the
// line order; fewer bits save sort passes (24: -1.4 ms at C3) but a collision that interleaves
// two chains changes the MatchList (chains.hip), so 32 stays.
#ifndef MUMS_LINE_HASH_BITS
#define MUMS_LINE_HASH_BITS 32
#endif
constexpr int kLineHashBits = MUMS_LINE_HASH_BITS;
template <int MG>
__device__ __forceinline__ uint64_t line_hash64(const Mhe<MG>& P, int G) {
    const int ref = first_start(P);
    const int64_t x = start_at(P, ref);
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)ref;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        if (g < G && g > ref && P.s[g] != 0) {
            const int64_t s = P.s[g];
            const uint64_t d = s > 0 ? (uint64_t)(s - x) : (uint64_t)(-s + x) ^ 0x8000000000000000ull;
            h = mix64(h ^ d ^ ((uint64_t)g << 56));
        } else {
            h = mix64(h ^ ((uint64_t)g << 48));
        }
    }
    return h;
}
template <int MG>
__device__ __forceinline__ uint32_t line_hash(const Mhe<MG>& P, int G) {
    return (uint32_t)(line_hash64<MG>(P, G) >> (64 - kLineHashBits));
}


// Materialized probes: the AddHashEntry arguments of the seed stage in key order, one
// row of G+1 int64 per probe: the signed 1-based starts (after SetDirection) and the
// CalculateOffset value.  The chain labelling and the replay read probes only through
// this (one contiguous row per probe instead of G+1 gathers from the record stream);
// the sharded FindMatches ships the same rows between ranks.
// rows32 (optional, G <= 16, every start below 2^31): the same rows as G int32 starts (stride32
// = G rounded up to 4) with the offset recomputed from them (probe_offset, seed length L32) --
// 32 B per probe at G = 8 instead of 72; the materialize pass checked the recomputation.
// rows is then null.
struct MatProbes {
    const int64_t* rows;           // [P][G + 1]
    const uint32_t* fs = nullptr;  // optional: probe k's first-genome start (the replay's keep test)
    const int32_t* rows32 = nullptr;
    uint32_t stride32 = 0;
    int L32 = 0;
};

// CalculateOffset of directed starts (the sum build_probe takes, MemHash.cpp:189-203)
template <int MG>
__device__ __forceinline__ int64_t probe_offset(const Mhe<MG>& P, int L) {
    const int ref = first_start(P);
    const int64_t sref = start_at(P, ref);
    int64_t off = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g)
        if (g > ref && P.s[g] != 0) off += P.s[g] - sref - (P.s[g] < 0 ? (int64_t)L : 0);
    return off;
}

__host__ __device__ inline uint32_t line_row_stride(int G) { return (uint32_t)((G + 3) & ~3); }

// one row of int32 starts (16-B aligned, stride a multiple of 4)
template <int MG>
__device__ __forceinline__ void load_probe32(const int32_t* __restrict__ row, int G, int L, int Loff, Mhe<MG>& P) {
    P.len = L;
    P.mersize = L;
    if constexpr (MG % 4 == 0) {
        #pragma unroll
        for (int q = 0; q < MG / 4; ++q) {
            int4 v = make_int4(0, 0, 0, 0);
            if (4 * q < G) v = *reinterpret_cast<const int4*>(row + 4 * q);
            P.s[4 * q] = v.x;
            P.s[4 * q + 1] = 4 * q + 1 < G ? v.y : 0;
            P.s[4 * q + 2] = 4 * q + 2 < G ? v.z : 0;
            P.s[4 * q + 3] = 4 * q + 3 < G ? v.w : 0;
        }
    } else {
        #pragma unroll
        for (int g = 0; g < MG; ++g) P.s[g] = (g < G) ? row[g] : 0;
    }
    P.offset = probe_offset<MG>(P, Loff);
}

template <int MG>
__device__ __forceinline__ void load_probe(const MatProbes& m, uint64_t k, int G, int L, Mhe<MG>& P) {
    if (m.rows32) {   // kernel argument: a uniform branch
        load_probe32<MG>(m.rows32 + k * (uint64_t)m.stride32, G, L, m.L32, P);
        return;
    }
    const int64_t* row = m.rows + k * (uint64_t)(G + 1);
    P.len = L;
    P.mersize = L;
    P.offset = row[G];
    #pragma unroll
    for (int g = 0; g < MG; ++g) P.s[g] = (g < G) ? row[g] : 0;
}

// The chain kernels' copy of the probe rows in line order when every start fits 31 bits:
// G int32 starts per row (stride G rounded up to 4, 16-B aligned rows) and the offset
// recomputed from them -- 32 B per probe instead of 72 at G = 8.  The gather that writes
// it checks the recomputed offset against the materialized one (launch_gather_line_rows).
struct LineRows {
    const int32_t* rows;
    uint32_t stride;
    int L;                           // seed length of the offset sum
    const uint32_t* ord = nullptr;   // set: rows in key order, read through the line order
};

template <int MG>
__device__ __forceinline__ void load_probe(const LineRows& m, uint64_t k, int G, int L, Mhe<MG>& P) {
    const uint64_t r = m.ord ? (uint64_t)m.ord[k] : k;
    load_probe32<MG>(m.rows + r * (uint64_t)m.stride, G, L, m.L, P);
}

__device__ __forceinline__ uint32_t bucket_of(int64_t offset, uint32_t table_size) {
    const int64_t T = (int64_t)table_size;
    return (uint32_t)(((offset % T) + T) % T);  // MemHash.cpp:213
}

}  // namespace mums
