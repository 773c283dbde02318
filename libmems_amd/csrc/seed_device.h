// seed_device.h -- canonical spaced-seed key of one position (rows A2-A3), device side.
//
// Packed sequence layout = the reference's SortedMerList::sequence (translate32,
// SortedMerList.cpp:425-460): base i of a genome in bits [31-2(i%16), 30-2(i%16)] of
// word i/16, >= 2 zero pad words after the last base.  Genome g starts at word
// gt.woff[g] of one packed array.
#pragma once

#include "mums_internal.h"

namespace mums {

// XCD-grouped block order (a bijective blockIdx swizzle, cdna_hip_programming.md T1): the
// dispatcher hands workgroups to the 8 XCDs round-robin, so blocks b, b + 8, b + 16 ...
// share one L2; they get consecutive work indices (placement is a speed matter only)
__device__ __forceinline__ uint32_t xcd_grouped_block(uint32_t b, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7u, x = b & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// 2w-bit reverse complement (RevCompMer, SortedMerList.cpp:597-614, on bottom-aligned bits)
__device__ __forceinline__ uint64_t revcomp2w(uint64_t v, int w) {
    uint64_t x = ~v;
    x = __builtin_bitreverse64(x);
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    return x >> (64 - 2 * w);
}

// compact canonical key (v << 1) | parity from a 64-bit window whose first base sits in
// bits 63-62 (GetMer, :321-342): v = min(forward seed, reverse-complement seed)
// (GetSeedMer :726-762 + GetDnaSeedMer :764-769); parity = 1 iff the RC was chosen.
__device__ __forceinline__ uint64_t ckey_finish(uint64_t v, int w) {
    const uint64_t rc = revcomp2w(v, w);
    const uint64_t par = rc < v ? 1ull : 0ull;
    return ((par ? rc : v) << 1) | par;
}

__device__ __forceinline__ uint64_t ckey_from_mer(uint64_t mer, const SeedSpec& ss) {
    uint64_t v = 0;
    for (int r = 0; r < ss.nruns; ++r) {
        const int sh = ss.run_sh[r];
        v |= (sh >= 0 ? (mer >> sh) : (mer << -sh)) & ss.run_mask[r];
    }
    return ckey_finish(v, ss.w);
}

// Compile-time seed patterns (the BASELINE seeds): the run table is a constant, so the
// extraction unrolls to one shift + mask + or per run with immediate operands.
struct SeedRuns {
    int n = 0, L = 0, w = 0;
    int sh[kMaxSeedRuns] = {};
    uint64_t mask[kMaxSeedRuns] = {};
};

// same derivation as the host's make_seed_spec (mums_capi.hip)
constexpr SeedRuns seed_runs(uint64_t pat) {
    SeedRuns R{};
    int lo = 0, hi = 63;
    while (lo < 64 && !((pat >> lo) & 1)) ++lo;
    while (hi >= 0 && !((pat >> hi) & 1)) --hi;
    R.L = hi - lo + 1;
    int start[kMaxSeedRuns] = {}, len[kMaxSeedRuns] = {};
    int r = -1;
    bool prev = false;
    for (int k = 0; k < R.L; ++k) {
        const bool care = (pat >> (R.L - 1 - k)) & 1;
        if (care) {
            if (!prev) { ++r; start[r] = k; len[r] = 0; }
            ++len[r];
            ++R.w;
        }
        prev = care;
    }
    R.n = r + 1;
    int cum = 0;
    for (int i = 0; i < R.n; ++i) {
        cum += len[i];
        const int dst = 2 * (R.w - cum);
        R.sh[i] = 64 - 2 * (start[i] + len[i]) - dst;
        R.mask[i] = ((len[i] >= 32) ? ~0ull : ((1ull << (2 * len[i])) - 1)) << dst;
    }
    return R;
}

template <uint64_t PAT>
__device__ __forceinline__ uint64_t ckey_static(uint64_t mer) {
    constexpr SeedRuns R = seed_runs(PAT);
    static_assert(R.n > 0 && R.n <= kMaxSeedRuns, "bad static seed");
    uint64_t v = 0;
    #pragma unroll
    for (int r = 0; r < R.n; ++r) v |= (R.sh[r] >= 0 ? (mer >> R.sh[r]) : (mer << -R.sh[r])) & R.mask[r];
    return ckey_finish(v, R.w);
}

// key of a 64-bit window: static pattern PAT when non-zero, else the run table of ss
template <uint64_t PAT>
__device__ __forceinline__ uint64_t ckey_of(uint64_t mer, const SeedSpec& ss) {
    if constexpr (PAT != 0) return ckey_static<PAT>(mer);
    else return ckey_from_mer(mer, ss);
}

// Top K bits of the (2w+1)-bit canonical key of a static pattern, without building the
// key: ckey = min(v, rc) << 1 | parity, so its top K bits are the top K bits of
// min(v, rc) = min(top_K(v), top_K(rc)) (the minimum of two equal-width integers has the
// smaller prefix).  top_K(v) needs only the runs under v's top K bits, top_K(rc) only
// v's low ceil(K/2) bases (complemented, base order reversed); the constant run masks
// let the compiler drop every other run.  Used for the MSD histogram of the keys pass.
template <uint64_t PAT, int K>
__device__ __forceinline__ uint32_t ckey_top_static(uint64_t mer) {
    constexpr SeedRuns R = seed_runs(PAT);
    constexpr int B = (K + 1) / 2;
    static_assert(K >= 1 && 2 * B <= 2 * R.w && 2 * B <= 32, "top digit wider than the seed");
    uint64_t v = 0;
    #pragma unroll
    for (int r = 0; r < R.n; ++r) v |= (R.sh[r] >= 0 ? (mer >> R.sh[r]) : (mer << -R.sh[r])) & R.mask[r];
    const uint32_t ft = (uint32_t)(v >> (2 * R.w - K));
    const uint32_t lowc = ~(uint32_t)v & (uint32_t)((1ull << (2 * B)) - 1);
    uint32_t rr = __builtin_bitreverse32(lowc) >> (32 - 2 * B);
    rr = ((rr >> 1) & 0x55555555u) | ((rr & 0x55555555u) << 1);
    const uint32_t rt = rr >> (2 * B - K);
    return ft < rt ? ft : rt;
}

// the patterns with compiled-in run tables (getSeed(15), getSeed(19): SeedMasks.h)
constexpr uint64_t kSeedW15 = 0x7ac9afull;
constexpr uint64_t kSeedW19 = 0x7b974efull;
constexpr uint64_t kSeedW21 = 0x7ddaddfull;   // getSeed(21): default weight of genomes above ~1.07 Gbp

__device__ __forceinline__ uint64_t window_at(const uint32_t* __restrict__ W, uint64_t p) {
    const uint64_t wi = p >> 4;
    const int sh = 2 * (int)(p & 15);
    const uint64_t hi = ((uint64_t)W[wi] << 32) | W[wi + 1];
    const uint64_t lo = W[wi + 2];
    return (hi << sh) | ((lo << sh) >> 32);
}

__device__ __forceinline__ uint64_t ckey_at(const uint32_t* __restrict__ W, uint64_t p, const SeedSpec& ss) {
    return ckey_from_mer(window_at(W, p), ss);
}

// ---- views of the merged, key-sorted stream ------------------------------------
struct RecFields {
    uint64_t gk;    // group key (masked ckey)
    uint32_t par;   // strand parity
    uint64_t idx;   // global seed-mer index
};

// PairView: (ckey, global index) pairs (generic path, any weight); 64-bit indices (I =
// uint64_t) for the chunked mode's enumerations above 2^32 seed-mers.
template <typename K, typename I = uint32_t>
struct PairView {
    const K* key;
    const I* idx;
    __device__ __forceinline__ uint64_t gkey(uint64_t i) const { return (uint64_t)key[i] >> 1; }
    __device__ __forceinline__ uint32_t par(uint64_t i) const { return (uint32_t)(key[i] & 1); }
    __device__ __forceinline__ uint64_t gidx(uint64_t i) const { return idx[i]; }
    __device__ __forceinline__ RecFields get(uint64_t i) const {
        const uint64_t k = (uint64_t)key[i];
        return RecFields{k >> 1, (uint32_t)(k & 1), idx[i]};
    }
};

// RecView: packed records (ckey_low << IB | global index), IB index bits (32; 33 in the
// chunked mode for > 2^32 seed-mers); the top ckey bits are the MSD bucket the record
// sits in, so groups never cross a bucket boundary.
template <int IB = 32>
struct RecViewT {
    static constexpr int kIB = IB;
    const uint64_t* rec;
    __device__ __forceinline__ uint64_t gkey(uint64_t i) const { return rec[i] >> (IB + 1); }
    __device__ __forceinline__ uint32_t par(uint64_t i) const { return (uint32_t)(rec[i] >> IB) & 1u; }
    __device__ __forceinline__ uint64_t gidx(uint64_t i) const { return rec[i] & ((1ull << IB) - 1); }
    __device__ __forceinline__ RecFields get(uint64_t i) const {
        const uint64_t r = rec[i];
        return RecFields{r >> (IB + 1), (uint32_t)(r >> IB) & 1u, r & ((1ull << IB) - 1)};
    }
};
using RecView = RecViewT<32>;

// index bits of a packed-record view (0 for the pair views)
template <class V>
struct RecIB { static constexpr int value = 0; };
template <int IB>
struct RecIB<RecViewT<IB>> { static constexpr int value = IB; };

}  // namespace mums
