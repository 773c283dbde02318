// seed_device.h -- canonical spaced-seed key of one position (rows A2-A3), device side.
//
// Packed sequence layout = the reference's SortedMerList::sequence (translate32,
// SortedMerList.cpp:425-460): base i of a genome in bits [31-2(i%16), 30-2(i%16)] of
// word i/16, >= 2 zero pad words after the last base.  Genome g starts at word
// gt.woff[g] of one packed array.
#pragma once

#include "mums_internal.h"

namespace mums {

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
__device__ __forceinline__ uint64_t ckey_from_mer(uint64_t mer, const SeedSpec& ss) {
    uint64_t v = 0;
    for (int r = 0; r < ss.nruns; ++r) {
        const int s = ss.run_start[r], l = ss.run_len[r];
        v |= ((mer >> (64 - 2 * (s + l))) & ((1ull << (2 * l)) - 1)) << ss.run_dst[r];
    }
    const uint64_t rc = revcomp2w(v, ss.w);
    const uint64_t par = rc < v ? 1ull : 0ull;
    return ((par ? rc : v) << 1) | par;
}

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
    uint32_t idx;   // global seed-mer index
};

// PairView: (ckey, global index) pairs (generic path, any weight).
template <typename K>
struct PairView {
    const K* key;
    const uint32_t* idx;
    __device__ __forceinline__ uint64_t gkey(uint64_t i) const { return (uint64_t)key[i] >> 1; }
    __device__ __forceinline__ uint32_t par(uint64_t i) const { return (uint32_t)(key[i] & 1); }
    __device__ __forceinline__ uint32_t gidx(uint64_t i) const { return idx[i]; }
    __device__ __forceinline__ RecFields get(uint64_t i) const {
        const uint64_t k = (uint64_t)key[i];
        return RecFields{k >> 1, (uint32_t)(k & 1), idx[i]};
    }
};

// RecView: packed records (ckey_low << 32 | global index); the top ckey bits are the
// MSD bucket the record sits in, so groups never cross a bucket boundary.
struct RecView {
    const uint64_t* rec;
    __device__ __forceinline__ uint64_t gkey(uint64_t i) const { return rec[i] >> 33; }
    __device__ __forceinline__ uint32_t par(uint64_t i) const { return (uint32_t)(rec[i] >> 32) & 1u; }
    __device__ __forceinline__ uint32_t gidx(uint64_t i) const { return (uint32_t)rec[i]; }
    __device__ __forceinline__ RecFields get(uint64_t i) const {
        const uint64_t r = rec[i];
        return RecFields{r >> 33, (uint32_t)(r >> 32) & 1u, (uint32_t)r};
    }
};

}  // namespace mums
