// seedmasks.cpp -- spaced-seed patterns and default weight (row A1).
//
// The pattern table is data from Darling et al. 2006 as shipped in libMems'
// SeedMasks.h:44-260 (low 32-bit words; the high words are all 0).  getSeed /
// getSeedLength / getSeedWeight / getDefaultSeedWeight semantics follow
// SeedMasks.h:298-401, including its table quirks (getSeed(11) returns a
// weight-12 pattern; non-palindromic rank-1/2 entries are kept verbatim).
#include <climits>
#include <cmath>
#include <cstdint>

#include "../../include/mums.h"

namespace {

const uint32_t kSeedTable[32][6] = {
    {0}, {0}, {0},
    {0xb, 0, 0, 0, 0, 0},
    {0x3b, 0, 0, 0, 0, 0},
    {0x6b, 0x139, 0x193, 0x6b, 0, 0},
    {0x58D, 0x653, 0x1AB, 0xdb, 0, 0},
    {0x1953, 0x588d, 0x688b, 0x17d, 0x164d, 0},
    {0x3927, 0x1CA7, 0x6553, 0xb6d, 0, 0},
    {0x7497, 0x1c927, 0x72a7, 0x6fb, 0x16ed, 0},
    {0x1d297, 0x3A497, 0xE997, 0x6D5B, 0, 0},
    {0x7954f, 0x75257, 0x1c9527, 0x5bed, 0x5b26d, 0},
    {0x7954f, 0x3D32F, 0x768B7, 0x5B56D, 0, 0},
    {0x792a4f, 0x1d64d7, 0x1d3597, 0x1b7db, 0x75ad7, 0},
    {0x1e6acf, 0xF59AF, 0x3D4CAF, 0x35AD6B, 0, 0},
    {0x7ac9af, 0x7b2a6f, 0x79aacf, 0x16df6d, 0x6b5d6b, 0},
    {0xf599af, 0xEE5A77, 0x7CD59F, 0xEB5AD7, 0, 0},
    {0x6dbedb, 0, 0, 0, 0, 0},
    {0x3E6B59F, 0x3EB335F, 0x7B3566F, 0, 0, 0},
    {0x7b974ef, 0x7d6735f, 0x1edd74f, 0, 0, 0},
    {0x1F59B35F, 0x3EDCEDF, 0xFAE675F, 0, 0, 0},
    {0x7ddaddf, 0xaeb3f, 0x7eb76bf, 0, 0, 0},
    {0x003fffff, 0, 0, 0, 0, 0},
    {0x007fffff, 0, 0, 0, 0, 0},
    {0x00ffffff, 0, 0, 0, 0, 0},
    {0x01ffffff, 0, 0, 0, 0, 0},
    {0x03ffffff, 0, 0, 0, 0, 0},
    {0x07ffffff, 0, 0, 0, 0, 0},
    {0x0fffffff, 0, 0, 0, 0, 0},
    {0x1fffffff, 0, 0, 0, 0, 0},
    {0x3fffffff, 0, 0, 0, 0, 0},
    {0x7fffffff, 0, 0, 0, 0, 0},
};

int64_t solid(int weight) { return (int64_t)((((uint64_t)1) << weight) - 1); }

}  // namespace

extern "C" int64_t mums_get_seed(int weight, int seed_rank) {
    if (seed_rank == INT_MAX) return solid(weight);       // SOLID_SEED
    if (weight > 31) return solid(32);
    if (seed_rank > 5) return solid(weight);
    if (weight < 0 || seed_rank < 0 || kSeedTable[weight][seed_rank] == 0) return solid(weight);
    return (int64_t)kSeedTable[weight][seed_rank];
}

extern "C" uint32_t mums_default_seed_weight(uint64_t avg_len) {
    uint32_t m = (uint32_t)std::ceil((std::log((double)avg_len) / std::log(2.0)) / 1.5);
    if (!(m & 1)) ++m;                 // odd weights cannot be reverse-complement palindromes
    m = m < 5 ? 0 : m;
    if (avg_len == 0) m = 0;
    return m > 31 ? 31 : m;
}
