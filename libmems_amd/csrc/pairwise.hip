// pairwise.hip -- group enumerations that issue several AddHashEntry calls per seed group,
// written as probe rows for the FindMatches tail:
//   * PairwiseMatchFinder (PairwiseMatchFinder.h:23-33);
//   * MemHash with enumeration tolerance > 1 (MemHash::EnumerateMatches, MemHash.cpp:139-162,
//     -> MatchFinder::EnumerateMatches' odometer, MatchFinder.cpp:342-393).
//
// PairwiseMatchFinder is a MemHash whose EnumerateMatches (PairwiseMatchFinder.cpp:37-73)
// hashes, for every masked-key group, each PAIR of genomes that occur exactly once in
// the group (the group sorted by genome id, pairs in list order), through the unchanged
// MemHash::HashMatch -> AddHashEntry.  On the GPU the sorted (ckey, index) stream is
// scanned per group head: pw_count_kernel counts the pairs of each group, an exclusive
// scan places them, and pw_emit_kernel writes one probe row per pair (the G+1 int64
// {signed starts after SetDirection, CalculateOffset} rows the FindMatches tail replays).
#include <hip/hip_runtime.h>

#include "match_device.h"
#include "mums_internal.h"
#include "seed_device.h"

#include <type_traits>

namespace mums {
namespace {

template <typename View>
__device__ __forceinline__ bool pw_head(const View& v, uint64_t i) {
    return i == 0 || v.gkey(i) != v.gkey(i - 1);
}

// genomes present exactly once in the group starting at head h; *size = group size
// (walk stops past MER_REPEAT_LIMIT: SearchRange skips such groups, MatchFinder.cpp:215)
template <int MG>
using PwMask = typename std::conditional<(MG > 32), uint64_t, uint32_t>::type;

template <int MG, typename View>
__device__ __forceinline__ PwMask<MG> pw_unique(const View& v, uint64_t h, uint64_t N, const GenomeTable& gt,
                                                uint32_t* size) {
    const uint64_t k0 = v.gkey(h);
    PwMask<MG> seen = 0, dup = 0;
    uint32_t n = 0;
    for (uint64_t j = h; j < N && v.gkey(j) == k0; ++j) {
        ++n;
        const PwMask<MG> b = (PwMask<MG>)1 << genome_of(gt, v.gidx(j));
        dup |= seen & b;
        seen |= b;
    }
    *size = n;
    return seen & ~dup;
}

template <int MG, typename View>
__global__ void pw_count_kernel(View v, uint64_t N, GenomeTable gt, uint32_t* __restrict__ npairs,
                                DevCounters* __restrict__ ctr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t c = 0;
    if (pw_head(v, i)) {
        uint32_t size = 0;
        const PwMask<MG> u = pw_unique<MG>(v, i, N, gt, &size);
        const uint32_t k = (uint32_t)__builtin_popcountll((uint64_t)u);
        // a group above MER_REPEAT_LIMIT that survived the restart fix-up (restart.hip) is
        // enumerated like any other (SearchRange hands it to EnumerateMatches, :242-246)
        if (size > (uint32_t)kRepeatLimit) atomicAdd(&ctr->repeat_limit, 1ull);
        if (size >= 2) c = k * (k - 1) / 2;
    }
    npairs[i] = c;
}

// PairwiseMatchFinder::EnumerateMatches pairs (a < b over the single-copy genomes) ->
// MemHash::HashMatch (MemHash.cpp:167-187): starts pos+1, SetDirection (:189-203: the
// lower genome is the reference, the other is negated when its strand parity differs),
// CalculateOffset (MatchHashEntry.cpp:141-160).
template <int MG, typename View>
__global__ void pw_emit_kernel(View v, uint64_t N, GenomeTable gt, int L, const uint32_t* __restrict__ npairs,
                               const uint32_t* __restrict__ off, int64_t* __restrict__ rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || npairs[i] == 0) return;
    const int G = gt.G;
    uint32_t size = 0;
    const PwMask<MG> u = pw_unique<MG>(v, i, N, gt, &size);
    int64_t s[MG];
    uint32_t par[MG];
    const uint64_t k0 = v.gkey(i);
    for (uint64_t j = i; j < N && v.gkey(j) == k0; ++j) {
        const RecFields r = v.get(j);
        const int g = genome_of(gt, r.idx);
        if ((u >> g) & 1) {
            s[g] = (int64_t)(r.idx - gt.base[g]) + 1;
            par[g] = r.par;
        }
    }
    uint64_t o = off[i];
    for (int a = 0; a < G; ++a) {
        if (!((u >> a) & 1)) continue;
        for (int b = a + 1; b < G; ++b) {
            if (!((u >> b) & 1)) continue;
            int64_t* row = rows + o * (uint64_t)(G + 1);
            for (int g = 0; g < G; ++g) row[g] = 0;
            const int64_t sb = (par[b] != par[a]) ? -s[b] : s[b];
            row[a] = s[a];
            row[b] = sb;
            row[G] = sb - s[a] - (sb < 0 ? (int64_t)L : 0);
            ++o;
        }
    }
}

// ---- enumeration tolerance > 1 -------------------------------------------------------
constexpr int kEnumMax = 8;   // enum_tol bound of the slot kernels (per-genome record slots); above: the walk kernels

// MemHash::EnumerateMatches over the group at head h (per genome in SML order): per genome the
// first min(count, enum_tol) records; rejected (false) when a genome has more than
// repeat_tol + 1 records (groups above MER_REPEAT_LIMIT reach here only when the
// reference's merge hands them over whole: restart.hip).  c[g] = kept records of g,
// pos[g][i] / par[g][i] their positions and strand parities.
template <int MG, typename View>
__device__ bool en_collect(const View& v, uint64_t h, uint64_t N, const GenomeTable& gt, const MatchParams& mp,
                           uint32_t (&c)[MG], uint32_t (&pos)[MG][kEnumMax], uint8_t (&par)[MG][kEnumMax],
                           uint32_t* size) {
    const uint64_t k0 = v.gkey(h);
    uint32_t tally[MG];
    for (int g = 0; g < MG; ++g) { tally[g] = 0; c[g] = 0; }
    uint32_t n = 0;
    bool ok = true;
    // stream order inside a group = (parity, genome, position): restricted to one genome
    // that is its SortedMerList order (full key, then position)
    for (uint64_t j = h; j < N && v.gkey(j) == k0; ++j) {
        ++n;
        const RecFields r = v.get(j);
        const int g = genome_of(gt, r.idx);
        if (tally[g] < mp.enum_tol) {
            pos[g][c[g]] = (uint32_t)(r.idx - gt.base[g]);
            par[g][c[g]] = (uint8_t)r.par;
            ++c[g];
        }
        if (tally[g] > mp.repeat_tol) ok = false;
        ++tally[g];
    }
    *size = n;
    return ok;
}

// AddHashEntry calls of a group: the odometer's combinations (one record per present
// genome), or the single HashMatch of a two-record list; HashMatch / MaskedMemHash::
// HashMatch decide whether each combination is added (same genome set for all of them).
template <int MG>
__device__ __forceinline__ uint64_t en_calls(const uint32_t (&c)[MG], int G, const MatchParams& mp, bool* two) {
    uint64_t total = 0, nid = 0, combos = 1;
    uint64_t mn = 0;
    for (int g = 0; g < G; ++g) {
        total += c[g];
        mn <<= 1;
        if (c[g]) { ++nid; combos = combos > (1ull << 32) ? combos : combos * c[g]; mn |= 1; }
    }
    *two = total == 2;
    if (total < 2) return 0;
    // Multiplicity = genomes present (a two-record list of one genome has 1: no AddHashEntry)
    const bool add = mp.masked ? (mp.seq_mask == 0 || mn == mp.seq_mask) : nid >= 2;
    if (!add) return 0;
    return (total == 2) ? 1u : combos;
}

// a group's AddHashEntry calls as a 32-bit row count; above 2^31 (enum_tol^genomes) the row
// stream cannot hold them: DevCounters::err bit 64, the host refuses the find
__device__ __forceinline__ uint32_t en_rows32(uint64_t k, DevCounters* ctr) {
    if (k <= 0x7FFFFFFFull) return (uint32_t)k;
    atomicOr(&ctr->err, 64u);
    return 0;
}

template <int MG, typename View>
__global__ void en_count_kernel(View v, uint64_t N, GenomeTable gt, MatchParams mp, uint32_t* __restrict__ ncalls,
                                DevCounters* __restrict__ ctr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t k = 0;
    if (pw_head(v, i)) {
        uint32_t c[MG], pos[MG][kEnumMax], size = 0;
        uint8_t par[MG][kEnumMax];
        const bool ok = en_collect<MG>(v, i, N, gt, mp, c, pos, par, &size);
        if (size > (uint32_t)kRepeatLimit) atomicAdd(&ctr->repeat_limit, 1ull);
        bool two;
        if (ok && size >= 2) k = en_rows32(en_calls<MG>(c, gt.G, mp, &two), ctr);
    }
    ncalls[i] = k;
}

template <int MG, typename View>
__global__ void en_emit_kernel(View v, uint64_t N, GenomeTable gt, MatchParams mp, int L,
                               const uint32_t* __restrict__ ncalls, const uint32_t* __restrict__ off,
                               int64_t* __restrict__ rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || ncalls[i] == 0) return;
    const int G = gt.G;
    uint32_t c[MG], pos[MG][kEnumMax], size = 0;
    uint8_t par[MG][kEnumMax];
    (void)en_collect<MG>(v, i, N, gt, mp, c, pos, par, &size);
    bool two;
    const uint64_t K = en_calls<MG>(c, G, mp, &two);
    uint64_t o = off[i];
    for (uint64_t t = 0; t < K; ++t) {
        int64_t sv[MG];
        uint32_t pv[MG];
        for (int g = 0; g < G; ++g) { sv[g] = 0; pv[g] = 0; }
        if (two) {   // HashMatch of the two listed records (MatchFinder.cpp:344-347)
            for (int g = 0; g < G; ++g)
                for (uint32_t q = 0; q < c[g]; ++q) { sv[g] = (int64_t)pos[g][q] + 1; pv[g] = par[g][q]; }
        } else {     // odometer: the last genome varies fastest (MatchFinder.cpp:371-390)
            uint64_t rem = t;
            for (int g = G - 1; g >= 0; --g) {
                if (!c[g]) continue;
                const uint32_t q = (uint32_t)(rem % c[g]);
                rem /= c[g];
                sv[g] = (int64_t)pos[g][q] + 1;
                pv[g] = par[g][q];
            }
        }
        // SetDirection (MemHash.cpp:189-203) + CalculateOffset (MatchHashEntry.cpp:141-160)
        int ref = -1;
        for (int g = 0; g < G && ref < 0; ++g)
            if (sv[g] != 0) ref = g;
        int64_t offset = 0;
        for (int g = ref + 1; g < G; ++g) {
            if (sv[g] == 0) continue;
            if (pv[g] != pv[ref]) sv[g] = -sv[g];
            offset += sv[g] - sv[ref] - (sv[g] < 0 ? (int64_t)L : 0);
        }
        int64_t* row = rows + (o + t) * (uint64_t)(G + 1);
        for (int g = 0; g < G; ++g) row[g] = sv[g];
        row[G] = offset;
    }
}

// ---- enumeration tolerance above kEnumMax ---------------------------------------------
// Same AddHashEntry calls as en_count / en_emit, without per-genome record slots: the count
// keeps c[g] = min(count, enum_tol) only, and each odometer combination re-walks the group,
// taking the q[g]-th record of genome g (a genome's records in the group are in its
// SortedMerList order, so its first c[g] records are the ones MemHash::EnumerateMatches
// lists, MemHash.cpp:146-152).  O(group size) per AddHashEntry call: the rare large
// tolerances pay for the walk, enum_tol <= kEnumMax keeps the slot kernels above.
template <int MG, typename View>
__device__ bool en_tally(const View& v, uint64_t h, uint64_t N, const GenomeTable& gt, const MatchParams& mp,
                         uint32_t (&c)[MG], uint32_t* size) {
    const uint64_t k0 = v.gkey(h);
    uint32_t tally[MG];
    for (int g = 0; g < MG; ++g) { tally[g] = 0; c[g] = 0; }
    uint32_t n = 0;
    bool ok = true;
    for (uint64_t j = h; j < N && v.gkey(j) == k0; ++j) {
        ++n;
        const int g = genome_of(gt, v.gidx(j));
        if (tally[g] < mp.enum_tol) ++c[g];
        if (tally[g] > mp.repeat_tol) ok = false;
        ++tally[g];
    }
    *size = n;
    return ok;
}

template <int MG, typename View>
__global__ void en_count_walk_kernel(View v, uint64_t N, GenomeTable gt, MatchParams mp, uint32_t* __restrict__ ncalls,
                                     DevCounters* __restrict__ ctr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t k = 0;
    if (pw_head(v, i)) {
        uint32_t c[MG], size = 0;
        const bool ok = en_tally<MG>(v, i, N, gt, mp, c, &size);
        if (size > (uint32_t)kRepeatLimit) atomicAdd(&ctr->repeat_limit, 1ull);
        bool two;
        if (ok && size >= 2) k = en_rows32(en_calls<MG>(c, gt.G, mp, &two), ctr);
    }
    ncalls[i] = k;
}

template <int MG, typename View>
__global__ void en_emit_walk_kernel(View v, uint64_t N, GenomeTable gt, MatchParams mp, int L,
                                    const uint32_t* __restrict__ ncalls, const uint32_t* __restrict__ off,
                                    int64_t* __restrict__ rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || ncalls[i] == 0) return;
    const int G = gt.G;
    uint32_t c[MG], size = 0;
    (void)en_tally<MG>(v, i, N, gt, mp, c, &size);
    bool two;
    const uint64_t K = en_calls<MG>(c, G, mp, &two);
    const uint64_t k0 = v.gkey(i);
    uint64_t o = off[i];
    for (uint64_t t = 0; t < K; ++t) {
        uint32_t q[MG];   // the record of each genome this combination takes (two: every kept one)
        int64_t sv[MG];
        uint32_t pv[MG];
        for (int g = 0; g < G; ++g) { sv[g] = 0; pv[g] = 0; q[g] = 0; }
        if (!two) {   // odometer: the last genome varies fastest (MatchFinder.cpp:371-390)
            uint64_t rem = t;
            for (int g = G - 1; g >= 0; --g) {
                if (!c[g]) continue;
                q[g] = (uint32_t)(rem % c[g]);
                rem /= c[g];
            }
        }
        uint32_t seen[MG];
        for (int g = 0; g < G; ++g) seen[g] = 0;
        for (uint64_t j = i; j < N && v.gkey(j) == k0; ++j) {
            const RecFields r = v.get(j);
            const int g = genome_of(gt, r.idx);
            const uint32_t s = seen[g]++;
            if (s >= c[g]) continue;   // past the genome's first enum_tol records
            if (two || s == q[g]) {    // (two: the list's records, the later one of a genome wins as in en_emit)
                sv[g] = (int64_t)(r.idx - gt.base[g]) + 1;
                pv[g] = r.par;
            }
        }
        // SetDirection (MemHash.cpp:189-203) + CalculateOffset (MatchHashEntry.cpp:141-160)
        int ref = -1;
        for (int g = 0; g < G && ref < 0; ++g)
            if (sv[g] != 0) ref = g;
        int64_t offset = 0;
        for (int g = ref + 1; g < G; ++g) {
            if (sv[g] == 0) continue;
            if (pv[g] != pv[ref]) sv[g] = -sv[g];
            offset += sv[g] - sv[ref] - (sv[g] < 0 ? (int64_t)L : 0);
        }
        int64_t* row = rows + (o + t) * (uint64_t)(G + 1);
        for (int g = 0; g < G; ++g) row[g] = sv[g];
        row[G] = offset;
    }
}

inline dim3 grid_of(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

template <typename View>
hipError_t launch_pairwise_count(View v, uint64_t N, const GenomeTable& gt, uint32_t* npairs, void* ctr,
                                 hipStream_t st) {
    if (N == 0) return hipSuccess;
    if (gt.G > 32)
        hipLaunchKernelGGL((pw_count_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, npairs, (DevCounters*)ctr);
    else
        hipLaunchKernelGGL((pw_count_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, npairs, (DevCounters*)ctr);
    return hipGetLastError();
}

template <typename View>
hipError_t launch_pairwise_emit(View v, uint64_t N, const GenomeTable& gt, int L, const uint32_t* npairs,
                                const uint32_t* off, int64_t* rows, hipStream_t st) {
    if (N == 0) return hipSuccess;
    if (gt.G > 32)
        hipLaunchKernelGGL((pw_emit_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, L, npairs, off, rows);
    else
        hipLaunchKernelGGL((pw_emit_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, L, npairs, off, rows);
    return hipGetLastError();
}

template <typename View>
hipError_t launch_enum_count(View v, uint64_t N, const GenomeTable& gt, const MatchParams& mp, uint32_t* ncalls,
                             void* ctr, hipStream_t st) {
    if (N == 0) return hipSuccess;
    const bool walk = mp.enum_tol > (uint32_t)kEnumMax;
    if (gt.G > 32 && walk)
        hipLaunchKernelGGL((en_count_walk_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, ncalls, (DevCounters*)ctr);
    else if (walk)
        hipLaunchKernelGGL((en_count_walk_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, ncalls, (DevCounters*)ctr);
    else if (gt.G > 32)
        hipLaunchKernelGGL((en_count_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, ncalls, (DevCounters*)ctr);
    else
        hipLaunchKernelGGL((en_count_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, ncalls, (DevCounters*)ctr);
    return hipGetLastError();
}

template <typename View>
hipError_t launch_enum_emit(View v, uint64_t N, const GenomeTable& gt, const MatchParams& mp, int L,
                            const uint32_t* ncalls, const uint32_t* off, int64_t* rows, hipStream_t st) {
    if (N == 0) return hipSuccess;
    const bool walk = mp.enum_tol > (uint32_t)kEnumMax;
    if (gt.G > 32 && walk)
        hipLaunchKernelGGL((en_emit_walk_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, L, ncalls, off, rows);
    else if (walk)
        hipLaunchKernelGGL((en_emit_walk_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, L, ncalls, off, rows);
    else if (gt.G > 32)
        hipLaunchKernelGGL((en_emit_kernel<64, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, L, ncalls, off, rows);
    else
        hipLaunchKernelGGL((en_emit_kernel<32, View>), grid_of(N), dim3(256), 0, st, v, N, gt, mp, L, ncalls, off, rows);
    return hipGetLastError();
}

#define MUMS_INST_PW(V)                                                                                             \
    template hipError_t launch_pairwise_count<V>(V, uint64_t, const GenomeTable&, uint32_t*, void*, hipStream_t);   \
    template hipError_t launch_pairwise_emit<V>(V, uint64_t, const GenomeTable&, int, const uint32_t*,              \
                                                const uint32_t*, int64_t*, hipStream_t);                            \
    template hipError_t launch_enum_count<V>(V, uint64_t, const GenomeTable&, const MatchParams&, uint32_t*, void*, \
                                             hipStream_t);                                                          \
    template hipError_t launch_enum_emit<V>(V, uint64_t, const GenomeTable&, const MatchParams&, int,               \
                                            const uint32_t*, const uint32_t*, int64_t*, hipStream_t);
MUMS_INST_PW(PairView<uint32_t>)
MUMS_INST_PW(PairView<uint64_t>)
typedef PairView<uint64_t, uint64_t> PairView64;
MUMS_INST_PW(PairView64)

namespace {
// chunk of the chunked mode (records key_low(31) << 33 | index, the 2w+1-31 top key bits
// implicit: bucket j of the chunk is digit digit0 + j) as (full ckey, 64-bit index) pairs
__global__ void chunk_pairs_kernel(const uint64_t* __restrict__ rec, uint64_t n, const uint32_t* __restrict__ bstart,
                                   uint32_t nb, uint64_t digit0, uint64_t* __restrict__ key, uint64_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = nb;   // bucket of i: the last start <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)bstart[mid] <= i) lo = mid;
        else hi = mid;
    }
    const uint64_t r = rec[i];
    key[i] = ((digit0 + lo) << 31) | (r >> 33);
    idx[i] = r & ((1ull << 33) - 1);
}
}  // namespace

hipError_t launch_chunk_pairs(const uint64_t* rec, uint64_t n, const uint32_t* bstart, uint32_t nb, uint64_t digit0,
                              uint64_t* key, uint64_t* idx, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(chunk_pairs_kernel, grid_of(n), dim3(256), 0, st, rec, n, bstart, nb, digit0, key, idx);
    return hipGetLastError();
}

}  // namespace mums
