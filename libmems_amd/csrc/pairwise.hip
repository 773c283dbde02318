// pairwise.hip -- PairwiseMatchFinder (PairwiseMatchFinder.h:23-33).
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

namespace mums {
namespace {

template <typename View>
__device__ __forceinline__ bool pw_head(const View& v, uint64_t i) {
    return i == 0 || v.gkey(i) != v.gkey(i - 1);
}

// genomes present exactly once in the group starting at head h; *size = group size
// (walk stops past MER_REPEAT_LIMIT: SearchRange skips such groups, MatchFinder.cpp:215)
template <typename View>
__device__ __forceinline__ uint32_t pw_unique(const View& v, uint64_t h, uint64_t N, const GenomeTable& gt,
                                              uint32_t* size) {
    const uint64_t k0 = v.gkey(h);
    uint32_t seen = 0, dup = 0, n = 0;
    for (uint64_t j = h; j < N && v.gkey(j) == k0; ++j) {
        if (++n > (uint32_t)kRepeatLimit) break;
        const uint32_t b = 1u << genome_of(gt, v.gidx(j));
        dup |= seen & b;
        seen |= b;
    }
    *size = n;
    return seen & ~dup;
}

template <typename View>
__global__ void pw_count_kernel(View v, uint64_t N, GenomeTable gt, uint32_t* __restrict__ npairs,
                                DevCounters* __restrict__ ctr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t c = 0;
    if (pw_head(v, i)) {
        uint32_t size = 0;
        const uint32_t u = pw_unique(v, i, N, gt, &size);
        const uint32_t k = (uint32_t)__builtin_popcount(u);
        if (size > (uint32_t)kRepeatLimit) atomicAdd(&ctr->repeat_limit, 1ull);
        else if (size >= 2) c = k * (k - 1) / 2;
    }
    npairs[i] = c;
}

// PairwiseMatchFinder::EnumerateMatches pairs (a < b over the single-copy genomes) ->
// MemHash::HashMatch (MemHash.cpp:167-187): starts pos+1, SetDirection (:189-203: the
// lower genome is the reference, the other is negated when its strand parity differs),
// CalculateOffset (MatchHashEntry.cpp:141-160).
template <typename View>
__global__ void pw_emit_kernel(View v, uint64_t N, GenomeTable gt, int L, const uint32_t* __restrict__ npairs,
                               const uint32_t* __restrict__ off, int64_t* __restrict__ rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || npairs[i] == 0) return;
    const int G = gt.G;
    uint32_t size = 0;
    const uint32_t u = pw_unique(v, i, N, gt, &size);
    int64_t s[kMaxG];
    uint32_t par[kMaxG];
    const uint64_t k0 = v.gkey(i);
    for (uint64_t j = i; j < N && v.gkey(j) == k0; ++j) {
        const RecFields r = v.get(j);
        const int g = genome_of(gt, r.idx);
        if ((u >> g) & 1u) {
            s[g] = (int64_t)(r.idx - gt.base[g]) + 1;
            par[g] = r.par;
        }
    }
    uint64_t o = off[i];
    for (int a = 0; a < G; ++a) {
        if (!((u >> a) & 1u)) continue;
        for (int b = a + 1; b < G; ++b) {
            if (!((u >> b) & 1u)) continue;
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

inline dim3 grid_of(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

template <typename View>
hipError_t launch_pairwise_count(View v, uint64_t N, const GenomeTable& gt, uint32_t* npairs, void* ctr,
                                 hipStream_t st) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(pw_count_kernel<View>, grid_of(N), dim3(256), 0, st, v, N, gt, npairs, (DevCounters*)ctr);
    return hipGetLastError();
}

template <typename View>
hipError_t launch_pairwise_emit(View v, uint64_t N, const GenomeTable& gt, int L, const uint32_t* npairs,
                                const uint32_t* off, int64_t* rows, hipStream_t st) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(pw_emit_kernel<View>, grid_of(N), dim3(256), 0, st, v, N, gt, L, npairs, off, rows);
    return hipGetLastError();
}

#define MUMS_INST_PW(V)                                                                                             \
    template hipError_t launch_pairwise_count<V>(V, uint64_t, const GenomeTable&, uint32_t*, void*, hipStream_t);   \
    template hipError_t launch_pairwise_emit<V>(V, uint64_t, const GenomeTable&, int, const uint32_t*,              \
                                                const uint32_t*, int64_t*, hipStream_t);
MUMS_INST_PW(PairView<uint32_t>)
MUMS_INST_PW(PairView<uint64_t>)

}  // namespace mums
