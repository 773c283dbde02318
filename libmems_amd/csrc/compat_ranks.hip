// compat_ranks.hip -- ParallelMemHash compat over several ranks.
//
// Every rank runs the chunked compat search (compat.hip) on a contiguous range of the chunks
// with tables of its own (mums_capi.hip, ctx->compat_ranks > 1); the bucket owners then re-add
// the ranks' tables rank after rank the way MergeTable (ParallelMemHash.cpp:105-121) re-adds a
// thread table: every entry, in bucket / vector order, through AddHashEntry's lower_bound
// insert or collision (MemHash.cpp:209-251).  The oracle's model of that schedule
// (oracle_find_matches with parallel_compat = 16 + ranks) gives the one-thread MatchList.
//
// One merge step, accumulated table A and the next rank's table B (each bucket in vector order):
//   rank_lb_kernel    : lower_bound of B[k] in A_b (std::lower_bound's probes), B[k] a duplicate
//                       when equal to A_b[lb]; B must ascend strictly under MheCompare
//   scan of the non-duplicate flags
//   rank_place_a / _b : the union: A[i] after the non-duplicate B entries below it, B[k] at
//                       lb + the non-duplicate B entries before it (ids per bucket, tblcat)
//   rank_check_kernel : the union ascends pair by pair and no entry Contains another of its
//                       class (first start, genome set): MheCompare (MatchHashEntry.h:121-143)
//                       is then the lexicographic order of (first start, genome set, starts) on
//                       it, a strict weak order, and the sequential inserts land where the
//                       union puts them
//   buckets that fail a check take the exact sequential merge (compat_merge_fix_kernel) from A_b.
#include <hip/hip_runtime.h>

#include "match_device.h"
#include "mums_internal.h"

namespace mums {
namespace {

constexpr int kWindowCap = 64;   // entries scanned for a containing / contained neighbour

// last b with off[b] <= k (off: nb + 1 non-decreasing offsets, k < off[nb])
__device__ __forceinline__ uint32_t bucket_at(const uint32_t* __restrict__ off, uint32_t nb, uint64_t k) {
    uint32_t lo = 0, n = nb + 1;   // upper_bound(off, off + nb + 1, k) - 1
    while (n > 0) {
        const uint32_t h = n >> 1;
        if ((uint64_t)off[lo + h] <= k) { lo += h + 1; n -= h + 1; }
        else n = h;
    }
    return lo - 1;
}

template <int MG>
__device__ __forceinline__ bool mhe_same(const Mhe<MG>& a, const Mhe<MG>& b) {
    bool eq = a.len == b.len;
    #pragma unroll
    for (int g = 0; g < MG; ++g) eq = eq && a.s[g] == b.s[g];
    return eq;
}

template <int MG>
__device__ __forceinline__ bool same_class(const Mhe<MG>& a, const Mhe<MG>& b) {
    bool eq = true;
    #pragma unroll
    for (int g = 0; g < MG; ++g) eq = eq && ((a.s[g] == 0) == (b.s[g] == 0));
    return eq;
}

// std::lower_bound over the pool rows [first0, first0 + n)
template <int MG>
__device__ __forceinline__ uint32_t lower_bound_rows(const int64_t* __restrict__ pool, int G, uint64_t first0, uint32_t n,
                                                     const Mhe<MG>& val) {
    uint32_t first = 0, len = n;
    Mhe<MG> e;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        load_entry(pool, (uint32_t)(first0 + mid), G, e);
        if (mhe_less(e, val)) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

// rows of the context's table in bucket order (emit_kernel's walk, whole pool rows)
__global__ __launch_bounds__(kBlock) void rank_rows_kernel(const uint32_t* __restrict__ obase,
                                                           const uint32_t* __restrict__ bstart,
                                                           const uint32_t* __restrict__ tbl,
                                                           const int64_t* __restrict__ pool, int G, uint32_t Tb,
                                                           uint64_t M, int64_t* __restrict__ rows) {
    const uint64_t o = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (o >= M) return;
    const uint32_t b = bucket_at(obase, Tb - 1, o);
    const uint32_t id = tbl[bstart[b] + (uint32_t)(o - obase[b])];
    const int64_t* e = pool + (uint64_t)id * (uint64_t)(G + 2);
    int64_t* r = rows + o * (uint64_t)(G + 2);
    for (int g = 0; g < G + 2; ++g) r[g] = e[g];
}

// B[k] (pool row nA + k): its lower_bound in A_b, the duplicate flag, B's own order
template <int MG>
__global__ __launch_bounds__(kBlock) void rank_lb_kernel(const int64_t* __restrict__ pool, int G, uint32_t nA,
                                                         const uint32_t* __restrict__ offA,
                                                         const uint32_t* __restrict__ offB, uint32_t nb, uint32_t nB,
                                                         uint32_t* __restrict__ lbA, uint32_t* __restrict__ nd,
                                                         uint32_t* __restrict__ bad) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= nB) return;
    const uint32_t b = bucket_at(offB, nb, k);
    Mhe<MG> e;
    load_entry(pool, nA + k, G, e);
    const uint32_t a0 = offA[b], na = offA[b + 1] - a0;
    const uint32_t lb = lower_bound_rows<MG>(pool, G, a0, na, e);
    bool dup = false, fail = false;
    if (lb < na) {
        Mhe<MG> x;
        load_entry(pool, a0 + lb, G, x);
        dup = mhe_same(x, e);
        fail = !dup && !mhe_less(x, e) && !mhe_less(e, x);   // equivalent, not equal: Contains
    }
    if (k > offB[b]) {
        Mhe<MG> p;
        load_entry(pool, nA + k - 1, G, p);
        fail = fail || !(mhe_less(p, e) && !mhe_less(e, p));
    }
    if (fail) bad[b] = 1u;
    lbA[k] = lb;
    nd[k] = dup ? 0u : 1u;
}

// A[i]: its place in the union = i + the non-duplicate B entries below it (ndp: exclusive
// prefix of the non-duplicate flags, nB + 1 words)
template <int MG>
__global__ __launch_bounds__(kBlock) void rank_place_a_kernel(const int64_t* __restrict__ pool, int G, uint32_t nA,
                                                              const uint32_t* __restrict__ offA,
                                                              const uint32_t* __restrict__ offB,
                                                              const uint32_t* __restrict__ catoff, uint32_t nb,
                                                              const uint32_t* __restrict__ ndp,
                                                              uint32_t* __restrict__ tblcat) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nA) return;
    const uint32_t b = bucket_at(offA, nb, i);
    Mhe<MG> e;
    load_entry(pool, i, G, e);
    const uint32_t b0 = offB[b], nbb = offB[b + 1] - b0;
    const uint32_t lb = lower_bound_rows<MG>(pool, G, (uint64_t)nA + b0, nbb, e);
    tblcat[catoff[b] + (i - offA[b]) + (ndp[b0 + lb] - ndp[b0])] = i;
}

__global__ __launch_bounds__(kBlock) void rank_place_b_kernel(uint32_t nA, const uint32_t* __restrict__ offB,
                                                              const uint32_t* __restrict__ catoff, uint32_t nb,
                                                              uint32_t nB, const uint32_t* __restrict__ lbA,
                                                              const uint32_t* __restrict__ ndp,
                                                              uint32_t* __restrict__ tblcat) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= nB || ndp[k + 1] == ndp[k]) return;   // a duplicate: AddHashEntry's collision
    const uint32_t b = bucket_at(offB, nb, k);
    tblcat[catoff[b] + lbA[k] + (ndp[k] - ndp[offB[b]])] = nA + k;
}

__global__ __launch_bounds__(kBlock) void rank_sizes_kernel(const uint32_t* __restrict__ offA,
                                                            const uint32_t* __restrict__ offB,
                                                            const uint32_t* __restrict__ ndp, uint32_t nb,
                                                            uint32_t* __restrict__ catoff, uint32_t* __restrict__ tsize) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b > nb) return;
    catoff[b] = offA[b] + offB[b];
    if (b < nb) tsize[b] = (offA[b + 1] - offA[b]) + (ndp[offB[b + 1]] - ndp[offB[b]]);
}

// the union of every bucket: ascending pair by pair, first starts forward, no Contains pair
// inside a class (a contained entry starts inside its container: the scan stops past it)
template <int MG>
__global__ __launch_bounds__(kBlock) void rank_check_kernel(const int64_t* __restrict__ pool, int G,
                                                            const uint32_t* __restrict__ catoff,
                                                            const uint32_t* __restrict__ tsize, uint32_t nb,
                                                            uint32_t ncat, const uint32_t* __restrict__ tblcat,
                                                            uint32_t* __restrict__ bad) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= ncat) return;
    const uint32_t b = bucket_at(catoff, nb, g);
    const uint32_t i = g - catoff[b], n = tsize[b];
    if (i >= n) return;
    Mhe<MG> e, x;
    load_entry(pool, tblcat[g], G, e);
    const int fa = first_start(e);
    const int64_t s0 = start_at(e, fa);
    bool fail = s0 <= 0;
    if (i > 0) {
        load_entry(pool, tblcat[g - 1], G, x);
        fail = fail || !(mhe_less(x, e) && !mhe_less(e, x));
    }
    uint32_t j = i + 1;
    for (; !fail && j < n && j <= i + kWindowCap; ++j) {
        load_entry(pool, tblcat[catoff[b] + j], G, x);
        if (!same_class(e, x) || start_at(x, fa) > s0 + e.len) break;
        fail = mhe_contains(e, x) || mhe_contains(x, e);
    }
    if (!fail && j < n && j > i + kWindowCap) fail = true;   // window not closed: the exact merge decides
    if (fail) bad[b] = 1u;
}

// buckets that failed a check: [A_b ids, B_b ids] for the sequential merge from |A_b|
__global__ __launch_bounds__(kBlock) void rank_exact_init_kernel(uint32_t nA, const uint32_t* __restrict__ offA,
                                                                 const uint32_t* __restrict__ offB,
                                                                 const uint32_t* __restrict__ catoff, uint32_t nb,
                                                                 uint32_t ncat, const uint32_t* __restrict__ bad,
                                                                 uint32_t* __restrict__ tblcat,
                                                                 uint32_t* __restrict__ tsize,
                                                                 uint32_t* __restrict__ first_fail) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= ncat) return;
    const uint32_t b = bucket_at(catoff, nb, g);
    if (!bad[b]) return;
    const uint32_t i = g - catoff[b], na = offA[b + 1] - offA[b], nbb = offB[b + 1] - offB[b];
    tblcat[g] = i < na ? offA[b] + i : nA + offB[b] + (i - na);
    if (i == 0) {
        tsize[b] = na + nbb;
        first_fail[b] = na;
    }
}

__global__ __launch_bounds__(kBlock) void rank_gather_kernel(const int64_t* __restrict__ pool, int G,
                                                             const uint32_t* __restrict__ catoff,
                                                             const uint32_t* __restrict__ tsize, uint32_t nb,
                                                             uint32_t ncat, const uint32_t* __restrict__ tblcat,
                                                             const uint32_t* __restrict__ newoff,
                                                             int64_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= ncat) return;
    const uint32_t b = bucket_at(catoff, nb, g);
    const uint32_t i = g - catoff[b];
    if (i >= tsize[b]) return;
    const int64_t* e = pool + (uint64_t)tblcat[g] * (uint64_t)(G + 2);
    int64_t* r = out + (uint64_t)(newoff[b] + i) * (uint64_t)(G + 2);
    for (int k = 0; k < G + 2; ++k) r[k] = e[k];
}

__global__ __launch_bounds__(kBlock) void rank_list_kernel(const int64_t* __restrict__ rows, int G, uint64_t M,
                                                           uint64_t* __restrict__ out_len, int64_t* __restrict__ out_s) {
    const uint64_t o = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (o >= M) return;
    const int64_t* e = rows + o * (uint64_t)(G + 2);
    out_len[o] = (uint64_t)e[0];
    for (int g = 0; g < G; ++g) out_s[o * (uint64_t)G + g] = e[2 + g];
}

inline dim3 grid_n(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace

hipError_t launch_rank_rows(const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl, const int64_t* pool,
                            int G, uint32_t Tb, uint64_t M, int64_t* rows, hipStream_t st) {
    if (M == 0) return hipSuccess;
    hipLaunchKernelGGL(rank_rows_kernel, grid_n(M), dim3(kBlock), 0, st, obase, bstart, tbl, pool, G, Tb, M, rows);
    return hipGetLastError();
}

hipError_t launch_rank_lb(const int64_t* pool, int G, uint32_t nA, const uint32_t* offA, const uint32_t* offB,
                          uint32_t nb, uint32_t nB, uint32_t* lbA, uint32_t* nd, uint32_t* bad, hipStream_t st) {
    if (nB == 0) return hipSuccess;
#define MUMS_RANK_LB(MGV) \
    hipLaunchKernelGGL(rank_lb_kernel<MGV>, grid_n(nB), dim3(kBlock), 0, st, pool, G, nA, offA, offB, nb, nB, lbA, nd, bad)
    if (G <= 4) MUMS_RANK_LB(4);
    else if (G <= 8) MUMS_RANK_LB(8);
    else if (G <= 16) MUMS_RANK_LB(16);
    else if (G <= 32) MUMS_RANK_LB(32);
    else MUMS_RANK_LB(64);
#undef MUMS_RANK_LB
    return hipGetLastError();
}

hipError_t launch_rank_place(const int64_t* pool, int G, uint32_t nA, const uint32_t* offA, const uint32_t* offB,
                             uint32_t nb, uint32_t nB, const uint32_t* lbA, const uint32_t* ndp, uint32_t* catoff,
                             uint32_t* tsize, uint32_t* tblcat, hipStream_t st) {
    hipLaunchKernelGGL(rank_sizes_kernel, grid_n((uint64_t)nb + 1), dim3(kBlock), 0, st, offA, offB, ndp, nb, catoff,
                       tsize);
    if (nA) {
#define MUMS_RANK_PA(MGV)                                                                                          \
    hipLaunchKernelGGL(rank_place_a_kernel<MGV>, grid_n(nA), dim3(kBlock), 0, st, pool, G, nA, offA, offB, catoff, nb, \
                       ndp, tblcat)
        if (G <= 4) MUMS_RANK_PA(4);
        else if (G <= 8) MUMS_RANK_PA(8);
        else if (G <= 16) MUMS_RANK_PA(16);
        else if (G <= 32) MUMS_RANK_PA(32);
        else MUMS_RANK_PA(64);
#undef MUMS_RANK_PA
    }
    if (nB)
        hipLaunchKernelGGL(rank_place_b_kernel, grid_n(nB), dim3(kBlock), 0, st, nA, offB, catoff, nb, nB, lbA, ndp,
                           tblcat);
    return hipGetLastError();
}

hipError_t launch_rank_check(const int64_t* pool, int G, const uint32_t* catoff, const uint32_t* tsize, uint32_t nb,
                             uint32_t ncat, const uint32_t* tblcat, uint32_t* bad, hipStream_t st) {
    if (ncat == 0) return hipSuccess;
#define MUMS_RANK_CHECK(MGV) \
    hipLaunchKernelGGL(rank_check_kernel<MGV>, grid_n(ncat), dim3(kBlock), 0, st, pool, G, catoff, tsize, nb, ncat, tblcat, bad)
    if (G <= 4) MUMS_RANK_CHECK(4);
    else if (G <= 8) MUMS_RANK_CHECK(8);
    else if (G <= 16) MUMS_RANK_CHECK(16);
    else if (G <= 32) MUMS_RANK_CHECK(32);
    else MUMS_RANK_CHECK(64);
#undef MUMS_RANK_CHECK
    return hipGetLastError();
}

hipError_t launch_rank_exact_init(uint32_t nA, const uint32_t* offA, const uint32_t* offB, const uint32_t* catoff,
                                  uint32_t nb, uint32_t ncat, const uint32_t* bad, uint32_t* tblcat, uint32_t* tsize,
                                  uint32_t* first_fail, hipStream_t st) {
    hipError_t e = hipMemsetAsync(first_fail, 0xFF, (size_t)nb * 4 + 4, st);
    if (e != hipSuccess || ncat == 0) return e;
    hipLaunchKernelGGL(rank_exact_init_kernel, grid_n(ncat), dim3(kBlock), 0, st, nA, offA, offB, catoff, nb, ncat, bad,
                       tblcat, tsize, first_fail);
    return hipGetLastError();
}

hipError_t launch_rank_gather(const int64_t* pool, int G, const uint32_t* catoff, const uint32_t* tsize, uint32_t nb,
                              uint32_t ncat, const uint32_t* tblcat, const uint32_t* newoff, int64_t* out,
                              hipStream_t st) {
    if (ncat == 0) return hipSuccess;
    hipLaunchKernelGGL(rank_gather_kernel, grid_n(ncat), dim3(kBlock), 0, st, pool, G, catoff, tsize, nb, ncat, tblcat,
                       newoff, out);
    return hipGetLastError();
}

hipError_t launch_rank_list(const int64_t* rows, int G, uint64_t M, uint64_t* out_len, int64_t* out_s, hipStream_t st) {
    if (M == 0) return hipSuccess;
    hipLaunchKernelGGL(rank_list_kernel, grid_n(M), dim3(kBlock), 0, st, rows, G, M, out_len, out_s);
    return hipGetLastError();
}

}  // namespace mums
