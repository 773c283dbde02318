// overlaps.hip -- EliminateOverlaps (libMems/Aligner.cpp:62-176) on the device MatchList
// (the step after MemHash::FindMatches in both aligners).
//
// Per genome seqI the reference std::sorts its vector of Match* with SingleStartComparator
// (AbstractMatch.h:324-351: key = LeftEnd(seqI) = |start|, NO_MATCH 0 first) and walks it
// once, cropping / deleting the smaller of every overlapping pair and appending the cut-off
// overlaps (minus genome seqI) as new matches.
//
//   * The order of equal keys is part of the result (it is the MatchList order the caller
//     sees, and it decides which of two tied matches is matchI), so the sort here replays
//     libstdc++'s introsort (GCC bits/stl_algo.h) exactly, level-parallel: every segment of
//     a level runs __move_median_to_first, and its __unguarded_partition is computed in
//     closed form -- the k-th left stopper (key >= pivot) swaps with the k-th right stopper
//     (key <= pivot, from the right) while it lies left of it, and the cut is the
//     (K+1)-th left stopper or the K-th right stopper, whichever comes first (K = swaps).
//     Segments at depth 0 run the heap sort of __partial_sort on one lane; leaves (<= 16)
//     are insertion-sorted (the final insertion sort never moves an element across a leaf).
//   * Matches only shrink, so a match whose LeftEnd is at or past the end of every match
//     before it in the sorted order never interacts with them: the sorted list splits into
//     clusters (running max of the ends) and each cluster is replayed sequentially on one
//     lane.  New matches are numbered (cluster, creation order) and appended in that order.
#include <algorithm>
#include <vector>

#include "mums_internal.h"

namespace mums {
namespace {

constexpr uint32_t kDel = 0xFFFFFFFFu;
constexpr uint32_t kLeaf = 16;   // _S_threshold

struct SortSeg {
    uint32_t f, l, d, pad;
};

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

__device__ __forceinline__ void swap_kv(uint64_t* K, uint32_t* V, uint32_t a, uint32_t b) {
    const uint64_t k = K[a];
    K[a] = K[b];
    K[b] = k;
    const uint32_t v = V[a];
    V[a] = V[b];
    V[b] = v;
}

// __move_median_to_first(first, first + 1, mid, last - 1); piv[s] = the pivot key
__global__ void median_kernel(uint64_t* K, uint32_t* V, const SortSeg* __restrict__ segs, uint32_t S,
                              uint64_t* __restrict__ piv) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const SortSeg g = segs[s];
    const uint32_t a = g.f + 1, b = g.f + (g.l - g.f) / 2, c = g.l - 1;
    const uint64_t ka = K[a], kb = K[b], kc = K[c];
    uint32_t m;
    if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
    else m = ka < kc ? a : (kb < kc ? c : b);
    swap_kv(K, V, g.f, m);
    piv[s] = K[g.f];
}

// active segment holding position i (segments sorted by f), or -1
__device__ __forceinline__ int seg_of(const SortSeg* __restrict__ segs, uint32_t S, uint32_t i) {
    uint32_t lo = 0, n = S;   // last segment with f <= i
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (segs[lo + h].f <= i) { lo += h + 1; n -= h + 1; } else n = h;
    }
    if (lo == 0) return -1;
    const SortSeg g = segs[lo - 1];
    return (i > g.f && i < g.l) ? (int)(lo - 1) : -1;
}

// stopper flags of the partition range [f + 1, l): fl = key >= pivot, fr = key <= pivot
__global__ void classify_kernel(const uint64_t* __restrict__ K, const SortSeg* __restrict__ segs, uint32_t S,
                                const uint64_t* __restrict__ piv, uint32_t n, uint32_t* __restrict__ fl,
                                uint32_t* __restrict__ fr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    uint32_t a = 0, b = 0;
    if (i < n) {
        const int s = seg_of(segs, S, i);
        if (s >= 0) {
            const uint64_t p = piv[s], k = K[i];
            a = !(k < p);
            b = !(p < k);
        }
    }
    fl[i] = a;
    fr[i] = b;
}

// after the exclusive scans: Lpos[f + 1 + k] = k-th left stopper (0-based, from the left),
// Rpos[f + 1 + k] = k-th right stopper (from the right)
__global__ void rank_kernel(const SortSeg* __restrict__ segs, uint32_t S, uint32_t n, const uint32_t* __restrict__ fl,
                            const uint32_t* __restrict__ fr, uint32_t* __restrict__ Lpos,
                            uint32_t* __restrict__ Rpos) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int s = seg_of(segs, S, i);
    if (s < 0) return;
    const SortSeg g = segs[s];
    if (fl[i + 1] != fl[i]) Lpos[g.f + 1 + (fl[i] - fl[g.f + 1])] = i;
    if (fr[i + 1] != fr[i]) Rpos[g.f + 1 + (fr[g.l] - fr[i + 1])] = i;
}

// pair k swaps iff L_k < R_k (a prefix of k); nswap[s] = K
__global__ void swap_kernel(uint64_t* K, uint32_t* V, const SortSeg* __restrict__ segs, uint32_t S, uint32_t n,
                            const uint32_t* __restrict__ fl, const uint32_t* __restrict__ fr,
                            const uint32_t* __restrict__ Lpos, const uint32_t* __restrict__ Rpos,
                            uint32_t* __restrict__ nswap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || fl[i + 1] == fl[i]) return;
    const int s = seg_of(segs, S, i);
    if (s < 0) return;
    const SortSeg g = segs[s];
    const uint32_t k = fl[i] - fl[g.f + 1];
    const uint32_t cntR = fr[g.l] - fr[g.f + 1];
    if (k >= cntR) return;
    const uint32_t j = Rpos[g.f + 1 + k];
    if (!(i < j)) return;
    swap_kv(K, V, i, j);
    // the swapping pairs are a prefix: its last pair writes the count (no per-swap atomic
    // on one counter, which serialises large segments)
    const uint32_t cntL = fl[g.l] - fl[g.f + 1];
    if (k + 1 >= cntL || k + 1 >= cntR || !(Lpos[g.f + 1 + k + 1] < Rpos[g.f + 1 + k + 1])) nswap[s] = k + 1;
}

// cut = min(L_{K+1}, R_K) (R_0 = l); children [f, cut), [cut, l) at depth d - 1 into
// out[2s], out[2s + 1] with act = 1 when they partition again; depth-0 children > 16 go to
// the heap list
__global__ void cut_kernel(const SortSeg* __restrict__ segs, uint32_t S, const uint32_t* __restrict__ fl,
                           const uint32_t* __restrict__ Lpos, const uint32_t* __restrict__ Rpos,
                           const uint32_t* __restrict__ nswap, SortSeg* __restrict__ out, uint32_t* __restrict__ act,
                           SortSeg* __restrict__ heap, uint32_t* __restrict__ nheap, uint8_t* __restrict__ bound) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0) act[2 * S] = 0;
    if (s >= S) return;
    const SortSeg g = segs[s];
    const uint32_t K = nswap[s];
    const uint32_t cntL = fl[g.l] - fl[g.f + 1];
    uint32_t cut = K > 0 ? Rpos[g.f + 1 + K - 1] : g.l;
    if (K < cntL) cut = min(cut, Lpos[g.f + 1 + K]);
    bound[cut] = 1;
    const uint32_t d = g.d - 1;
    const SortSeg c0{g.f, cut, d, 0}, c1{cut, g.l, d, 0};
    const SortSeg ch[2] = {c0, c1};
    for (int t = 0; t < 2; ++t) {
        const bool big = ch[t].l - ch[t].f > kLeaf;
        out[2 * s + t] = ch[t];
        act[2 * s + t] = (big && d > 0) ? 1u : 0u;
        if (big && d == 0) heap[atomicAdd(nheap, 1u)] = ch[t];
    }
}

__global__ void compact_segs_kernel(const SortSeg* __restrict__ in, const uint32_t* __restrict__ act, uint32_t n2,
                                    SortSeg* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n2 && act[i + 1] != act[i]) out[act[i]] = in[i];
}

// libstdc++ heap sort of one segment (std::__partial_sort(first, last, last): make_heap,
// then __pop_heap from the back; stl_heap.h __adjust_heap / __push_heap)
__device__ void adjust_heap(uint64_t* K, uint32_t* V, int64_t hole, int64_t len, uint64_t vk, uint32_t vv) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (K[child] < K[child - 1]) child--;
        K[hole] = K[child];
        V[hole] = V[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        K[hole] = K[child - 1];
        V[hole] = V[child - 1];
        hole = child - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && K[parent] < vk) {
        K[hole] = K[parent];
        V[hole] = V[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    K[hole] = vk;
    V[hole] = vv;
}

__global__ void heap_kernel(uint64_t* K, uint32_t* V, const SortSeg* __restrict__ segs, uint32_t S) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    uint64_t* k = K + segs[s].f;
    uint32_t* v = V + segs[s].f;
    int64_t len = segs[s].l - segs[s].f;
    for (int64_t parent = (len - 2) / 2;; --parent) {   // make_heap
        adjust_heap(k, v, parent, len, k[parent], v[parent]);
        if (parent == 0) break;
    }
    while (len > 1) {   // sort_heap
        --len;
        const uint64_t vk = k[len];
        const uint32_t vv = v[len];
        k[len] = k[0];
        v[len] = v[0];
        adjust_heap(k, v, 0, len, vk, vv);
    }
}

// stable insertion sort of every leaf (<= 16 elements between two bounds)
__global__ void leaf_kernel(uint64_t* K, uint32_t* V, const uint8_t* __restrict__ bound, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !bound[i]) return;
    uint32_t e = i + 1;
    while (e <= n && e - i <= kLeaf && !bound[e]) ++e;
    if (e - i > kLeaf || e > n) return;   // a heap-sorted segment
    for (uint32_t a = i + 1; a < e; ++a) {
        const uint64_t vk = K[a];
        const uint32_t vv = V[a];
        uint32_t b = a;
        while (b > i && vk < K[b - 1]) {
            K[b] = K[b - 1];
            V[b] = V[b - 1];
            --b;
        }
        K[b] = vk;
        V[b] = vv;
    }
}

// ---- the EliminateOverlaps pass ------------------------------------------------------
__global__ void keys_kernel(const uint32_t* __restrict__ V, const int64_t* __restrict__ ps, int G, int seqI,
                            uint32_t n, uint64_t* __restrict__ K) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = ps[(uint64_t)V[i] * G + seqI];
    K[i] = (uint64_t)(s < 0 ? -s : s);
}

// cluster heads: flag[i] = 1 at the first defined match and wherever LeftEnd >= every end
// before it (ends = LeftEnd + len; tile maxima in tmax for the second pass)
constexpr int kEoTile = 1024;
__global__ void tile_max_kernel(const uint64_t* __restrict__ K, const uint32_t* __restrict__ V,
                                const int64_t* __restrict__ plen, uint32_t n, uint64_t* __restrict__ tmax) {
    __shared__ uint64_t red[kBlock];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    uint64_t m = 0;
    for (uint32_t i = t * kEoTile + tid; i < min(n, (t + 1) * kEoTile); i += kBlock)
        if (K[i]) m = max(m, K[i] + (uint64_t)plen[V[i]]);
    red[tid] = m;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (tid < w) red[tid] = max(red[tid], red[tid + w]);
        __syncthreads();
    }
    if (tid == 0) tmax[t] = red[0];
}

__global__ void tile_prefix_kernel(uint64_t* tmax, uint32_t T) {   // exclusive max-scan, one lane
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t t = 0; t < T; ++t) {
            const uint64_t x = tmax[t];
            tmax[t] = run;
            run = max(run, x);
        }
    }
}

__global__ void heads_kernel(const uint64_t* __restrict__ K, const uint32_t* __restrict__ V,
                             const int64_t* __restrict__ plen, uint32_t n, const uint64_t* __restrict__ tmax,
                             uint32_t* __restrict__ flag) {
    // one wave per tile of kEoTile: sequential max over 16 chunks of 64 (wave shuffles)
    const uint32_t t = blockIdx.x, lane = threadIdx.x;
    uint64_t run = tmax[t];
    for (uint32_t c = 0; c < kEoTile / 64; ++c) {
        const uint32_t i = t * kEoTile + c * 64 + lane;
        const uint64_t k = i < n ? K[i] : 0;
        const uint64_t e = k ? k + (uint64_t)plen[V[i]] : 0;
        uint64_t x = e;   // inclusive max-scan over the wave
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if ((int)lane >= d) x = max(x, y);
        }
        uint64_t before = __shfl_up(x, 1);
        if (lane == 0) before = 0;
        before = max(before, run);
        if (i < n) flag[i] = (k != 0 && k >= before) ? 1u : 0u;
        run = max(run, __shfl(x, 63));
    }
    if (t == gridDim.x - 1 && lane == 0) flag[n] = 0;
}

__global__ void cluster_starts_kernel(const uint32_t* __restrict__ flag_scan, uint32_t n,
                                      uint32_t* __restrict__ cstart, uint32_t C) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flag_scan[i + 1] != flag_scan[i]) cstart[flag_scan[i]] = i;
    if (i == n) cstart[C] = n;
}

__global__ void cluster_bound_kernel(const uint32_t* __restrict__ cstart, uint32_t C,
                                     unsigned long long* __restrict__ cap) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t k = cstart[c + 1] - cstart[c];
    if (k >= 2) atomicAdd(cap, (unsigned long long)(k * (k - 1) / 2));
}

__device__ __forceinline__ int mult_of(const int64_t* s, int G) {
    int m = 0;
    for (int g = 0; g < G; ++g) m += s[g] != 0;
    return m;
}
__device__ __forceinline__ void crop_start(int64_t* len, int64_t* s, int G, int64_t a) {   // UngappedLocalAlignment.h:138
    *len -= a;
    for (int g = 0; g < G; ++g)
        if (s[g] > 0) s[g] += a;
}
__device__ __forceinline__ void crop_end(int64_t* len, int64_t* s, int G, int64_t a) {     // :147
    *len -= a;
    for (int g = 0; g < G; ++g)
        if (s[g] < 0) s[g] -= a;
}

// the reference's matchI / nextI loops (Aligner.cpp:81-160) over one cluster
__global__ void cluster_sim_kernel(uint32_t* V, int64_t* plen, int64_t* ps, int G, int seqI,
                                   const uint32_t* __restrict__ cstart, uint32_t C, uint64_t pool_n,
                                   unsigned long long* __restrict__ nnew, uint64_t* __restrict__ nm_key,
                                   uint32_t* __restrict__ nm_id, unsigned long long* __restrict__ ndel,
                                   unsigned long long* __restrict__ nkeep) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int64_t a = cstart[c], b = cstart[c + 1];
    if (b - a < 2) return;
    uint32_t local = 0;
    unsigned long long dels = 0, keeps = 0;
    for (int64_t mi = a; mi < b; mi++) {
        if (V[mi] == kDel) continue;
        for (int64_t nj = mi + 1; nj < b; nj++) {
            if (V[nj] == kDel) continue;
            bool deleted_i = false;
            const uint64_t I = V[mi], J = V[nj];
            int64_t* sI = ps + I * G;
            int64_t* sJ = ps + J * G;
            const int64_t startI = sI[seqI], lenI = plen[I], startJ = sJ[seqI];
            int64_t diff = (startJ < 0 ? -startJ : startJ) - (startI < 0 ? -startI : startI) - lenI;
            if (diff >= 0) break;   // there are no more overlaps
            diff = -diff;
            const int mJ = mult_of(sJ, G), mI = mult_of(sI, G);
            const bool i_smaller = mJ > mI || (mJ == mI && plen[J] > plen[I]);
            const uint64_t src = i_smaller ? I : J;
            const unsigned long long q = atomicAdd(nnew, 1ull);
            const uint64_t nm = pool_n + q;
            int64_t* sN = ps + nm * G;
            int64_t lenN = plen[src];
            for (int g = 0; g < G; ++g) sN[g] = ps[src * G + g];
            if (i_smaller) {
                if (diff >= lenI) {
                    V[mi] = kDel;
                    deleted_i = true;
                    ++dels;
                } else if (startI > 0) {
                    crop_end(&plen[I], sI, G, diff);
                    crop_start(&lenN, sN, G, lenN - diff);
                } else {
                    crop_start(&plen[I], sI, G, diff);
                    crop_end(&lenN, sN, G, lenN - diff);
                }
            } else {
                if (diff >= plen[J]) {
                    V[nj] = kDel;
                    ++dels;
                } else if (startJ > 0) {
                    crop_start(&plen[J], sJ, G, diff);
                    crop_end(&lenN, sN, G, lenN - diff);
                } else {
                    crop_end(&plen[J], sJ, G, diff);
                    crop_start(&lenN, sN, G, lenN - diff);
                }
            }
            sN[seqI] = 0;   // new_match->SetStart( seqI, 0 )
            plen[nm] = lenN;
            const bool keep = mult_of(sN, G) > 1 && lenN > 0;
            nm_key[q] = keep ? (((uint64_t)c << 32) | local) : ~0ull;   // dropped copies sort last
            keeps += keep ? 1 : 0;
            nm_id[q] = (uint32_t)nm;
            ++local;
            if (deleted_i) break;   // (matchI-- then ++ in the reference: the same index, now NULL)
        }
    }
    if (dels) atomicAdd(ndel, dels);
    if (keeps) atomicAdd(nkeep, keeps);
}

__global__ void keep_kernel(const uint32_t* __restrict__ V, uint32_t n, uint32_t* __restrict__ keep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) keep[i] = (i < n && V[i] != kDel) ? 1u : 0u;
}

__global__ void compact_ids_kernel(const uint32_t* __restrict__ V, const uint32_t* __restrict__ keep, uint32_t n,
                                   uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && keep[i + 1] != keep[i]) out[keep[i]] = V[i];
}

__global__ void init_pool_kernel(const uint64_t* __restrict__ len, const int64_t* __restrict__ s, uint64_t M, int G,
                                 int64_t* __restrict__ plen, int64_t* __restrict__ ps, uint32_t* __restrict__ V) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    plen[i] = (int64_t)len[i];
    for (int g = 0; g < G; ++g) ps[i * G + g] = s[i * G + g];
    V[i] = (uint32_t)i;
}

__global__ void gather_out_kernel(const uint32_t* __restrict__ V, uint32_t n, int G, const int64_t* __restrict__ plen,
                                  const int64_t* __restrict__ ps, uint64_t* __restrict__ len, int64_t* __restrict__ s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t id = V[i];
    len[i] = (uint64_t)plen[id];
    for (int g = 0; g < G; ++g) s[i * G + g] = ps[id * G + g];
}

#define EOCHK(x)                              \
    do {                                      \
        hipError_t e_ = (x);                  \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

}  // namespace

// ---- host side -----------------------------------------------------------------------
EoWork::~EoWork() { release(); }

void EoWork::release() {
    for (void** p : {&K, &V, &V2, &fl, &fr, &Lpos, &Rpos, &bound, &segA, &segB, &act, &heap, &piv, &nsw, &scratch,
                     &plen, &ps, &nm_key, &nm_id, &nk2, &nv2, &nk3, &nv3, &radix, &ctr}) {   // NOLINT
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    cap_n = cap_pool = cap_new = pool_n = 0;
}

static hipError_t grow(void** p, size_t bytes) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    return hipMalloc(p, bytes ? bytes : 16);
}

// libstdc++ std::sort of (K, V)[0, n) by K (SortSeg levels; one host sync per level)
static hipError_t std_sort_device(EoWork& w, uint32_t n, int depth_override, hipStream_t st) {
    uint64_t* K = (uint64_t*)w.K;
    uint32_t* V = (uint32_t*)w.V;
    uint8_t* bound = (uint8_t*)w.bound;
    uint32_t* hc = (uint32_t*)w.hbuf;
    EOCHK(hipMemsetAsync(bound, 0, (size_t)n + 1, st));
    EOCHK(hipMemsetAsync(w.ctr, 0, 64, st));
    uint32_t* d_nheap = (uint32_t*)w.ctr;
    uint32_t S = 0;
    if (n > kLeaf) {
        const uint32_t lg = 31 - __builtin_clz(n);
        SortSeg top{0, n, depth_override >= 0 ? (uint32_t)depth_override : 2 * lg, 0};
        if (top.d == 0) {   // heap sort of everything
            EOCHK(hipMemcpyAsync(w.heap, &top, sizeof(top), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(heap_kernel, dim3(1), dim3(64), 0, st, K, V, (const SortSeg*)w.heap, 1u);
            EOCHK(hipGetLastError());
        } else {
            EOCHK(hipMemcpyAsync(w.segA, &top, sizeof(top), hipMemcpyHostToDevice, st));
            S = 1;
        }
    }
    uint8_t one = 1;
    EOCHK(hipMemcpyAsync(bound, &one, 1, hipMemcpyHostToDevice, st));
    EOCHK(hipMemcpyAsync(bound + n, &one, 1, hipMemcpyHostToDevice, st));
    uint32_t* fl = (uint32_t*)w.fl;
    uint32_t* fr = (uint32_t*)w.fr;
    SortSeg* segA = (SortSeg*)w.segA;
    SortSeg* segB = (SortSeg*)w.segB;
    uint32_t* act = (uint32_t*)w.act;
    uint32_t* nsw = (uint32_t*)w.nsw;
    uint32_t* d_nact = (uint32_t*)w.ctr + 4;
    while (S > 0) {
        hipLaunchKernelGGL(median_kernel, dim3(grid_of(S)), dim3(kBlock), 0, st, K, V, segA, S, (uint64_t*)w.piv);
        hipLaunchKernelGGL(classify_kernel, dim3(grid_of((uint64_t)n + 1)), dim3(kBlock), 0, st, K, segA, S,
                           (const uint64_t*)w.piv, n, fl, fr);
        EOCHK(hipGetLastError());
        EOCHK(exclusive_scan_u32(fl, (uint64_t)n + 1, w.scratch, nullptr, st));
        EOCHK(exclusive_scan_u32(fr, (uint64_t)n + 1, w.scratch, nullptr, st));
        hipLaunchKernelGGL(rank_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, segA, S, n, fl, fr, (uint32_t*)w.Lpos,
                           (uint32_t*)w.Rpos);
        EOCHK(hipMemsetAsync(nsw, 0, (size_t)S * 4, st));
        hipLaunchKernelGGL(swap_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, K, V, segA, S, n, fl, fr, (const uint32_t*)w.Lpos,
                           (const uint32_t*)w.Rpos, nsw);
        hipLaunchKernelGGL(cut_kernel, dim3(grid_of(S)), dim3(kBlock), 0, st, segA, S, fl, (const uint32_t*)w.Lpos,
                           (const uint32_t*)w.Rpos, nsw, segB, act, (SortSeg*)w.heap, d_nheap, bound);
        EOCHK(hipGetLastError());
        EOCHK(exclusive_scan_u32(act, 2ull * S + 1, w.scratch, d_nact, st));
        hipLaunchKernelGGL(compact_segs_kernel, dim3(grid_of(2ull * S)), dim3(kBlock), 0, st, segB, act, 2 * S, segA);
        EOCHK(hipGetLastError());
        EOCHK(hipMemcpyAsync(hc, d_nact, 4, hipMemcpyDeviceToHost, st));
        EOCHK(hipStreamSynchronize(st));
        S = hc[0];
    }
    EOCHK(hipMemcpyAsync(hc, d_nheap, 4, hipMemcpyDeviceToHost, st));
    EOCHK(hipStreamSynchronize(st));
    if (hc[0] > 0) {
        hipLaunchKernelGGL(heap_kernel, dim3(grid_of(hc[0])), dim3(kBlock), 0, st, K, V, (const SortSeg*)w.heap, hc[0]);
        EOCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(leaf_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, K, V, bound, n);
    return hipGetLastError();
}

// work arrays for n ids; the live ids in V survive a growth
static hipError_t ensure_n(EoWork& w, uint64_t n, hipStream_t st) {
    if (n + 2 <= w.cap_n) return hipSuccess;
    const uint64_t c = n + (n >> 2) + 1024;
    EOCHK(grow(&w.K, c * 8));
    void* nv = nullptr;
    EOCHK(hipMalloc(&nv, c * 4));
    if (w.V && w.cap_n) {
        EOCHK(hipMemcpyAsync(nv, w.V, w.cap_n * 4, hipMemcpyDeviceToDevice, st));
        EOCHK(hipStreamSynchronize(st));
    }
    if (w.V) (void)hipFree(w.V);
    w.V = nv;
    EOCHK(grow(&w.V2, c * 4));
    EOCHK(grow(&w.fl, c * 4));
    EOCHK(grow(&w.fr, c * 4));
    EOCHK(grow(&w.Lpos, c * 4));
    EOCHK(grow(&w.Rpos, c * 4));
    EOCHK(grow(&w.bound, c));
    EOCHK(grow(&w.segA, (c / (kLeaf + 1) + 2) * sizeof(SortSeg) * 2));
    EOCHK(grow(&w.segB, (c / (kLeaf + 1) + 2) * sizeof(SortSeg) * 2));
    EOCHK(grow(&w.act, (c / (kLeaf + 1) + 2) * 8 + 64));
    EOCHK(grow(&w.heap, (c / (kLeaf + 1) + 2) * sizeof(SortSeg)));
    EOCHK(grow(&w.piv, (c / (kLeaf + 1) + 2) * 8));
    EOCHK(grow(&w.nsw, (c / (kLeaf + 1) + 2) * 4));
    EOCHK(grow(&w.scratch, scan_tmp_bytes(2 * c + 2) + (c / kEoTile + 2) * 8 + 4096));
    if (!w.ctr) EOCHK(hipMalloc(&w.ctr, 256));
    w.cap_n = c;
    return hipSuccess;
}

hipError_t eo_sort_ids(EoWork& w, const uint64_t* d_keys, uint32_t n, int depth_override, uint32_t* d_ids_out,
                       hipStream_t st) {
    EOCHK(ensure_n(w, n, st));
    EOCHK(hipMemcpyAsync(w.K, d_keys, (size_t)n * 8, hipMemcpyDeviceToDevice, st));
    std::vector<uint32_t> iota(n);
    for (uint32_t i = 0; i < n; ++i) iota[i] = i;
    EOCHK(hipMemcpyAsync(w.V, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    EOCHK(std_sort_device(w, n, depth_override, st));
    EOCHK(hipMemcpyAsync(d_ids_out, w.V, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    return hipStreamSynchronize(st);
}

hipError_t eliminate_overlaps_device(EoWork& w, const uint64_t* d_len, const int64_t* d_s, uint64_t M, int G,
                                     uint64_t* M_out, hipStream_t st) {
    if (M >= 0xFFFFFFF0ull) return hipErrorInvalidValue;
    EOCHK(ensure_n(w, M, st));
    unsigned long long* hl = (unsigned long long*)w.hbuf;
    // pool: the M input matches, new ones appended pass by pass
    auto ensure_pool = [&](uint64_t need) -> hipError_t {
        if (need <= w.cap_pool) return hipSuccess;
        const uint64_t c = need + (need >> 1) + 1024;
        void *nl = nullptr, *ns = nullptr;
        EOCHK(hipMalloc(&nl, c * 8));
        EOCHK(hipMalloc(&ns, c * (uint64_t)G * 8));
        if (w.plen && w.pool_n) {
            EOCHK(hipMemcpyAsync(nl, w.plen, w.pool_n * 8, hipMemcpyDeviceToDevice, st));
            EOCHK(hipMemcpyAsync(ns, w.ps, w.pool_n * (uint64_t)G * 8, hipMemcpyDeviceToDevice, st));
            EOCHK(hipStreamSynchronize(st));
        }
        if (w.plen) (void)hipFree(w.plen);
        if (w.ps) (void)hipFree(w.ps);
        w.plen = nl;
        w.ps = ns;
        w.cap_pool = c;
        return hipSuccess;
    };
    w.pool_n = 0;
    EOCHK(ensure_pool(M + 1));
    if (M > 0)
        hipLaunchKernelGGL(init_pool_kernel, dim3(grid_of(M)), dim3(kBlock), 0, st, d_len, d_s, M, G,
                           (int64_t*)w.plen, (int64_t*)w.ps, (uint32_t*)w.V);
    EOCHK(hipGetLastError());
    w.pool_n = M;
    uint64_t n = M;
    if (M >= 2) {   // if( ml.size() < 2 ) return;
        for (int seqI = 0; seqI < G; ++seqI) {
            EOCHK(ensure_n(w, n, st));
            uint32_t* V = (uint32_t*)w.V;
            uint64_t* K = (uint64_t*)w.K;
            hipLaunchKernelGGL(keys_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, V, (const int64_t*)w.ps, G, seqI,
                               (uint32_t)n, K);
            EOCHK(hipGetLastError());
            EOCHK(std_sort_device(w, (uint32_t)n, -1, st));
            // clusters of the defined part
            const uint32_t T = (uint32_t)((n + kEoTile - 1) / kEoTile);
            uint64_t* tmax = (uint64_t*)((char*)w.scratch + scan_tmp_bytes(2 * w.cap_n + 2));
            uint32_t* flag = (uint32_t*)w.fl;
            hipLaunchKernelGGL(tile_max_kernel, dim3(T), dim3(kBlock), 0, st, K, V, (const int64_t*)w.plen,
                               (uint32_t)n, tmax);
            hipLaunchKernelGGL(tile_prefix_kernel, dim3(1), dim3(64), 0, st, tmax, T);
            hipLaunchKernelGGL(heads_kernel, dim3(T), dim3(64), 0, st, K, V, (const int64_t*)w.plen, (uint32_t)n,
                               (const uint64_t*)tmax, flag);
            EOCHK(hipGetLastError());
            uint32_t* d_C = (uint32_t*)w.ctr + 8;
            EOCHK(exclusive_scan_u32(flag, n + 1, w.scratch, d_C, st));
            unsigned long long* d_cap = (unsigned long long*)w.ctr + 8;   // bytes 64..
            unsigned long long* d_nnew = d_cap + 1;
            unsigned long long* d_ndel = d_cap + 2;
            unsigned long long* d_nkeep = d_cap + 3;
            EOCHK(hipMemsetAsync(d_cap, 0, 32, st));
            EOCHK(hipMemcpyAsync(hl, d_C, 4, hipMemcpyDeviceToHost, st));
            EOCHK(hipStreamSynchronize(st));
            const uint32_t C = (uint32_t)(hl[0] & 0xFFFFFFFFull);
            uint32_t* cstart = (uint32_t*)w.fr;
            hipLaunchKernelGGL(cluster_starts_kernel, dim3(grid_of(n + 1)), dim3(kBlock), 0, st, flag, (uint32_t)n,
                               cstart, C);
            if (C > 0)
                hipLaunchKernelGGL(cluster_bound_kernel, dim3(grid_of(C)), dim3(kBlock), 0, st, cstart, C, d_cap);
            EOCHK(hipGetLastError());
            EOCHK(hipMemcpyAsync(hl, d_cap, 8, hipMemcpyDeviceToHost, st));
            EOCHK(hipStreamSynchronize(st));
            const uint64_t bound_new = hl[0];
            if (bound_new == 0) continue;   // no overlapping pair: nothing changes this pass
            EOCHK(ensure_pool(w.pool_n + bound_new + 1));
            if (bound_new + 2 > w.cap_new) {
                const uint64_t c = bound_new + (bound_new >> 1) + 1024;
                EOCHK(grow(&w.nm_key, c * 8));
                EOCHK(grow(&w.nm_id, c * 4));
                EOCHK(grow(&w.nk2, c * 8));
                EOCHK(grow(&w.nv2, c * 4));
                EOCHK(grow(&w.nk3, c * 8));
                EOCHK(grow(&w.nv3, c * 4));
                EOCHK(grow(&w.radix, radix_tmp_bytes(c)));
                w.cap_new = c;
            }
            hipLaunchKernelGGL(cluster_sim_kernel, dim3(grid_of(C)), dim3(kBlock), 0, st, V, (int64_t*)w.plen,
                               (int64_t*)w.ps, G, seqI, cstart, C, w.pool_n, d_nnew, (uint64_t*)w.nm_key,
                               (uint32_t*)w.nm_id, d_ndel, d_nkeep);
            EOCHK(hipGetLastError());
            EOCHK(hipMemcpyAsync(hl, d_nnew, 24, hipMemcpyDeviceToHost, st));
            EOCHK(hipStreamSynchronize(st));
            const uint64_t nnew_all = hl[0], ndel = hl[1], nkeep = hl[2];
            w.pool_n += nnew_all;
            uint64_t wn = n;
            if (ndel > 0) {
                uint32_t* keep = (uint32_t*)w.fl;
                hipLaunchKernelGGL(keep_kernel, dim3(grid_of(n + 1)), dim3(kBlock), 0, st, V, (uint32_t)n, keep);
                EOCHK(exclusive_scan_u32(keep, n + 1, w.scratch, nullptr, st));
                hipLaunchKernelGGL(compact_ids_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, V, keep, (uint32_t)n,
                                   (uint32_t*)w.V2);
                EOCHK(hipGetLastError());
                std::swap(w.V, w.V2);
                wn = n - ndel;
            }
            if (nkeep > 0) {   // new matches in (cluster, creation) order; dropped copies last
                int buf = 0;
                EOCHK(radix_sort<uint64_t>((const uint64_t*)w.nm_key, (const uint32_t*)w.nm_id, nnew_all, 64,
                                           (uint64_t*)w.nk2, (uint32_t*)w.nv2, (uint64_t*)w.nk3, (uint32_t*)w.nv3,
                                           w.radix, &buf, st));
                const uint64_t* sk = buf ? (const uint64_t*)w.nk3 : (const uint64_t*)w.nk2;
                const uint32_t* sv = buf ? (const uint32_t*)w.nv3 : (const uint32_t*)w.nv2;
                (void)sk;
                EOCHK(ensure_n(w, wn + nkeep, st));
                EOCHK(hipMemcpyAsync((uint32_t*)w.V + wn, sv, nkeep * 4, hipMemcpyDeviceToDevice, st));
            }
            n = wn + nkeep;
        }
    }
    *M_out = n;
    w.n_final = n;
    return hipStreamSynchronize(st);
}

hipError_t eo_gather(EoWork& w, int G, uint64_t* d_len_out, int64_t* d_s_out, hipStream_t st) {
    const uint64_t n = w.n_final;
    if (n > 0)
        hipLaunchKernelGGL(gather_out_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, (const uint32_t*)w.V,
                           (uint32_t)n, G, (const int64_t*)w.plen, (const int64_t*)w.ps, d_len_out, d_s_out);
    EOCHK(hipGetLastError());
    return hipStreamSynchronize(st);
}

}  // namespace mums
