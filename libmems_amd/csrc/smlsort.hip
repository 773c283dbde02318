// smlsort.hip -- the order of equal seed mers in every SortedMerList.
//
// MemorySML::Create (libMems/MemorySML.cpp:45-60) fills {position, mer} in position order
// (FillDnaSeedSML, SortedMerList.cpp:771-783) and std::sorts it with bmer_lessthan, which
// compares the mer only (SortedMerList.h:311-314).  Equal mers therefore stay in the order
// libstdc++'s introsort leaves them, and that order is observable:
//   * MER_REPEAT_LIMIT restarts, FindMatchesFromPosition start points and ParallelMemHash
//     chunk starts are SML indices (GetBreakpoint's FindMer + 1, MatchFinder.cpp:113-121):
//     a start inside a run of equal mers decides which copies are searched;
//   * repeat / enumeration tolerance hash the first copies of a genome in SML order
//     (MemHash.cpp:139-162, the odometer MatchFinder.cpp:342-393);
//   * the SML itself (DNAFileSML positions, mums_build_sml).
// The seed stage sorts stably (ties by position).  This file replays the introsort on
// the device, level-parallel, for the runs of equal mers that matter, and yields the
// std::sort order of those runs:
//   * slot space = the genome-major SML slots [base_g, base_g + m_g) (= global seed-mer
//     indices); K / V = keys / seed-mer ids at the slots, initially in position order;
//   * every level runs __move_median_to_first on each active segment and computes its
//     __unguarded_partition in closed form over the segment's elements only (the k-th
//     left stopper, key >= pivot, swaps with the k-th right stopper, key <= pivot from the
//     right, while it lies left of it; the cut is the (K+1)-th left stopper or the K-th
//     right stopper, whichever comes first);
//   * the runs that matter are flagged (pairs of equal sorted keys: all of them, or the
//     runs a start point falls into); a segment [f, l) holds exactly the keys sorted[f, l)
//     (quicksort invariant), so it is partitioned further iff [f, l) holds a slot of a
//     flagged run (a prefix count over the slot flags), and every other segment is
//     dropped -- restarts touch a few runs, so that work is quickselect-like, not n log n;
//   * depth-0 segments run __partial_sort's heap sort on one lane; leaves (<= 16) the
//     final insertion sort (it never moves an element across a partition boundary).
// The oracle restates std::sort in oracle/std_sort.h, pinned to the real std::sort.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mums_internal.h"

namespace mums {

namespace {

constexpr uint32_t kLeaf = 16;   // _S_threshold

struct TieSeg {
    uint32_t f, l, d, pad;
};

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

inline char* align_up(char* p) { return (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255); }

__device__ __forceinline__ void swap_kv(uint64_t* K, uint32_t* V, uint32_t a, uint32_t b) {
    const uint64_t k = K[a];
    K[a] = K[b];
    K[b] = k;
    const uint32_t v = V[a];
    V[a] = V[b];
    V[b] = v;
}

// genome of slot t (dbase: G + 1 slot bases)
__device__ __forceinline__ int slot_genome(const uint64_t* __restrict__ dbase, int G, uint64_t t) {
    int g = 0;
    for (int k = 1; k < G; ++k) g += (t >= dbase[k]) ? 1 : 0;
    return g;
}

// pf[t] = 1 when sorted slots t and t + 1 hold equal keys of one genome
__global__ void mark_all_kernel(const uint64_t* __restrict__ ck, uint64_t n, const uint64_t* __restrict__ dbase,
                                const uint64_t* __restrict__ dm, int G, uint32_t* __restrict__ pf) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n) return;
    uint32_t f = 0;
    if (t + 1 < n && ck[t] == ck[t + 1]) {
        const int g = slot_genome(dbase, G, t);
        f = t + 1 < dbase[g] + dm[g] ? 1u : 0u;
    }
    pf[t] = f;
}

// start points sp[r * G + g] (SML indices of genome g): when slots s - 1 and s hold equal
// keys, every pair of that run is flagged
__global__ void mark_starts_kernel(const uint64_t* __restrict__ ck, const uint64_t* __restrict__ dbase,
                                   const uint64_t* __restrict__ dm, int G, const uint64_t* __restrict__ sp,
                                   uint64_t rows, uint32_t* __restrict__ pf) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * (uint64_t)G) return;
    const int g = (int)(i % (uint64_t)G);
    const uint64_t s = sp[i], m = dm[g];
    if (s == 0 || s >= m) return;
    const uint64_t* a = ck + dbase[g];
    const uint64_t k = a[s];
    if (a[s - 1] != k) return;
    uint64_t lo = s - 1, hi = s + 1;
    while (lo > 0 && a[lo - 1] == k) --lo;
    while (hi < m && a[hi] == k) ++hi;
    for (uint64_t t = lo; t + 1 < hi; ++t) pf[dbase[g] + t] = 1u;
}

__global__ void iota_kernel(uint32_t* __restrict__ V, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) V[t] = (uint32_t)t;
}

// slot flags: sf[t] = slot t lies in a flagged run (pair t - 1 or pair t flagged)
__global__ void slot_flags_kernel(const uint32_t* __restrict__ pf, uint64_t n, uint32_t* __restrict__ sf) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n) return;
    sf[t] = t < n ? ((pf[t] | (t > 0 ? pf[t - 1] : 0u)) != 0u ? 1u : 0u) : 0u;
}

// a segment [f, l) holds a slot of a flagged run (ts = exclusive scan of the slot flags);
// a dropped segment holds none, so every flagged slot ends in a fully sorted segment
__device__ __forceinline__ bool seg_wanted(const uint32_t* __restrict__ ts, uint32_t f, uint32_t l) {
    return ts[l] != ts[f];
}

// top segments: one per genome (depth 2 * __lg(m)), kept when they hold a flagged slot;
// genome bounds marked for the leaf pass
__global__ void top_kernel(const uint64_t* __restrict__ dbase, const uint64_t* __restrict__ dm, int G,
                           const uint32_t* __restrict__ ts, TieSeg* __restrict__ out, uint32_t* __restrict__ act,
                           TieSeg* __restrict__ heap, uint32_t* __restrict__ nheap, uint8_t* __restrict__ bound) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) act[G] = 0;
    if (g >= G) return;
    const uint32_t f = (uint32_t)dbase[g], l = (uint32_t)(dbase[g] + dm[g]);
    bound[f] = 1;
    bound[l] = 1;
    const uint64_t m = dm[g];
    const bool big = m > kLeaf && seg_wanted(ts, f, l);
    const uint32_t d = m > 0 ? 2u * (63u - (uint32_t)__builtin_clzll(m)) : 0u;
    out[g] = TieSeg{f, l, d, 0};
    act[g] = (big && d > 0) ? 1u : 0u;
    if (big && d == 0) heap[atomicAdd(nheap, 1u)] = out[g];
}

__global__ void compact_segs_kernel(const TieSeg* __restrict__ in, const uint32_t* __restrict__ act, uint32_t n2,
                                    TieSeg* __restrict__ out, uint32_t* __restrict__ sz) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n2 && act[i + 1] != act[i]) {
        const TieSeg g = in[i];
        out[act[i]] = g;
        sz[act[i]] = g.l - g.f - 1;   // partition range [f + 1, l)
    }
}

// __move_median_to_first(first, first + 1, mid, last - 1); piv[s] = the pivot key
__global__ void median_kernel(uint64_t* K, uint32_t* V, const TieSeg* __restrict__ segs, uint32_t S,
                              uint64_t* __restrict__ piv) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const TieSeg g = segs[s];
    const uint32_t a = g.f + 1, b = g.f + (g.l - g.f) / 2, c = g.l - 1;
    const uint64_t ka = K[a], kb = K[b], kc = K[c];
    uint32_t m;
    if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
    else m = ka < kc ? a : (kb < kc ? c : b);
    swap_kv(K, V, g.f, m);
    piv[s] = K[g.f];
}

// segment of compacted element t: last s with off[s] <= t
__device__ __forceinline__ uint32_t seg_of(const uint32_t* __restrict__ off, uint32_t S, uint32_t t) {
    uint32_t lo = 0, n = S;
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (off[lo + h] <= t) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo - 1;
}

// stopper flags of the partition ranges: fl = key >= pivot, fr = key <= pivot
__global__ void classify_kernel(const uint64_t* __restrict__ K, const TieSeg* __restrict__ segs,
                                const uint32_t* __restrict__ off, uint32_t S, const uint64_t* __restrict__ piv,
                                uint32_t A, uint32_t* __restrict__ fl, uint32_t* __restrict__ fr) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > A) return;
    uint32_t a = 0, b = 0;
    if (t < A) {
        const uint32_t s = seg_of(off, S, t);
        const uint32_t i = segs[s].f + 1 + (t - off[s]);
        const uint64_t p = piv[s], k = K[i];
        a = !(k < p);
        b = !(p < k);
    }
    fl[t] = a;
    fr[t] = b;
}

// after the exclusive scans: Lpos[off + k] = k-th left stopper (from the left),
// Rpos[off + k] = k-th right stopper (from the right)
__global__ void rank_kernel(const TieSeg* __restrict__ segs, const uint32_t* __restrict__ off, uint32_t S, uint32_t A,
                            const uint32_t* __restrict__ fl, const uint32_t* __restrict__ fr,
                            uint32_t* __restrict__ Lpos, uint32_t* __restrict__ Rpos) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A) return;
    const uint32_t s = seg_of(off, S, t);
    const uint32_t b = off[s], e = off[s + 1];
    const uint32_t i = segs[s].f + 1 + (t - b);
    if (fl[t + 1] != fl[t]) Lpos[b + (fl[t] - fl[b])] = i;
    if (fr[t + 1] != fr[t]) Rpos[b + (fr[e] - fr[t + 1])] = i;
}

// pair k swaps iff L_k < R_k (a prefix of k); nswap[s] = K
__global__ void swap_kernel(uint64_t* K, uint32_t* V, const TieSeg* __restrict__ segs,
                            const uint32_t* __restrict__ off, uint32_t S, uint32_t A, const uint32_t* __restrict__ fl,
                            const uint32_t* __restrict__ fr, const uint32_t* __restrict__ Lpos,
                            const uint32_t* __restrict__ Rpos, uint32_t* __restrict__ nswap) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A || fl[t + 1] == fl[t]) return;
    const uint32_t s = seg_of(off, S, t);
    const uint32_t b = off[s], e = off[s + 1];
    const uint32_t i = segs[s].f + 1 + (t - b);
    const uint32_t k = fl[t] - fl[b];
    const uint32_t cntR = fr[e] - fr[b];
    if (k >= cntR) return;
    const uint32_t j = Rpos[b + k];
    if (!(i < j)) return;
    swap_kv(K, V, i, j);
    // the swapping pairs are a prefix (L_k rises, R_k falls): its last pair writes the count.
    // (One atomic per swap on the segment's counter serialised 1.5e9 swaps of a 3 Gbp SML:
    // 28 s per restart at BASELINE config 5.)
    const uint32_t cntL = fl[e] - fl[b];
    if (k + 1 >= cntL || k + 1 >= cntR || !(Lpos[b + k + 1] < Rpos[b + k + 1])) nswap[s] = k + 1;
}

// cut = min(L_{K+1}, R_K) (R_0 = l); children [f, cut), [cut, l) at depth d - 1 into
// out[2s], out[2s + 1], kept (act = 1) when they partition again and hold a flagged slot;
// depth-0 children > 16 go to the heap list
__global__ void cut_kernel(const TieSeg* __restrict__ segs, const uint32_t* __restrict__ off, uint32_t S,
                           const uint32_t* __restrict__ fl, const uint32_t* __restrict__ Lpos,
                           const uint32_t* __restrict__ Rpos, const uint32_t* __restrict__ nswap,
                           const uint32_t* __restrict__ ts, TieSeg* __restrict__ out, uint32_t* __restrict__ act,
                           TieSeg* __restrict__ heap, uint32_t* __restrict__ nheap, uint8_t* __restrict__ bound) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0) act[2 * S] = 0;
    if (s >= S) return;
    const TieSeg g = segs[s];
    const uint32_t b = off[s], e = off[s + 1];
    const uint32_t K = nswap[s];
    const uint32_t cntL = fl[e] - fl[b];
    uint32_t cut = K > 0 ? Rpos[b + K - 1] : g.l;
    if (K < cntL) cut = min(cut, Lpos[b + K]);
    bound[cut] = 1;
    const uint32_t d = g.d - 1;
    const TieSeg ch[2] = {TieSeg{g.f, cut, d, 0}, TieSeg{cut, g.l, d, 0}};
    for (int c = 0; c < 2; ++c) {
        const bool big = ch[c].l - ch[c].f > kLeaf && seg_wanted(ts, ch[c].f, ch[c].l);
        out[2 * s + c] = ch[c];
        act[2 * s + c] = (big && d > 0) ? 1u : 0u;
        if (big && d == 0) heap[atomicAdd(nheap, 1u)] = ch[c];
    }
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

__global__ void heap_kernel(uint64_t* K, uint32_t* V, const TieSeg* __restrict__ segs, uint32_t S) {
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

// insertion sort of every leaf (<= 16 slots between two bounds) that holds a flagged slot
__global__ void leaf_kernel(uint64_t* K, uint32_t* V, const uint8_t* __restrict__ bound,
                            const uint32_t* __restrict__ ts, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !bound[i]) return;
    uint32_t e = i + 1;
    while (e <= n && e - i <= kLeaf && !bound[e]) ++e;
    if (e - i > kLeaf || e > n || !seg_wanted(ts, i, e)) return;   // heap-sorted / dropped segments
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

// slot t lies in a flagged run
__device__ __forceinline__ bool slot_flagged(const uint32_t* __restrict__ ts, uint64_t t) {
    return ts[t + 1] != ts[t];
}

// stream record j (SML slot inv[j]) of a flagged run takes the id at its slot
__global__ void writeback_kernel(uint64_t* rec, uint32_t* idx, const uint32_t* __restrict__ inv,
                                 const uint32_t* __restrict__ ts, const uint32_t* __restrict__ V, uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t t = inv[j];
    if (!slot_flagged(ts, t)) return;
    if (rec) rec[j] = (rec[j] & 0xFFFFFFFF00000000ull) | V[t];
    else idx[j] = V[t];
}

__global__ void scatter_keys_kernel(const uint64_t* __restrict__ ckf, const uint32_t* __restrict__ inv_unused,
                                    const uint64_t* __restrict__ rec, const uint32_t* __restrict__ idx, uint64_t n,
                                    uint64_t* __restrict__ K) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    (void)inv_unused;
    const uint64_t gi = rec ? (rec[j] & 0xFFFFFFFFull) : idx[j];
    K[gi] = ckf[j];
}

__global__ void slots_out_kernel(const uint32_t* __restrict__ ts, const uint32_t* __restrict__ V, uint64_t n,
                                 uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n && slot_flagged(ts, t)) out[t] = V[t];
}

}  // namespace

TieWs tie_ws_layout(void* base, uint64_t n, int G) {
    TieWs w{};
    char* p = align_up((char*)base);
    auto take = [&](size_t bytes) {
        char* r = p;
        p = align_up(p + bytes);
        return (void*)r;
    };
    const uint64_t n1 = n + 64;
    const uint64_t smax = n / (kLeaf + 1) + (uint64_t)G + 64;   // active segments hold > 16 slots
    w.n = n;
    w.G = G;
    w.smax = smax;
    w.ts = (uint32_t*)take(n1 * 4);
    w.K = (uint64_t*)take(n1 * 8);
    w.V = (uint32_t*)take(n1 * 4);
    w.fl = (uint32_t*)take(n1 * 4);
    w.pf = w.fl;   // the pair flags are dead once tie_prepare has scanned them into ts
    w.fr = (uint32_t*)take(n1 * 4);
    w.Lpos = (uint32_t*)take(n1 * 4);
    w.Rpos = (uint32_t*)take(n1 * 4);
    w.bound = (uint8_t*)take(n1);
    w.segA = take(2 * smax * 16);
    w.segB = take(2 * smax * 16);
    w.heap = take(2 * smax * 16);
    w.act = (uint32_t*)take((2 * smax + 64) * 4);
    w.off = (uint32_t*)take((2 * smax + 64) * 4);
    w.piv = (uint64_t*)take(smax * 8);
    w.nsw = (uint32_t*)take(smax * 4);
    w.ctr = (uint32_t*)take(256);
    w.dbase = (uint64_t*)take((size_t)(G + 1) * 8);
    w.dm = (uint64_t*)take((size_t)(G + 1) * 8);
    w.tmp = take(scan_tmp_bytes(std::max<uint64_t>(n + 1, 4 * smax + 1)));
    w.bytes = (size_t)(p - (char*)base);
    return w;
}

size_t tie_ws_bytes(uint64_t n, int G) { return tie_ws_layout(nullptr, n, G).bytes + 256; }

hipError_t tie_set_genomes(const TieWs& w, const uint64_t* base, const uint64_t* m, hipStream_t st) {
    std::vector<uint64_t> hb(w.G + 1, 0), hm(w.G + 1, 0);
    for (int g = 0; g < w.G; ++g) {
        hb[g] = base[g];
        hm[g] = m[g];
    }
    hb[w.G] = w.n;
    hipError_t e = hipMemcpyAsync(w.dbase, hb.data(), hb.size() * 8, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(w.dm, hm.data(), hm.size() * 8, hipMemcpyHostToDevice, st);
}

hipError_t tie_clear_flags(const TieWs& w, hipStream_t st) { return hipMemsetAsync(w.pf, 0, (w.n + 1) * 4, st); }

hipError_t tie_mark_all(const TieWs& w, const uint64_t* ck, hipStream_t st) {
    hipLaunchKernelGGL(mark_all_kernel, dim3(grid_of(w.n + 1)), dim3(kBlock), 0, st, ck, w.n, w.dbase, w.dm, w.G, w.pf);
    return hipGetLastError();
}

hipError_t tie_mark_starts(const TieWs& w, const uint64_t* ck, const uint64_t* d_sp, uint64_t rows, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(mark_starts_kernel, dim3(grid_of(rows * (uint64_t)w.G)), dim3(kBlock), 0, st, ck, w.dbase,
                       w.dm, w.G, d_sp, rows, w.pf);
    return hipGetLastError();
}

hipError_t tie_scatter_keys(const TieWs& w, const uint64_t* ckf, const uint64_t* rec, const uint32_t* idx,
                            hipStream_t st) {
    if (w.n == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_keys_kernel, dim3(grid_of(w.n)), dim3(kBlock), 0, st, ckf, nullptr, rec, idx, w.n, w.K);
    return hipGetLastError();
}

// slot flags of the flagged runs, scanned; *flagged = flagged slots (0: nothing to replay)
hipError_t tie_prepare(const TieWs& w, uint64_t* flagged, hipStream_t st) {
    const uint64_t n = w.n;
    *flagged = 0;
    if (n == 0) return hipSuccess;
    uint32_t hc = 0;
    hipLaunchKernelGGL(slot_flags_kernel, dim3(grid_of(n + 1)), dim3(kBlock), 0, st, w.pf, n, w.ts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = exclusive_scan_u32(w.ts, n + 1, w.tmp, w.ctr, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&hc, w.ctr, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    *flagged = hc;
    return hipSuccess;
}

// libstdc++ std::sort of every genome's slots (K) by key, restricted to the segments that
// hold a flagged slot (after tie_prepare); V = the ids in std::sort order at the flagged
// slots.
hipError_t tie_replay(const TieWs& w, hipStream_t st) {
    const uint64_t n = w.n;
    if (n == 0) return hipSuccess;
    uint32_t* ctr = w.ctr;
    uint32_t* d_nheap = ctr + 1;
    uint32_t* d_nact = ctr + 2;
    uint32_t* d_A = ctr + 3;
    uint32_t hc[4] = {0, 0, 0, 0};
    hipError_t e;
    if ((e = hipMemsetAsync(ctr, 0, 64, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.bound, 0, n + 1, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(iota_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, w.V, n);
    TieSeg* segA = (TieSeg*)w.segA;
    TieSeg* segB = (TieSeg*)w.segB;
    TieSeg* heap = (TieSeg*)w.heap;
    hipLaunchKernelGGL(top_kernel, dim3(grid_of(w.G)), dim3(kBlock), 0, st, w.dbase, w.dm, w.G, w.ts, segB, w.act,
                       heap, d_nheap, w.bound);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t n2 = (uint32_t)w.G;
    const bool dbg = getenv("MUMS_DEV_RESTART_TIMING") != nullptr;   // development: levels and sizes
    int level = 0;
    uint64_t a_sum = 0;
    for (;;) {
        // compact the kept children of the last level into segA, their partition sizes into off
        if ((e = exclusive_scan_u32(w.act, (uint64_t)n2 + 1, w.tmp, d_nact, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(compact_segs_kernel, dim3(grid_of(n2)), dim3(kBlock), 0, st, segB, w.act, n2, segA, w.off);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(hc, d_nact, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        const uint32_t S = hc[0];
        if (S == 0) break;
        if (S > w.smax) return hipErrorInvalidValue;
        if ((e = hipMemsetAsync(w.off + S, 0, 4, st)) != hipSuccess) return e;
        if ((e = exclusive_scan_u32(w.off, (uint64_t)S + 1, w.tmp, d_A, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(hc + 1, d_A, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(median_kernel, dim3(grid_of(S)), dim3(kBlock), 0, st, w.K, w.V, segA, S, w.piv);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        const uint32_t A = hc[1];
        a_sum += A;
        if (dbg && (level < 8 || (level % 8) == 0)) fprintf(stderr, "tie replay level %d: %u segments, %u elements\n", level, S, A);
        ++level;
        hipLaunchKernelGGL(classify_kernel, dim3(grid_of((uint64_t)A + 1)), dim3(kBlock), 0, st, w.K, segA, w.off, S,
                           w.piv, A, w.fl, w.fr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = exclusive_scan_u32(w.fl, (uint64_t)A + 1, w.tmp, nullptr, st)) != hipSuccess) return e;
        if ((e = exclusive_scan_u32(w.fr, (uint64_t)A + 1, w.tmp, nullptr, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(rank_kernel, dim3(grid_of(A)), dim3(kBlock), 0, st, segA, w.off, S, A, w.fl, w.fr, w.Lpos,
                           w.Rpos);
        if ((e = hipMemsetAsync(w.nsw, 0, (size_t)S * 4, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(swap_kernel, dim3(grid_of(A)), dim3(kBlock), 0, st, w.K, w.V, segA, w.off, S, A, w.fl, w.fr,
                           w.Lpos, w.Rpos, w.nsw);
        hipLaunchKernelGGL(cut_kernel, dim3(grid_of(S)), dim3(kBlock), 0, st, segA, w.off, S, w.fl, w.Lpos, w.Rpos,
                           w.nsw, w.ts, segB, w.act, heap, d_nheap, w.bound);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        n2 = 2 * S;
    }
    if ((e = hipMemcpyAsync(hc + 2, d_nheap, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (dbg) fprintf(stderr, "tie replay: %d levels, %lu elements partitioned, %u heap segments\n", level,
                     (unsigned long)a_sum, hc[2]);
    if (hc[2] > 0) {
        hipLaunchKernelGGL(heap_kernel, dim3(grid_of(hc[2])), dim3(kBlock), 0, st, w.K, w.V, heap, hc[2]);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(leaf_kernel, dim3(grid_of(n)), dim3(kBlock), 0, st, w.K, w.V, w.bound, w.ts, (uint32_t)n);
    return hipGetLastError();
}

hipError_t tie_writeback(const TieWs& w, uint64_t* rec, uint32_t* idx, const uint32_t* inv, hipStream_t st) {
    if (w.n == 0) return hipSuccess;
    hipLaunchKernelGGL(writeback_kernel, dim3(grid_of(w.n)), dim3(kBlock), 0, st, rec, idx, inv, w.ts, w.V, w.n);
    return hipGetLastError();
}

hipError_t tie_slots_out(const TieWs& w, uint32_t* out, hipStream_t st) {
    if (w.n == 0) return hipSuccess;
    hipLaunchKernelGGL(slots_out_kernel, dim3(grid_of(w.n)), dim3(kBlock), 0, st, w.ts, w.V, w.n, out);
    return hipGetLastError();
}

}  // namespace mums
