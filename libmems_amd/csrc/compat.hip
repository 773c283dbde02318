// compat.hip -- ParallelMemHash chunk-compat mode.
//
// ParallelMemHash::FindMatches (ParallelMemHash.cpp:42-103) cuts the SMLs into chunks:
// chunk starts come from MatchFinder::GetBreakpoint (MatchFinder.cpp:89-126) every
// CHUNK_SIZE (200000) mers of the longest SML, each chunk is searched on its own
// (SearchRange, MatchFinder.cpp:172-340) and the thread tables are re-added into one
// table (MergeTable, :105-121).  A masked-key group whose records straddle a chunk
// boundary in some genome is therefore searched as several smaller groups.
//
// On the GPU the chunk becomes part of the sort key: every record gets
// key2 = (chunk << (2w+1)) | ckey, so one stable sort of (key2, index) yields the
// chunk-major probe order the reference's AddHashEntry calls follow, and the unchanged
// group / probe / chain / replay kernels run on it.  The MergeTable re-insertion is
// replayed per bucket at the end (compat_merge_kernel).
//
//   1. genome_keys_kernel     key' = genome << kbits | ckey; one stable sort of key'
//                             gives every genome's SortedMerList as a segment
//   2. compat_breaks_kernel   chunk starts on the longest SML (sequential walk)
//   3. compat_find_kernel     FindMer (bsearch) of each break mer in the other SMLs
//   4. compat_chunk_keys      chunk of every record -> key2
//   5. compat_cand / fire /   MER_REPEAT_LIMIT inside a chunk: SearchRange returns false and
//      drop kernels           ParallelMemHash.cpp:97 ignores it, so the rest of that chunk is
//                             never searched -- its records from the firing group on are dropped
//   6. compat_merge_kernel    MergeTable: re-add each bucket's entries in vector order
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "match_device.h"
#include "mums_internal.h"
#include "restart_plan.h"

namespace mums {
namespace {

// key' = genome << kbits | ckey (the genome's SML becomes a contiguous segment of the
// sorted key' order: positions ascending within equal ckey, MemorySML.cpp:45-60)
__global__ void genome_keys_kernel(uint64_t* __restrict__ ckey, uint64_t N, GenomeTable gt, int kbits) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    ckey[i] |= (uint64_t)genome_of(gt, i) << kbits;
}

// MatchFinder::GetBreakpoint on the longest SML mx, repeated as ParallelMemHash.cpp:75-83
// does: start = previous + chunk; walk back to the first index of the start's masked key.
// cs[k * G + g] = start of chunk k in SML g (row 0 pre-zeroed); bm[k] = break mer.
// Error bits: 4 = chunk cap exceeded (a masked-key group >= chunk: the reference loops
// forever), 8 = start past the SML end (operator[] out of range in the reference).
__global__ void compat_breaks_kernel(const uint64_t* __restrict__ sk, GenomeTable gt, uint64_t kmask, int mx,
                                     uint64_t chunk, uint64_t* __restrict__ cs, uint64_t* __restrict__ bm,
                                     uint32_t cap, uint32_t* __restrict__ d_nch, uint32_t* __restrict__ err) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const uint64_t* seg = sk + gt.base[mx];
    const uint64_t m = gt.m[mx], n = gt.n[mx];
    const int G = gt.G;
    uint32_t k = 1;
    uint64_t s = 0;
    while (s + chunk < n) {   // Length() = sequence length (SortedMerList.cpp:284-286)
        if (k >= cap) { atomicOr(err, 4u); break; }
        uint64_t i = s + chunk;
        if (i >= m) { atomicOr(err, 8u); break; }
        const uint64_t b = seg[i] & kmask;
        uint64_t prev = b;
        while ((prev >> 1) == (b >> 1)) {   // masked key = ckey without the parity bit
            if (i == 0) { i = ~0ull; break; }
            --i;
            prev = seg[i] & kmask;
        }
        ++i;
        cs[(uint64_t)k * G + mx] = i;
        bm[k] = b;
        s = i;
        ++k;
    }
    *d_nch = k;
}

// The other SMLs' chunk starts: SortedMerList::FindMer (SortedMerList.cpp:170-179) with
// the full break mer; bsearch (:380-394) returns the probed middle when absent.  The
// backward loop of GetBreakpoint (MatchFinder.cpp:114-121) compares with
// (break_mer.mer && mer_mask), a bool: it never runs unless the break mer is 0, where it
// runs down to -1.  So a found mer starts the chunk one past it (or at 0 for mer 0).
__global__ void compat_find_kernel(const uint64_t* __restrict__ sk, GenomeTable gt, uint64_t kmask, int mx, int L,
                                   uint64_t* __restrict__ cs, const uint64_t* __restrict__ bm, uint32_t nch) {
    const int G = gt.G;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)(nch - 1) * G) return;
    const uint32_t k = 1 + (uint32_t)(t / G);
    const int g = (int)(t % G);
    if (g == mx) return;
    const uint64_t q = bm[k];
    const uint64_t n = gt.n[g];
    uint64_t cur = 0;   // FindMer's early return leaves the caller's value (0 here)
    if (n != 0 && n >= (uint64_t)L) {
        const uint64_t* seg = sk + gt.base[g];
        uint64_t start = 0, end = n - (uint64_t)L;
        for (;;) {
            const uint64_t mid = (start + end) / 2;
            const uint64_t v = seg[mid] & kmask;
            cur = mid;
            if (v == q) break;
            if (v < q && mid < end) start = mid + 1;
            else if (v > q && start < mid) end = mid - 1;
            else break;
        }
        if ((seg[cur] & kmask) == q) cur = (q == 0) ? 0 : cur + 1;
    }
    cs[(uint64_t)k * G + g] = cur;
}

// chunk of SML index r of genome g = last k with cs[k][g] <= r (cs[0][g] = 0); ck (optional)
// keeps the genome-major SMLs' keys without the genome bits for the truncation plan
__global__ void compat_chunk_keys_kernel(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint64_t N,
                                         GenomeTable gt, int kbits, const uint64_t* __restrict__ cs, uint32_t nch,
                                         uint64_t* __restrict__ key2, uint32_t* __restrict__ val2,
                                         uint64_t* __restrict__ ck) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const uint64_t kmask = (kbits >= 64) ? ~0ull : ((1ull << kbits) - 1);
    const uint64_t x = sk[j];
    const int g = (int)(x >> kbits);
    const uint64_t r = j - gt.base[g];
    const int G = gt.G;
    uint32_t lo = 0, hi = nch - 1;   // invariant: cs[lo][g] <= r
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (cs[(uint64_t)mid * G + g] <= r) lo = mid;
        else hi = mid - 1;
    }
    key2[j] = ((uint64_t)lo << kbits) | (x & kmask);
    val2[j] = sv[j];
    if (ck) ck[j] = x & kmask;
}

// MER_REPEAT_LIMIT inside a chunk.  Candidates: (chunk, masked key) groups of more than
// 1000 records in the chunk-major stream -- the stream index of every such group's first
// record (key2 >> 1 = chunk, masked key).
__global__ void compat_cand_kernel(const uint64_t* __restrict__ key2, uint64_t N, uint64_t* __restrict__ list,
                                   unsigned long long* __restrict__ cnt, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const uint64_t v = key2[j] >> 1;
    if (j > 0 && (key2[j - 1] >> 1) == v) return;
    const uint64_t e = j + restart::kRepeatLimit;
    if (e >= N || (key2[e] >> 1) != v) return;
    const unsigned long long k = atomicAdd(cnt, 1ull);
    if (k < cap) list[k] = j;
}

// Per candidate: does SearchRange's check (MatchFinder.cpp:253) fire on this group inside its
// chunk?  The chunk's SearchRange (ParallelMemHash.cpp:97) reads genome g from
// S = cs[i][g] for search_len = cs[i+1][g] - cs[i][g] records (the last chunk: to the SML's
// end) in MER_BUFFER_SIZE buffers from S; the group is collected genome run by genome run
// in the head order of restart_plan.h, and the check precedes every collection step.
// out[c] = 1 when it fires; cend[c] = stream index of the chunk's end (first record of
// chunk i + 1); cons (optional, C x (G + 1)): the SML positions the chunk's merge consumed
// in every genome when the check fired, then the chunk i (LogProgress of a cut chunk).
__global__ void compat_fire_kernel(restart::PlanData d, const uint64_t* __restrict__ key2, uint64_t N, int kbits,
                                   const uint64_t* __restrict__ cand, uint64_t C, const uint64_t* __restrict__ cs,
                                   uint32_t nch, uint32_t* __restrict__ out, uint64_t* __restrict__ cend,
                                   uint64_t* __restrict__ cons) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int G = d.G;
    const uint64_t j = cand[c];
    const uint64_t x2 = key2[j];
    const uint32_t i = (uint32_t)(x2 >> kbits);
    const uint64_t K = (x2 & ((1ull << kbits) - 1)) >> 1;
    uint64_t S[restart::kMaxGenomes], a[restart::kMaxGenomes], b[restart::kMaxGenomes], E[restart::kMaxGenomes];
    uint64_t U = 0;
    for (int g = 0; g < G; ++g) {
        const uint64_t m = d.m[g];
        S[g] = cs[(uint64_t)i * G + g];
        E[g] = i + 1 < nch ? cs[(uint64_t)(i + 1) * G + g] : m;
        if (S[g] > m) S[g] = m;
        if (E[g] > m) E[g] = m;
        if (E[g] < S[g]) E[g] = S[g];
        const uint64_t lo = restart::lower_bound_g(d, g, 0, m, K << 1), hi = restart::lower_bound_g(d, g, 0, m, (K + 1) << 1);
        a[g] = lo < S[g] ? S[g] : (lo > E[g] ? E[g] : lo);
        b[g] = hi < S[g] ? S[g] : (hi > E[g] ? E[g] : hi);
        if (b[g] > a[g]) U |= 1ull << g;
    }
    int ord[restart::kMaxGenomes];
    uint64_t steps = 0;
    const int n = restart::head_order(d, U, a, S, ord, &steps);
    uint64_t cum = 0;
    bool fired = false;
    uint64_t cz[restart::kMaxGenomes];   // consumed: every key below K, then the collected runs
    for (int g = 0; g < G; ++g) cz[g] = a[g];
    for (int k = 0; k < n && !fired; ++k) {
        const int g = ord[k];
        uint64_t x = a[g];
        while (x < b[g]) {
            if (cum > restart::kRepeatLimit) { fired = true; break; }
            const uint64_t nb = S[g] + ((x - S[g]) / restart::kMerBuffer + 1) * restart::kMerBuffer;
            const uint64_t y = b[g] < nb ? b[g] : nb;
            cum += y - x;
            x = y;
            cz[g] = x;
        }
        // a run ending on a buffer boundary with more of the chunk to read: the refilled
        // head still carries K for one more iteration
        if (!fired && (b[g] - S[g]) % restart::kMerBuffer == 0 && b[g] < E[g] && cum > restart::kRepeatLimit)
            fired = true;
    }
    out[c] = fired ? 1u : 0u;
    if (cons) {
        for (int g = 0; g < G; ++g) cons[c * (uint64_t)(G + 1) + g] = cz[g];
        cons[c * (uint64_t)(G + 1) + G] = i;
    }
    const uint64_t nxt = (uint64_t)(i + 1) << kbits;
    uint64_t lo = j, hi = N;   // first stream index with key2 >= nxt
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (key2[mid] < nxt) lo = mid + 1;
        else hi = mid;
    }
    cend[c] = lo;
}

// drop the stream ranges [rlo[r], rhi[r]) (sorted, disjoint; rpre[r] = records dropped
// before range r), order kept
__global__ void compat_drop_kernel(const uint64_t* __restrict__ k_in, const uint32_t* __restrict__ v_in, uint64_t N,
                                   const uint64_t* __restrict__ rlo, const uint64_t* __restrict__ rhi,
                                   const uint64_t* __restrict__ rpre, uint32_t R, uint64_t* __restrict__ k_out,
                                   uint32_t* __restrict__ v_out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    uint32_t lo = 0, hi = R;   // ranges starting at or before j
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rlo[mid] <= j) lo = mid + 1;
        else hi = mid;
    }
    uint64_t drop = 0;
    if (lo > 0) {
        if (j < rhi[lo - 1]) return;
        drop = rpre[lo - 1] + (rhi[lo - 1] - rlo[lo - 1]);
    }
    k_out[j - drop] = k_in[j];
    v_out[j - drop] = v_in[j];
}

// records of chunks [c0, c1) in the chunk-major stream: lower_bound of c0 << kbits and of
// c1 << kbits over key2 (sorted ascending), one lane each
__global__ void compat_chunk_span_kernel(const uint64_t* __restrict__ key2, uint64_t n, int kbits, uint32_t c0,
                                         uint32_t c1, uint64_t* __restrict__ out) {
    const int t = threadIdx.x;
    if (t >= 2) return;
    const uint64_t want = (uint64_t)(t ? c1 : c0) << kbits;
    uint64_t lo = 0, len = n;
    while (len > 0) {
        const uint64_t h = len >> 1;
        if (key2[lo + h] < want) { lo += h + 1; len -= h + 1; }
        else len = h;
    }
    out[t] = lo;
}

// MergeTable (ParallelMemHash.cpp:105-121): every entry of the thread table is re-added
// with AddHashEntry (MemHash.cpp:209-251) into the global table: lower_bound, a
// collision when equivalent (MheCompare both ways false), else inserted at the
// lower_bound; entries are already Extended() (:223), so nothing is re-extended.
//
// The table was built by the same lower_bound inserts, so nearly every re-add lands at the
// end of the merged prefix: while that holds the merged bucket IS the table's prefix.  Pass
// 1 (compat_merge_spec_kernel, one lane per entry of every bucket) checks exactly that:
// entry j's lower_bound over the table's own prefix [0, j) (std::lower_bound's probes).
// The first entry of a bucket that would not append -- an equivalent copy (A.10) or an
// insert inside the prefix -- starts pass 2 (compat_merge_fix_kernel) on that bucket only:
// the exact sequential merge from there, one workgroup, a batch of entries per round
// (each lower_bound over the merged prefix followed by the batch's earlier entries; the
// batch is applied up to its first entry that does not append, which is then dropped or
// inserted as the serial merge would).  Buckets of one diagonal hold most of a related
// input's matches (4.5 M at BASELINE config 3), so an in-place serial insertion merge of
// them is quadratic.
template <int MG>
__global__ __launch_bounds__(256) void compat_merge_spec_kernel(const uint32_t* __restrict__ tsize,
                                                                const uint32_t* __restrict__ bstart,
                                                                const uint32_t* __restrict__ tbl,
                                                                const int64_t* __restrict__ pool, int G, uint32_t Tb,
                                                                const uint32_t* __restrict__ tscan, uint64_t total,
                                                                uint32_t* __restrict__ first_fail) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total) return;
    uint32_t lo = 0, hi = Tb;   // the bucket: the last b with tscan[b] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tscan[mid] <= g) lo = mid;
        else hi = mid;
    }
    const uint32_t b = lo, j = (uint32_t)(g - tscan[b]);
    if (j == 0 || j >= tsize[b]) return;
    const uint32_t* v = tbl + bstart[b];
    Mhe<MG> e;
    load_entry(pool, v[j], G, e);
    if (lower_bound_tbl<MG>(v, j, pool, G, e) != j) atomicMin(&first_fail[b], j);
}

// lower_bound (std::lower_bound's probes) of e over the merged prefix v[0, out) followed by
// the batch entries v[j, j + t)
template <int MG>
__device__ __forceinline__ uint32_t lower_bound_merge(const uint32_t* v, uint32_t out, uint32_t j, uint32_t t,
                                                     const int64_t* __restrict__ pool, int G, const Mhe<MG>& e) {
    uint32_t first = 0, len = out + t;
    Mhe<MG> x;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        load_entry(pool, mid < out ? v[mid] : v[j + (mid - out)], G, x);
        if (mhe_less(x, e)) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

template <int MG, int kBlk>
__global__ __launch_bounds__(kBlk) void compat_merge_fix_kernel(uint32_t* __restrict__ tsize,
                                                               const uint32_t* __restrict__ bstart,
                                                               uint32_t* __restrict__ tbl,
                                                               const int64_t* __restrict__ pool, int G,
                                                               const uint32_t* __restrict__ first_fail,
                                                               unsigned long long* __restrict__ collisions) {
    const uint32_t b = blockIdx.x;
    const uint32_t j0 = first_fail[b];
    if (j0 == 0xFFFFFFFFu) return;
    __shared__ uint32_t s_bad, s_res, s_id;
    const uint32_t n = tsize[b];
    uint32_t* v = tbl + bstart[b];
    uint32_t out = j0, j = j0, dropped = 0;   // merged prefix v[0, out); unread entries v[j, n)
    while (j < n) {   // workgroup-uniform
        const uint32_t t = threadIdx.x;
        const uint32_t B = min((uint32_t)kBlk, n - j);
        if (t == 0) s_bad = B;
        __syncthreads();
        uint32_t id = 0, res = 0;
        if (t < B) {
            id = v[j + t];
            Mhe<MG> e;
            load_entry(pool, id, G, e);
            res = lower_bound_merge<MG>(v, out, j, t, pool, G, e);
            if (res != out + t) atomicMin(&s_bad, t);
        }
        __syncthreads();
        const uint32_t bad = s_bad;
        if (t == bad) {
            s_res = res;
            s_id = id;
        }
        if (out != j && t < bad) v[out + t] = id;   // (every lane read its entry before the barrier)
        __syncthreads();
        out += bad;
        j += bad;
        if (bad < B) {   // entry j: its lower_bound res was taken over exactly the merged prefix
            const uint32_t it = s_res, eid = s_id;
            Mhe<MG> e, x;
            load_entry(pool, eid, G, e);
            bool coll = false;
            if (it != out) {
                load_entry(pool, v[it], G, x);
                coll = !mhe_less(x, e) && !mhe_less(e, x);
            }
            if (coll) {
                ++dropped;
            } else {   // insert at it: v[it, out) moves up one slot (v[out] <= v[j], read already)
                for (uint32_t top = out; top > it;) {
                    const uint32_t low = top - it > (uint32_t)kBlk ? top - kBlk : it;
                    const uint32_t idx = low + t;
                    uint32_t tmp = 0;
                    if (idx < top) tmp = v[idx];
                    __syncthreads();
                    if (idx < top) v[idx + 1] = tmp;
                    __syncthreads();
                    top = low;
                }
                if (t == 0) v[it] = eid;
                ++out;
            }
            ++j;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        tsize[b] = out;
        if (dropped) atomicAdd(collisions, (unsigned long long)dropped);
    }
}

// Does a chunk start split a run of equal keys of its genome (sk: the genome-major SMLs)?
// Only such runs' SML order is observable by the chunked search under the default
// tolerances (which side of the start a copy falls on); without any, the tie replay is skipped.
__global__ void compat_split_kernel(const uint64_t* __restrict__ sk, GenomeTable gt, const uint64_t* __restrict__ cs,
                                    uint32_t nch, uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int G = gt.G;
    const uint64_t c = t / G;
    const int g = (int)(t % G);
    if (c >= nch) return;
    const uint64_t p = cs[c * G + g];
    if (p == 0 || p >= gt.m[g]) return;
    const uint64_t* k = sk + gt.base[g];
    if (k[p - 1] == k[p]) atomicOr(out, 1u);
}

// The chunk-major stream as packed records for the packed-record probe and materialize
// kernels (RecView): group key = masked-ckey bits 1-30 and the chunk's parity (a group cut
// by a chunk start, A.12, meets its other part across the boundary), parity, 32-bit index.
// Those kernels compare group keys of neighbours for equality only, so these bits serve
// wherever two different neighbouring masked keys differ in them; a boundary where they do
// not sets *clash and the caller numbers the groups by a scan of group heads instead (exact
// either way).  (compat_gid: mums_internal.h, shared with chunked.hip's direct records.)

// list / cnt (optional): compat_cand_kernel's candidates, collected in the same pass
__global__ void compat_recs_kernel(const uint64_t* __restrict__ key2, const uint32_t* __restrict__ idx, uint64_t n,
                                   int kbits, uint64_t* __restrict__ rec, uint32_t* __restrict__ clash,
                                   uint64_t* __restrict__ list, unsigned long long* __restrict__ cnt, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t k = key2[j], g = compat_gid(k, kbits);
    const uint64_t kp = j > 0 ? key2[j - 1] : ~k;
    if (j > 0 && (kp >> 1) != (k >> 1) && compat_gid(kp, kbits) == g) atomicOr(clash, 1u);
    if (list && (kp >> 1) != (k >> 1)) {   // a group head: more than MER_REPEAT_LIMIT records?
        const uint64_t e = j + restart::kRepeatLimit;
        if (e < n && (key2[e] >> 1) == (k >> 1)) {
            const unsigned long long q = atomicAdd(cnt, 1ull);
            if (q < cap) list[q] = j;
        }
    }
    rec[j] = (g << 33) | ((k & 1ull) << 32) | idx[j];
}

__global__ void compat_heads_kernel(const uint64_t* __restrict__ key2, uint64_t n, uint32_t* __restrict__ head) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    head[j] = (j == 0 || (key2[j] >> 1) != (key2[j - 1] >> 1)) ? 1u : 0u;
}

// group key = the group's ordinal (exclusive scan of the heads + own head) mod 2^31
__global__ void compat_recs_scan_kernel(const uint64_t* __restrict__ key2, const uint32_t* __restrict__ idx,
                                        const uint32_t* __restrict__ hscan, uint64_t n, uint64_t* __restrict__ rec) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t k = key2[j];
    const uint32_t head = (j == 0 || (k >> 1) != (key2[j - 1] >> 1)) ? 1u : 0u;
    const uint64_t g = (uint64_t)(hscan[j] + head) & 0x7FFFFFFFull;
    rec[j] = (g << 33) | ((k & 1ull) << 32) | idx[j];
}

// SetMatchLog in compat mode: the chunk of every probe is nondecreasing in AddHashEntry call
// order (the chunk-major stream), so the chunks are ranges of probes: pfirst[c] = first probe
// of chunk c (nch + 1 entries, pfirst[nch] = P).  probe_info low word = the group's first
// stream record, whose key2 carries the chunk above kbits.
__global__ void compat_probe_chunk_kernel(const uint64_t* __restrict__ probe_info, uint64_t P,
                                          const uint64_t* __restrict__ key2, int kbits, uint32_t nch,
                                          uint32_t* __restrict__ pfirst) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P) return;
    const uint64_t c = key2[probe_info[k] & 0xFFFFFFFFull] >> kbits;
    const int64_t cp = k ? (int64_t)(key2[probe_info[k - 1] & 0xFFFFFFFFull] >> kbits) : -1;
    for (int64_t x = cp + 1; x <= (int64_t)c && x <= (int64_t)nch; ++x) pfirst[x] = (uint32_t)k;
    if (k + 1 == P)
        for (uint64_t x = c + 1; x <= nch; ++x) pfirst[x] = (uint32_t)P;
}

__global__ void compat_strip_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n,
                                    uint64_t mask) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[j] = in[j] & mask;
}

}  // namespace

hipError_t launch_compat_strip(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t mask, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(compat_strip_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, out, n, mask);
    return hipGetLastError();
}

// scratch: n + 1 u32 (the scan fallback's heads), scan_tmp for exclusive_scan_u32 over n
hipError_t launch_compat_recs(const uint64_t* key2, const uint32_t* idx, uint64_t n, int kbits, uint64_t* rec,
                              uint32_t* clash, uint32_t* scratch, void* scan_tmp, bool force_scan, uint64_t* list,
                              unsigned long long* cnt, uint64_t cap, hipStream_t st) {
    hipError_t e;
    if (list && (e = hipMemsetAsync(cnt, 0, 8, st)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
    if (!force_scan || list) {   // (the candidates come from this pass either way)
        if ((e = hipMemsetAsync(clash, 0, 4, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(compat_recs_kernel, grid, blk, 0, st, key2, idx, n, kbits, rec, clash, list, cnt, cap);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        uint32_t h = 0;
        if ((e = hipMemcpyAsync(&h, clash, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        if (!h && !force_scan) return hipSuccess;
    }
    hipLaunchKernelGGL(compat_heads_kernel, grid, blk, 0, st, key2, n, scratch);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(scratch, n, scan_tmp, nullptr, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(compat_recs_scan_kernel, grid, blk, 0, st, key2, idx, (const uint32_t*)scratch, n, rec);
    return hipGetLastError();
}

hipError_t launch_compat_split(const uint64_t* sk, const GenomeTable& gt, const uint64_t* cs, uint32_t nch,
                               uint32_t* out, hipStream_t st) {
    hipError_t e = hipMemsetAsync(out, 0, 4, st);
    if (e != hipSuccess) return e;
    const uint64_t n = (uint64_t)nch * gt.G;
    hipLaunchKernelGGL(compat_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sk, gt, cs, nch, out);
    return hipGetLastError();
}

hipError_t launch_compat_probe_chunks(const uint64_t* probe_info, uint64_t P, const uint64_t* key2, int kbits,
                                      uint32_t nch, uint32_t* pfirst, hipStream_t st) {
    if (P == 0) return hipMemsetAsync(pfirst, 0, ((uint64_t)nch + 1) * 4, st);
    hipLaunchKernelGGL(compat_probe_chunk_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, probe_info, P,
                       key2, kbits, nch, pfirst);
    return hipGetLastError();
}

hipError_t launch_genome_keys(uint64_t* ckey, uint64_t N, const GenomeTable& gt, int kbits, hipStream_t st) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(genome_keys_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, ckey, N, gt, kbits);
    return hipGetLastError();
}

hipError_t launch_compat_breaks(const uint64_t* sk, const GenomeTable& gt, uint64_t kmask, int mx, uint64_t chunk,
                                uint64_t* cs, uint64_t* bm, uint32_t cap, uint32_t* d_nch, uint32_t* err,
                                hipStream_t st) {
    hipLaunchKernelGGL(compat_breaks_kernel, dim3(1), dim3(64), 0, st, sk, gt, kmask, mx, chunk, cs, bm, cap, d_nch,
                       err);
    return hipGetLastError();
}

hipError_t launch_compat_find(const uint64_t* sk, const GenomeTable& gt, uint64_t kmask, int mx, int L, uint64_t* cs,
                              const uint64_t* bm, uint32_t nch, hipStream_t st) {
    if (nch < 2) return hipSuccess;
    const uint64_t t = (uint64_t)(nch - 1) * gt.G;
    hipLaunchKernelGGL(compat_find_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, sk, gt, kmask, mx, L,
                       cs, bm, nch);
    return hipGetLastError();
}

hipError_t launch_compat_chunk_keys(const uint64_t* sk, const uint32_t* sv, uint64_t N, const GenomeTable& gt,
                                    int kbits, const uint64_t* cs, uint32_t nch, uint64_t* key2, uint32_t* val2,
                                    uint64_t* ck, hipStream_t st) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(compat_chunk_keys_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, sk, sv, N, gt,
                       kbits, cs, nch, key2, val2, ck);
    return hipGetLastError();
}

hipError_t launch_compat_cands(const uint64_t* key2, uint64_t N, uint64_t* list, unsigned long long* cnt, uint64_t cap,
                               hipStream_t st) {
    hipError_t e = hipMemsetAsync(cnt, 0, 8, st);
    if (e != hipSuccess || N == 0) return e;
    hipLaunchKernelGGL(compat_cand_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, key2, N, list, cnt, cap);
    return hipGetLastError();
}

hipError_t launch_compat_fire(const restart::PlanData& d, const uint64_t* key2, uint64_t N, int kbits,
                              const uint64_t* cand, uint64_t C, const uint64_t* cs, uint32_t nch, uint32_t* out,
                              uint64_t* cend, uint64_t* cons, hipStream_t st) {
    if (C == 0) return hipSuccess;
    hipLaunchKernelGGL(compat_fire_kernel, dim3((unsigned)((C + 63) / 64)), dim3(64), 0, st, d, key2, N, kbits, cand, C,
                       cs, nch, out, cend, cons);
    return hipGetLastError();
}

hipError_t launch_compat_drop(const uint64_t* k_in, const uint32_t* v_in, uint64_t N, const uint64_t* rlo,
                              const uint64_t* rhi, const uint64_t* rpre, uint32_t R, uint64_t* k_out, uint32_t* v_out,
                              hipStream_t st) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(compat_drop_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, k_in, v_in, N, rlo, rhi,
                       rpre, R, k_out, v_out);
    return hipGetLastError();
}

// tscan: exclusive scan of tsize (Tb entries), total = its sum; first_fail: Tb words (scratch)
hipError_t launch_compat_merge(uint32_t* tsize, const uint32_t* bstart, uint32_t* tbl, const int64_t* pool, int G,
                               uint32_t Tb, unsigned long long* collisions, const uint32_t* tscan, uint64_t total,
                               uint32_t* first_fail, hipStream_t st) {
    // test hook (read per call): every bucket through the exact merge from its first entry
    const bool all_exact = getenv("MUMS_DEV_COMPAT_MERGE_EXACT") != nullptr;
    hipError_t e = hipMemsetAsync(first_fail, all_exact ? 0x00 : 0xFF, (size_t)Tb * 4, st);
    if (e != hipSuccess || total == 0) return e;
    const dim3 sgrid((unsigned)((total + 255) / 256)), sblk(256);
#define MUMS_COMPAT_MERGE(MGV, BLK)                                                                                   \
    do {                                                                                                              \
        if (!all_exact)                                                                                               \
            hipLaunchKernelGGL(compat_merge_spec_kernel<MGV>, sgrid, sblk, 0, st, tsize, bstart, tbl, pool, G, Tb,    \
                               tscan, total, first_fail);                                                             \
        hipLaunchKernelGGL((compat_merge_fix_kernel<MGV, BLK>), dim3(Tb), dim3(BLK), 0, st, tsize, bstart, tbl, pool, \
                           G, first_fail, collisions);                                                                \
    } while (0)
    if (G <= 4) MUMS_COMPAT_MERGE(4, 1024);
    else if (G <= 8) MUMS_COMPAT_MERGE(8, 1024);
    else if (G <= 16) MUMS_COMPAT_MERGE(16, 512);
    else if (G <= 32) MUMS_COMPAT_MERGE(32, 256);
    else MUMS_COMPAT_MERGE(64, 256);
#undef MUMS_COMPAT_MERGE
    return hipGetLastError();
}

hipError_t launch_compat_chunk_span(const uint64_t* key2, uint64_t n, int kbits, uint32_t c0, uint32_t c1,
                                    uint64_t* out, hipStream_t st) {
    hipLaunchKernelGGL(compat_chunk_span_kernel, dim3(1), dim3(64), 0, st, key2, n, kbits, c0, c1, out);
    return hipGetLastError();
}

// the exact merge alone, from first_fail[b] (~0: bucket skipped) in each of nb buckets
hipError_t launch_compat_merge_from(uint32_t* tsize, const uint32_t* bstart, uint32_t* tbl, const int64_t* pool, int G,
                                    uint32_t nb, const uint32_t* first_fail, unsigned long long* collisions,
                                    hipStream_t st) {
    if (nb == 0) return hipSuccess;
#define MUMS_COMPAT_FIX(MGV, BLK)                                                                                     \
    hipLaunchKernelGGL((compat_merge_fix_kernel<MGV, BLK>), dim3(nb), dim3(BLK), 0, st, tsize, bstart, tbl, pool, G,  \
                       first_fail, collisions)
    if (G <= 4) MUMS_COMPAT_FIX(4, 1024);
    else if (G <= 8) MUMS_COMPAT_FIX(8, 1024);
    else if (G <= 16) MUMS_COMPAT_FIX(16, 512);
    else if (G <= 32) MUMS_COMPAT_FIX(32, 256);
    else MUMS_COMPAT_FIX(64, 256);
#undef MUMS_COMPAT_FIX
    return hipGetLastError();
}

}  // namespace mums
