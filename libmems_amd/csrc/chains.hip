// chains.hip -- seed-chain labelling of every probe before the bucket replay (rows A9, A11).
//
// MatchFinder::ExtendMatch (MatchFinder.h:218-374) grows a probe to the maximal
// chain of seed hits with gaps <= L through the probe's column 0.
// That chain depends only on the probe's "line" -- its genome set, the strands
// (SetDirection, MemHash.cpp:189-203) and the diagonal of every component -- and on
// which hit columns the chain contains, so every probe of one chain extends to the
// SAME MatchHashEntry.  Instead of extending the first new probe of a chain inside
// the (sequential) per-bucket replay, all probes are labelled here in parallel:
//
//   1. chain_key_kernel   : line hash (32 b) | reference-genome start -> sort key
//   2. radix sort (64-bit) : probes of one line become adjacent, by position
//   3. chain_link_kernel  : neighbours on one line are in one chain iff a chain of
//                           hits (gaps <= L) joins them: gap <= L, else a walk of
//                           the hit columns between them; segment ends walk on to
//                           the chain's end (left walks in chain_left_kernel)
//   4. chain_walk_kernel  : walks longer than a per-lane budget, one workgroup each
//                           (L-jumps speculated across 256 lanes, as ExtendMatch's
//                           directions 0/1, then the furthest hit within L)
//   5. chain_seg / chain_entry kernels: segment ids (scan), the extended entry of
//                           every chain and chain_of[probe].
// The replay (replay.hip) then inserts chain entries without extending anything.
// A 32-bit line-hash collision only splits runs of a line: every probe still gets
// its true chain ends (a segment end always walks to the real end of its chain).
#include <cstdio>
#include <cstdlib>

#include "match_device.h"
#include "seed_device.h"

namespace mums {

namespace {

#ifndef MUMS_WALK_BUDGET
#define MUMS_WALK_BUDGET 48   // measured: 24 / 48 / 96 / 384 -> chains 6.0 / 5.6 / 6.1 / 8.5 ms (related 4 x 10 Mbp)
#endif
constexpr int kWalkBudget = MUMS_WALK_BUDGET;   // hit evaluations per lane before a walk goes to a workgroup

struct WalkItem {
    uint32_t j;      // position in line order
    int32_t kind;    // 0: bridge j -> j+1, 1: right end, 2: left end
    int64_t cur;     // column reached so far (frame of probe ord[j])
    int64_t stop;    // bridge: done once cur >= stop
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

// probe of sorted-stream group k (the AddHashEntry argument), see build_probe
template <int MG, typename View>
__device__ __forceinline__ void probe_of(const View& v, const uint64_t* __restrict__ /*probe_info*/, uint32_t k,
                                         const GenomeTable& gt, const MatchParams& /*mp*/, int L, Mhe<MG>& P) {
    load_probe<MG>(v, k, gt.G, L, P);
}

// line invariants: reference start x = s_ref (> 0); per other component the
// diagonal s_g - s_ref (forward) or |s_g| + s_ref (reverse)
template <int MG>
__device__ __forceinline__ uint32_t line_hash(const Mhe<MG>& P, int G) {
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
    return (uint32_t)(h >> 32);
}

template <int MG>
__device__ __forceinline__ bool same_line(const Mhe<MG>& a, const Mhe<MG>& b) {
    const int ra = first_start(a), rb = first_start(b);
    if (ra != rb) return false;
    const int64_t xa = start_at(a, ra), xb = start_at(b, rb);
    bool ok = true;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t sa = a.s[g], sb = b.s[g];
        const bool za = sa == 0, zb = sb == 0;
        ok = ok && (za == zb) && ((sa < 0) == (sb < 0));
        if (!za && !zb) {
            const int64_t da = sa > 0 ? sa - xa : -sa + xa;
            const int64_t db = sb > 0 ? sb - xb : -sb + xb;
            ok = ok && (da == db);
        }
    }
    return ok;
}

// column range where every component's seed window lies inside its sequence
template <int MG>
__device__ __forceinline__ void frame_bounds(const Mhe<MG>& P, const GenomeTable& gt, int64_t* clo, int64_t* chi) {
    int64_t lo = INT64_MIN, hi = INT64_MAX;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t s = P.s[g];
        if (g < gt.G && s != 0) {
            const int64_t m = (int64_t)gt.m[g];
            const int64_t l = s > 0 ? 1 - s : -s - m;
            const int64_t u = s > 0 ? m - s : -s - 1;
            lo = l > lo ? l : lo;
            hi = u < hi ? u : hi;
        }
    }
    *clo = lo;
    *chi = hi;
}

// seed hit at column c (MatchFinder.h:265-293): all present components have the same
// canonical seed and strand-relative parity there, all windows inside the sequences
template <int MG>
__device__ __forceinline__ bool hit_lane(int64_t c, const Mhe<MG>& P, const GenomeTable& gt, int64_t clo, int64_t chi,
                                         const uint32_t* __restrict__ packed, const SeedSpec& ss) {
    if (c < clo || c > chi) return false;
    bool first = true, ok = true;
    uint64_t v0 = 0;
    uint32_t o0 = 0;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        const int64_t s = P.s[g];
        if (ok && g < gt.G && s != 0) {
            const int64_t p = s > 0 ? s - 1 + c : -s - 1 - c;
            const uint64_t k = ckey_at(packed + gt.woff[g], (uint64_t)p, ss);
            const uint64_t v = k >> 1;
            const uint32_t o = s > 0 ? (uint32_t)((k & 1) ^ 1) : (uint32_t)(k & 1);
            if (first) { v0 = v; o0 = o; first = false; }
            else ok = (v == v0) && (o == o0);
        }
    }
    return ok;
}

// Greedy walk along the chain from hit column cur in direction dir: repeatedly move
// to the furthest hit within L columns.  state 0: the chain ends at the returned
// column; 1: reached `stop`; 2: budget spent (returned column = progress so far).
template <int MG>
__device__ int64_t walk_lane(int dir, int64_t cur, int64_t stop, int budget, int L, const Mhe<MG>& P,
                             const GenomeTable& gt, int64_t clo, int64_t chi, const uint32_t* __restrict__ packed,
                             const SeedSpec& ss, int* state) {
    for (;;) {
        if (dir > 0 ? cur >= stop : cur <= stop) { *state = 1; return cur; }
        if (budget <= 0) { *state = 2; return cur; }
        int d = L;
        for (; d >= 1; --d) {
            --budget;
            if (hit_lane<MG>(cur + dir * (int64_t)d, P, gt, clo, chi, packed, ss)) break;
        }
        if (d == 0) { *state = 0; return cur; }
        cur += dir * (int64_t)d;
    }
}

__device__ __forceinline__ int wg_first_true(bool pred, int* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t b = __ballot(pred);
    if (lane == 0) red[wv] = b ? wv * 64 + (__ffsll((long long)b) - 1) : kBlock;
    __syncthreads();
    int r = red[0];
    #pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) r = min(r, red[w]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ int wg_last_true(bool pred, int* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t b = __ballot(pred);
    if (lane == 0) red[wv] = b ? wv * 64 + 63 - __clzll((long long)b) : -1;
    __syncthreads();
    int r = red[0];
    #pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) r = max(r, red[w]);
    __syncthreads();
    return r;
}

// ---- kernels ------------------------------------------------------------------------

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_key_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                           GenomeTable gt, MatchParams mp, int L,
                                                           uint64_t* __restrict__ lkey) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    Mhe<MG> Q;
    probe_of<MG, View>(v, probe_info, (uint32_t)k, gt, mp, L, Q);
    const int ref = first_start(Q);
    const uint64_t x = (uint64_t)start_at(Q, ref);
    lkey[k] = ((uint64_t)line_hash<MG>(Q, gt.G) << 32) | (x & 0xFFFFFFFFull);
}

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_link_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                            GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                            const uint32_t* __restrict__ ord,
                                                            const uint32_t* __restrict__ packed,
                                                            uint8_t* __restrict__ link, int64_t* __restrict__ rcol,
                                                            WalkItem* __restrict__ queue,
                                                            unsigned int* __restrict__ qcount) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    const int L = ss.L;
    Mhe<MG> A, B;
    probe_of<MG, View>(v, probe_info, ord[j], gt, mp, L, A);
    bool same = false;
    if (j + 1 < P) {
        probe_of<MG, View>(v, probe_info, ord[j + 1], gt, mp, L, B);
        same = same_line<MG>(A, B);
    }
    const int64_t xa = start_at(A, first_start(A));
    int64_t clo, chi;
    frame_bounds<MG>(A, gt, &clo, &chi);
    int state;
    if (same) {
        const int64_t stop = start_at(B, first_start(B)) - xa - L;
        const int64_t c = walk_lane<MG>(+1, 0, stop, kWalkBudget, L, A, gt, clo, chi, packed, ss, &state);
        if (state == 1) {
            link[j] = 1;
        } else if (state == 0) {
            link[j] = 0;
            rcol[j] = xa + c;
        } else {
            link[j] = 0;
            const unsigned q = atomicAdd(qcount, 1u);
            queue[q] = WalkItem{(uint32_t)j, 0, c, stop};
        }
    } else {
        link[j] = 0;
        const int64_t c = walk_lane<MG>(+1, 0, INT64_MAX, kWalkBudget, L, A, gt, clo, chi, packed, ss, &state);
        if (state == 0) {
            rcol[j] = xa + c;
        } else {
            const unsigned q = atomicAdd(qcount, 1u);
            queue[q] = WalkItem{(uint32_t)j, 1, c, INT64_MAX};
        }
    }
}

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_left_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                            GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                            const uint32_t* __restrict__ ord,
                                                            const uint32_t* __restrict__ packed,
                                                            const uint8_t* __restrict__ link,
                                                            int64_t* __restrict__ lcol, WalkItem* __restrict__ queue,
                                                            unsigned int* __restrict__ qcount) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    if (j > 0 && link[j - 1]) return;
    const int L = ss.L;
    Mhe<MG> A;
    probe_of<MG, View>(v, probe_info, ord[j], gt, mp, L, A);
    const int64_t xa = start_at(A, first_start(A));
    int64_t clo, chi;
    frame_bounds<MG>(A, gt, &clo, &chi);
    int state;
    const int64_t c = walk_lane<MG>(-1, 0, INT64_MIN, kWalkBudget, L, A, gt, clo, chi, packed, ss, &state);
    if (state == 0) {
        lcol[j] = xa + c;
    } else {
        const unsigned q = atomicAdd(qcount, 1u);
        queue[q] = WalkItem{(uint32_t)j, 2, c, INT64_MIN};
    }
}

// Long walks, one workgroup per item (grid-stride over the queue).  Each iteration
// evaluates the 1024 columns after the current chain end (4 per lane, one 64-column
// ballot word per wave and sub-step) and one lane scans the 16 words for the first
// run of >= L columns without a hit: the chain ends at the last hit before it (the
// maximal chain of hits with gaps <= L); without such a run the walk
// continues from the last hit of the window.
#ifndef MUMS_WALK_CPL
#define MUMS_WALK_CPL 4
#endif
constexpr int kWalkCols = MUMS_WALK_CPL * kBlock;   // columns per workgroup step (per lane: MUMS_WALK_CPL)

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_walk_kernel(View v, const uint64_t* __restrict__ probe_info,
                                                            GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                            const uint32_t* __restrict__ ord,
                                                            const uint32_t* __restrict__ packed,
                                                            const WalkItem* __restrict__ queue,
                                                            const unsigned int* __restrict__ qcount,
                                                            uint8_t* __restrict__ link, int64_t* __restrict__ rcol,
                                                            int64_t* __restrict__ lcol) {
    __shared__ uint64_t words[kWalkCols / 64];
    __shared__ int64_t s_adv;
    __shared__ int s_broke;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int L = ss.L;
    const unsigned nq = *qcount;
    for (unsigned qi = blockIdx.x; qi < nq; qi += gridDim.x) {
        const WalkItem it = queue[qi];
        Mhe<MG> A;
        probe_of<MG, View>(v, probe_info, ord[it.j], gt, mp, L, A);
        const int64_t xa = start_at(A, first_start(A));
        int64_t clo, chi;
        frame_bounds<MG>(A, gt, &clo, &chi);
        const int dir = it.kind == 2 ? -1 : +1;
        int64_t cur = it.cur;
        bool reached = false;
        for (;;) {
            if (dir > 0 ? cur >= it.stop : cur <= it.stop) { reached = true; break; }
            #pragma unroll
            for (int r = 0; r < kWalkCols / kBlock; ++r) {   // column offsets 1 + 256 r + tid
                const int64_t k = 1 + (int64_t)r * kBlock + tid;
                const uint64_t m = __ballot(hit_lane<MG>(cur + dir * k, A, gt, clo, chi, packed, ss));
                if (lane == 0) words[r * (kBlock / 64) + wv] = m;
            }
            __syncthreads();
            if (tid == 0) {
                int64_t last = 0;   // offset of the last reachable hit (0 = cur)
                int carry = 0;      // columns without a hit since it
                int broke = 0;
                for (int wi = 0; wi < kWalkCols / 64 && !broke; ++wi) {
                    const uint64_t x = words[wi];
                    if (x == 0) {
                        carry += 64;
                        broke = carry >= L;
                        continue;
                    }
                    const int f = __builtin_ctzll(x);
                    if (carry + f >= L) { broke = 1; break; }
                    // bit i of a: columns i .. i+L-1 of this word all miss
                    uint64_t a = ~x;
                    int len = 1;
                    while (2 * len <= L) { a &= a >> len; len *= 2; }
                    if (len < L) a &= a >> (L - len);
                    if (a) {
                        const int r0 = __builtin_ctzll(a);
                        const uint64_t below = x & ((1ull << r0) - 1);
                        last = (int64_t)wi * 64 + (63 - __builtin_clzll(below)) + 1;
                        broke = 1;
                        break;
                    }
                    const int hb = 63 - __builtin_clzll(x);
                    last = (int64_t)wi * 64 + hb + 1;
                    carry = 63 - hb;
                }
                s_adv = last;
                s_broke = broke;
            }
            __syncthreads();
            cur += dir * s_adv;
            const int broke = s_broke;
            __syncthreads();
            if (broke) {
                reached = dir > 0 ? cur >= it.stop : cur <= it.stop;
                break;
            }
        }
        if (tid == 0) {
            if (it.kind == 0) {
                link[it.j] = reached ? 1 : 0;
                if (!reached) rcol[it.j] = xa + cur;
            } else if (it.kind == 1) {
                rcol[it.j] = xa + cur;
            } else {
                lcol[it.j] = xa + cur;
            }
        }
        __syncthreads();
    }
}

// seg[j] = 1 at segment starts (scanned to segment ids afterwards)
__global__ __launch_bounds__(kBlock) void chain_flag_kernel(const uint8_t* __restrict__ link, uint64_t P,
                                                            uint32_t* __restrict__ seg) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    seg[j] = (j == 0 || !link[j - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void chain_seg_kernel(const uint8_t* __restrict__ link,
                                                           const uint32_t* __restrict__ ord,
                                                           const uint32_t* __restrict__ seg_excl, uint64_t P,
                                                           const int64_t* __restrict__ rcol,
                                                           uint32_t* __restrict__ chain_of,
                                                           int64_t* __restrict__ seg_r) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    const uint32_t f = (j == 0 || !link[j - 1]) ? 1u : 0u;
    const uint32_t s = seg_excl[j] + f - 1u;
    chain_of[ord[j]] = s;
    if (!link[j]) seg_r[s] = rcol[j];
}

// the extended entry of every chain (ExtendMatch write-back, MatchFinder.h:218-374;
// stored copies have m_mersize 0, MatchHashEntry.cpp:122): pool[s] = {len, offset, starts}
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void chain_entry_kernel(View v, const uint64_t* __restrict__ probe_info, uint64_t P,
                                                             GenomeTable gt, MatchParams mp, int L,
                                                             const uint32_t* __restrict__ ord,
                                                             const uint8_t* __restrict__ link,
                                                             const uint32_t* __restrict__ seg_excl,
                                                             const int64_t* __restrict__ lcol,
                                                             const int64_t* __restrict__ seg_r,
                                                             int64_t* __restrict__ pool) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= P) return;
    if (j > 0 && link[j - 1]) return;
    const uint32_t s = seg_excl[j];
    Mhe<MG> A;
    probe_of<MG, View>(v, probe_info, ord[j], gt, mp, L, A);
    const int64_t xa = start_at(A, first_start(A));
    const int64_t cmin = lcol[j] - xa, cmax = seg_r[s] - xa;
    int64_t* e = pool + (uint64_t)s * (uint64_t)(gt.G + 2);
    e[0] = cmax - cmin + L;
    e[1] = A.offset;
    #pragma unroll
    for (int g = 0; g < MG; ++g) {
        if (g < gt.G) {
            const int64_t sg = A.s[g];
            e[2 + g] = sg > 0 ? sg + cmin : (sg < 0 ? -((-sg) - cmax) : 0);
        }
    }
}

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

size_t chain_tmp_bytes(uint64_t P) {
    // lkey, sort A/B keys (3 x 8) + vals A/B (2 x 4) + link (1) + rcol, lcol, seg_r (3 x 8)
    // + seg (4) + queue (24) + padding
    return P * (24 + 8 + 1 + 24 + 4 + sizeof(WalkItem)) + 64 * 16;
}

// Chain labelling of the P probes (key order): chain_of[k] = chain of probe k;
// pool[c] = extended entry of chain c; *d_nchains (device) = number of chains.
template <int MG, typename View>
hipError_t launch_chains(View v, const uint64_t* probe_info, uint64_t P, const GenomeTable& gt, const MatchParams& mp,
                         const SeedSpec& ss, const uint32_t* packed, void* d_chain_tmp, void* d_scan_tmp,
                         void* d_radix_tmp, uint32_t* chain_of, int64_t* pool, uint32_t* d_nchains, hipStream_t st) {
    if (P == 0) return hipSuccess;
    char* p = (char*)d_chain_tmp;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    uint64_t* lkey = (uint64_t*)carve(P * 8);
    uint64_t* kA = (uint64_t*)carve(P * 8);
    uint64_t* kB = (uint64_t*)carve(P * 8);
    uint32_t* vA = (uint32_t*)carve(P * 4);
    uint32_t* vB = (uint32_t*)carve(P * 4);
    uint8_t* link = (uint8_t*)carve(P);
    int64_t* rcol = (int64_t*)carve(P * 8);
    int64_t* lcol = (int64_t*)carve(P * 8);
    int64_t* seg_r = (int64_t*)carve(P * 8);
    uint32_t* seg = (uint32_t*)carve(P * 4);
    WalkItem* queue = (WalkItem*)carve(P * sizeof(WalkItem));
    unsigned int* qcount = (unsigned int*)carve(64);
    hipError_t e;
    const unsigned grid = grid_of(P);
    hipLaunchKernelGGL((chain_key_kernel<MG, View>), dim3(grid), dim3(kBlock), 0, st, v, probe_info, P, gt, mp, ss.L,
                       lkey);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    int buf = 0;
    if ((e = radix_sort<uint64_t>(lkey, nullptr, P, 64, kA, vA, kB, vB, d_radix_tmp, &buf, st)) != hipSuccess) return e;
    const uint32_t* ord = buf ? vB : vA;
    const unsigned walk_grid = 2048;
    for (int pass = 0; pass < 2; ++pass) {
        if ((e = hipMemsetAsync(qcount, 0, 4, st)) != hipSuccess) return e;
        if (pass == 0)
            hipLaunchKernelGGL((chain_link_kernel<MG, View>), dim3(grid), dim3(kBlock), 0, st, v, probe_info, P, gt,
                               mp, ss, ord, packed, link, rcol, queue, qcount);
        else
            hipLaunchKernelGGL((chain_left_kernel<MG, View>), dim3(grid), dim3(kBlock), 0, st, v, probe_info, P, gt,
                               mp, ss, ord, packed, link, lcol, queue, qcount);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL((chain_walk_kernel<MG, View>), dim3(walk_grid), dim3(kBlock), 0, st, v, probe_info, gt, mp,
                           ss, ord, packed, queue, qcount, link, rcol, lcol);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (getenv("MUMS_DEV_CHAIN_DEBUG")) {   // development: long-walk queue sizes
            unsigned hq = 0;
            (void)hipMemcpyAsync(&hq, qcount, 4, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            fprintf(stderr, "chains: pass %d long walks %u of %lu probes\n", pass, hq, (unsigned long)P);
        }
    }
    hipLaunchKernelGGL(chain_flag_kernel, dim3(grid), dim3(kBlock), 0, st, link, P, seg);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(seg, P, d_scan_tmp, d_nchains, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(chain_seg_kernel, dim3(grid), dim3(kBlock), 0, st, link, ord, seg, P, rcol, chain_of, seg_r);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((chain_entry_kernel<MG, View>), dim3(grid), dim3(kBlock), 0, st, v, probe_info, P, gt, mp, ss.L,
                       ord, link, seg, lcol, seg_r, pool);
    return hipGetLastError();
}

#define MUMS_INST_CHAINS(MG, V)                                                                                   \
    template hipError_t launch_chains<MG, V>(V, const uint64_t*, uint64_t, const GenomeTable&, const MatchParams&, \
                                             const SeedSpec&, const uint32_t*, void*, void*, void*, uint32_t*,     \
                                             int64_t*, uint32_t*, hipStream_t);
MUMS_INST_CHAINS(4, MatProbes)
MUMS_INST_CHAINS(8, MatProbes)
MUMS_INST_CHAINS(16, MatProbes)
MUMS_INST_CHAINS(32, MatProbes)

}  // namespace mums
