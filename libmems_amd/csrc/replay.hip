// replay.hip -- per-bucket AddHashEntry replay + seed-chain extension (rows A10-A12).
//
// Reference: MemHash::AddHashEntry (MemHash.cpp:209-251) keeps every hash
// bucket as a vector sorted by MheCompare (MatchHashEntry.h:121-143); each probe
// is looked up with std::lower_bound, dropped as a collision when the entry
// there is equivalent, otherwise extended (MatchFinder::ExtendMatch,
// MatchFinder.h:218-374) and inserted at lower_bound of the extended copy
// (whose m_mersize is 0, MatchHashEntry.cpp:122).  Because MheCompare treats
// containment as equivalence it is not a strict weak ordering, so the exact
// binary-search probe sequence matters; it is replayed here
// with the libstdc++ __lower_bound recurrence.
//
// MI355X mapping: one 256-lane workgroup per hash bucket.  Buckets are
// independent; inside a bucket the workgroup evaluates up to 256 consecutive
// probes against the current table in parallel (one lower_bound per lane),
// takes the first non-colliding one (a workgroup ballot), extends it
// cooperatively and inserts it; everything before it is final.  Extension uses
// the fixpoint of ExtendMatch's L-jump / single-step / restart loop: the
// maximal chain of seed hits with gaps <= L through the probe,
// found with 256 speculative L-jumps per round and an L-wide fine step; a hit
// re-derives the components' seed keys from the resident 2-bit packed genomes.
#include "match_device.h"
#include "seed_device.h"

namespace mums {

namespace {

struct ExtComp {
    int64_t s;       // start (signed, 1-based)
    uint64_t woff;   // word offset of the genome in the packed array
};

__device__ __forceinline__ int block_first_true(bool pred, int* red) {
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

__device__ __forceinline__ int block_last_true(bool pred, int* red) {
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

// seed hit at alignment column c (MatchFinder.h:265-293): every component's
// masked key and strand-relative parity agree, all windows inside the sequences.
__device__ __forceinline__ bool hit_at(int64_t c, const ExtComp* comps, int nc, int64_t clo, int64_t chi,
                                       const uint32_t* __restrict__ packed, const SeedSpec& ss) {
    if (c < clo || c > chi) return false;
    uint64_t v0 = 0;
    uint32_t o0 = 0;
    bool ok = true;
    for (int j = 0; j < nc && ok; ++j) {
        const int64_t s = comps[j].s;
        const int64_t p = s > 0 ? s - 1 + c : -s - 1 - c;
        const uint64_t k = ckey_at(packed + comps[j].woff, (uint64_t)p, ss);
        const uint64_t v = k >> 1;
        const uint32_t o = s > 0 ? (uint32_t)((k & 1) ^ 1) : (uint32_t)(k & 1);
        if (j == 0) { v0 = v; o0 = o; }
        else ok = (v == v0) && (o == o0);
    }
    return ok;
}

// rightmost (dir=+1) / leftmost (dir=-1) column of the hit chain through column 0
__device__ int64_t chain_end(int dir, int L, const ExtComp* comps, int nc, int64_t clo, int64_t chi,
                             const uint32_t* __restrict__ packed, const SeedSpec& ss, int* red) {
    const int tid = threadIdx.x;
    int64_t cur = 0;
    for (;;) {
        for (;;) {  // ExtendMatch directions 0/1: jumps of L while the seed at the new end matches
            const bool h = hit_at(cur + dir * (int64_t)(tid + 1) * L, comps, nc, clo, chi, packed, ss);
            const int miss = block_first_true(!h, red);
            if (miss == kBlock) { cur += dir * (int64_t)kBlock * L; continue; }
            cur += dir * (int64_t)miss * L;
            break;
        }
        // directions 2/3: furthest hit within L single steps, then restart
        const bool h2 = tid < L ? hit_at(cur + dir * (int64_t)(tid + 1), comps, nc, clo, chi, packed, ss) : false;
        const int far = block_last_true(h2, red);
        if (far < 0) break;
        cur += dir * (int64_t)(far + 1);
    }
    return cur;
}

template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void replay_kernel(View v, uint64_t N, GenomeTable gt, MatchParams mp, SeedSpec ss,
                                                        const uint64_t* __restrict__ probe_info,
                                                        const uint32_t* __restrict__ ids,
                                                        const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ bend, uint32_t* tbl,
                                                        int64_t* pool, const uint32_t* __restrict__ packed,
                                                        uint32_t* __restrict__ tsize, DevCounters* ctr) {
    const int L = ss.L;
    __shared__ int red[kBlock / 64];
    __shared__ int64_t sP[MG + 2];
    __shared__ ExtComp comps[MG];
    __shared__ int s_nc;
    __shared__ int64_t s_clo, s_chi;
    __shared__ uint32_t s_ins, s_id;

    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t beg = bstart[b];
    const uint32_t K_b = bend[b] - beg;
    if (K_b == 0) return;
    const int G = gt.G;
    uint32_t* tb = tbl + beg;
    const uint32_t* hd = ids + beg;
    uint32_t t = 0, i = 0;
    unsigned long long coll = 0;

    while (i < K_b) {
        const uint32_t c = min((uint32_t)kBlock, K_b - i);
        bool isnew = false;
        Mhe<MG> P;
        if ((uint32_t)tid < c) {
            uint32_t gs;
            const uint64_t info = probe_info[hd[i + tid]];
            const uint64_t h = info & 0xFFFFFFFFull;
            build_probe<MG, View>(v, h, h + ((info >> 32) & 0xFFFFull), gt, mp, L, P, &gs);
            const uint32_t lb = lower_bound_tbl<MG>(tb, t, pool, G, P);
            if (lb < t) {
                Mhe<MG> E;
                load_entry<MG>(pool, tb[lb], G, E);
                isnew = mhe_less(E, P) || mhe_less(P, E);
            } else {
                isnew = true;
            }
        }
        const int first = block_first_true(isnew, red);
        if (first == kBlock) {
            coll += c;
            i += c;
            continue;
        }
        coll += (unsigned long long)first;
        if (tid == first) {
            sP[0] = P.len;
            sP[1] = P.offset;
            #pragma unroll
            for (int g = 0; g < MG; ++g) sP[2 + g] = P.s[g];
        }
        __syncthreads();
        if (tid == 0) {
            int nc = 0;
            int64_t clo = INT64_MIN, chi = INT64_MAX;
            for (int g = 0; g < G; ++g) {
                const int64_t s = sP[2 + g];
                if (s == 0) continue;
                comps[nc].s = s;
                comps[nc].woff = gt.woff[g];
                const int64_t m = (int64_t)gt.m[g];
                const int64_t lo = s > 0 ? 1 - s : -s - m;
                const int64_t hi = s > 0 ? m - s : -s - 1;
                clo = lo > clo ? lo : clo;
                chi = hi < chi ? hi : chi;
                ++nc;
            }
            s_nc = nc;
            s_clo = clo;
            s_chi = chi;
        }
        __syncthreads();
        const int nc = s_nc;
        const int64_t clo = s_clo, chi = s_chi;
        const int64_t cmax = chain_end(+1, L, comps, nc, clo, chi, packed, ss, red);
        const int64_t cmin = chain_end(-1, L, comps, nc, clo, chi, packed, ss, red);
        if (tid == 0) {
            const uint32_t id = (uint32_t)atomicAdd(&ctr->entries, 1ull);
            Mhe<MG> E;
            E.len = cmax - cmin + L;
            E.offset = sP[1];
            E.mersize = 0;
            #pragma unroll
            for (int g = 0; g < MG; ++g) {
                const int64_t s = sP[2 + g];
                E.s[g] = s > 0 ? s + cmin : (s < 0 ? -((-s) - cmax) : 0);
            }
            int64_t* e = pool + (uint64_t)id * (uint64_t)(G + 2);
            e[0] = E.len;
            e[1] = E.offset;
            #pragma unroll
            for (int g = 0; g < MG; ++g)
                if (g < G) e[2 + g] = E.s[g];
            s_ins = lower_bound_tbl<MG>(tb, t, pool, G, E);
            s_id = id;
        }
        __syncthreads();
        const uint32_t ins = s_ins;
        for (int64_t top = t; top > (int64_t)ins; top -= kBlock) {
            const int64_t lo = top - kBlock > (int64_t)ins ? top - kBlock : (int64_t)ins;
            const int64_t j = lo + tid;
            uint32_t v = 0;
            if (j < top) v = tb[j];
            __syncthreads();
            if (j < top) tb[j + 1] = v;
            __syncthreads();
        }
        if (tid == 0) tb[ins] = s_id;
        __syncthreads();
        t += 1;
        i += (uint32_t)first + 1;
    }
    if (tid == 0) {
        tsize[b] = t;
        atomicAdd(&ctr->collisions, coll);
    }
}

__global__ void bucket_ranges_kernel(const uint32_t* __restrict__ sb, uint64_t P, uint32_t* __restrict__ bstart,
                                     uint32_t* __restrict__ bend) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P) return;
    const uint32_t b = sb[k];
    if (k == 0 || sb[k - 1] != b) bstart[b] = (uint32_t)k;
    if (k == P - 1 || sb[k + 1] != b) bend[b] = (uint32_t)(k + 1);
}

// MemHash::GetMatchList (MemHash.h:182-203): bucket-major, vector order
__global__ __launch_bounds__(kBlock) void emit_kernel(const uint32_t* __restrict__ tsize,
                                                      const uint32_t* __restrict__ obase,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ tbl,
                                                      const int64_t* __restrict__ pool, int G,
                                                      uint64_t* __restrict__ out_len, int64_t* __restrict__ out_s) {
    const uint32_t b = blockIdx.x;
    const uint32_t n = tsize[b];
    if (n == 0) return;
    const uint64_t o = obase[b];
    const uint32_t beg = bstart[b];
    for (uint32_t k = threadIdx.x; k < n; k += kBlock) {
        const uint32_t id = tbl[beg + k];
        const int64_t* e = pool + (uint64_t)id * (uint64_t)(G + 2);
        out_len[o + k] = (uint64_t)e[0];
        for (int g = 0; g < G; ++g) out_s[(o + k) * (uint64_t)G + g] = e[2 + g];
    }
}

}  // namespace

hipError_t launch_bucket_ranges(const uint32_t* sb, uint64_t P, uint32_t* bstart, uint32_t* bend, hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(bucket_ranges_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, sb, P, bstart, bend);
    return hipGetLastError();
}

template <int MG, typename View>
hipError_t launch_replay(View v, uint64_t N, const GenomeTable& gt, const MatchParams& mp, const SeedSpec& ss,
                         const uint64_t* probe_info, const uint32_t* sorted_ids, const uint32_t* bstart,
                         const uint32_t* bend, uint32_t* tbl, int64_t* pool, const uint32_t* packed,
                         uint32_t* tsize, void* ctr, hipStream_t st) {
    hipLaunchKernelGGL((replay_kernel<MG, View>), dim3(mp.table_size), dim3(kBlock), 0, st, v, N, gt, mp, ss,
                       probe_info, sorted_ids, bstart, bend, tbl, pool, packed, tsize, (DevCounters*)ctr);
    return hipGetLastError();
}

hipError_t launch_emit(const uint32_t* tsize, const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl,
                       const int64_t* pool, int G, uint32_t table_size, uint64_t* out_len, int64_t* out_s,
                       hipStream_t st) {
    hipLaunchKernelGGL(emit_kernel, dim3(table_size), dim3(kBlock), 0, st, tsize, obase, bstart, tbl, pool, G,
                       out_len, out_s);
    return hipGetLastError();
}

#define MUMS_INST_REPLAY(MG, V)                                                                                   \
    template hipError_t launch_replay<MG, V>(V, uint64_t, const GenomeTable&, const MatchParams&, const SeedSpec&, \
                                             const uint64_t*, const uint32_t*, const uint32_t*, const uint32_t*,  \
                                             uint32_t*, int64_t*, const uint32_t*, uint32_t*, void*, hipStream_t);
MUMS_INST_REPLAY(4, PairView<uint32_t>)
MUMS_INST_REPLAY(8, PairView<uint32_t>)
MUMS_INST_REPLAY(16, PairView<uint32_t>)
MUMS_INST_REPLAY(32, PairView<uint32_t>)
MUMS_INST_REPLAY(4, PairView<uint64_t>)
MUMS_INST_REPLAY(8, PairView<uint64_t>)
MUMS_INST_REPLAY(16, PairView<uint64_t>)
MUMS_INST_REPLAY(32, PairView<uint64_t>)
MUMS_INST_REPLAY(4, RecView)
MUMS_INST_REPLAY(8, RecView)
MUMS_INST_REPLAY(16, RecView)
MUMS_INST_REPLAY(32, RecView)

}  // namespace mums
