// groups.hip -- segmented equal-range scan over the merged sorted key stream (rows A7-A9).
//
// Reference: MatchFinder::SearchRange (MatchFinder.cpp:172-340) walks the G
// sorted mer lists in masked-key order and hands every group of equal masked
// keys to MemHash::EnumerateMatches (MemHash.cpp:139-162), which accepts it or
// not and builds the seed probe (HashMatch :167-187, SetDirection :189-203,
// CalculateOffset MatchHashEntry.cpp:141-160) whose hash bucket is
// ((offset % T) + T) % T (MemHash.cpp:213).
//
// Here the merged stream is the radix-sorted (ckey, index) array; a group is a
// run of equal ckey>>1.  Two passes over 4096-record tiles (one lane per record
// per round, lane-contiguous key reads): pass 1 counts accepted probes per tile,
// an exclusive scan gives tile offsets, pass 2 re-derives the probes and writes
// them compacted in ascending key order (= the reference's AddHashEntry order).
#include "match_device.h"

namespace mums {

namespace {

constexpr int kGTile = 4096;
constexpr int kGRounds = kGTile / kBlock;

template <int MG, typename K, bool kEmit>
__global__ __launch_bounds__(kBlock) void probe_pass_kernel(const K* __restrict__ skey, const uint32_t* __restrict__ sidx,
                                                            uint64_t N, GenomeTable gt, MatchParams mp, int L,
                                                            uint32_t* __restrict__ partials,
                                                            uint32_t* __restrict__ probe_head,
                                                            uint32_t* __restrict__ probe_bucket,
                                                            DevCounters* __restrict__ ctr) {
    __shared__ uint32_t wcnt[kGRounds][kBlock / 64];
    __shared__ uint32_t red[kBlock / 64][2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kGTile;
    uint32_t okmask = 0;
    uint32_t bkt[kGRounds];
    uint32_t nheads = 0, nrep = 0, nok = 0;
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        bkt[r] = 0;
        const uint64_t i = tile0 + (uint64_t)r * kBlock + threadIdx.x;
        bool ok = false;
        if (i < N) {
            const bool head = (i == 0) || ((skey[i] >> 1) != (skey[i - 1] >> 1));
            if (head) {
                Mhe<MG> P;
                uint32_t gsz = 0;
                ok = build_probe<MG, K>(skey, sidx, N, i, gt, mp, L, P, &gsz);
                if (ok) bkt[r] = bucket_of(P.offset, mp.table_size);
                ++nheads;
                nrep += gsz > (uint32_t)kRepeatLimit;
            }
        }
        okmask |= (ok ? 1u : 0u) << r;
        nok += ok;
        if (kEmit) {
            const uint64_t bal = __ballot(ok);
            if (lane == 0) wcnt[r][wv] = (uint32_t)__popcll(bal);
        }
    }
    if (!kEmit) {
        // block totals -> partials, stats
        #pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            nok += __shfl_xor(nok, d, 64);
            nheads += __shfl_xor(nheads, d, 64);
            nrep += __shfl_xor(nrep, d, 64);
        }
        if (lane == 0) { red[wv][0] = nok; red[wv][1] = nheads; }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t a = 0, b = 0;
            for (int w = 0; w < kBlock / 64; ++w) { a += red[w][0]; b += red[w][1]; }
            partials[blockIdx.x] = a;
            atomicAdd(&ctr->groups, (unsigned long long)b);
        }
        if (lane == 0 && nrep) atomicAdd(&ctr->repeat_limit, (unsigned long long)nrep);
        return;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int r = 0; r < kGRounds; ++r)
            for (int w = 0; w < kBlock / 64; ++w) { uint32_t c = wcnt[r][w]; wcnt[r][w] = acc; acc += c; }
    }
    __syncthreads();
    const uint32_t base = partials[blockIdx.x];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const bool ok = (okmask >> r) & 1u;
        const uint64_t bal = __ballot(ok);
        if (ok) {
            const uint32_t o = base + wcnt[r][wv] + (uint32_t)__popcll(bal & lt);
            probe_head[o] = (uint32_t)(tile0 + (uint64_t)r * kBlock + threadIdx.x);
            probe_bucket[o] = bkt[r];
        }
    }
}

}  // namespace

uint64_t group_tiles(uint64_t N) { return (N + kGTile - 1) / kGTile; }

template <int MG, typename K>
hipError_t launch_probe_pass(const K* skey, const uint32_t* sidx, uint64_t N, const GenomeTable& gt,
                             const MatchParams& mp, int L, uint32_t* partials, uint32_t* probe_head,
                             uint32_t* probe_bucket, void* counters, bool emit, hipStream_t st) {
    const unsigned nb = (unsigned)group_tiles(N);
    if (nb == 0) return hipSuccess;
    if (emit)
        hipLaunchKernelGGL((probe_pass_kernel<MG, K, true>), dim3(nb), dim3(kBlock), 0, st, skey, sidx, N, gt, mp, L,
                           partials, probe_head, probe_bucket, (DevCounters*)counters);
    else
        hipLaunchKernelGGL((probe_pass_kernel<MG, K, false>), dim3(nb), dim3(kBlock), 0, st, skey, sidx, N, gt, mp, L,
                           partials, probe_head, probe_bucket, (DevCounters*)counters);
    return hipGetLastError();
}

#define MUMS_INST_PROBE(MG, K)                                                                                   \
    template hipError_t launch_probe_pass<MG, K>(const K*, const uint32_t*, uint64_t, const GenomeTable&,       \
                                                 const MatchParams&, int, uint32_t*, uint32_t*, uint32_t*, void*, \
                                                 bool, hipStream_t);
MUMS_INST_PROBE(4, uint32_t)
MUMS_INST_PROBE(8, uint32_t)
MUMS_INST_PROBE(16, uint32_t)
MUMS_INST_PROBE(32, uint32_t)
MUMS_INST_PROBE(4, uint64_t)
MUMS_INST_PROBE(8, uint64_t)
MUMS_INST_PROBE(16, uint64_t)
MUMS_INST_PROBE(32, uint64_t)

}  // namespace mums
