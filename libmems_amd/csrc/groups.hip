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
// run of equal ckey>>1.  One workgroup per 4096-record tile:
//   1. lane-contiguous head detection (16 rounds), heads compacted into an LDS
//      list in stream order (ballot + per-(round, wave) counts);
//   2. every lane builds the probe of one head (no lane idles on non-heads);
//   3. accepted probes are compacted in head order into the tile's slot range
//      (a group needs >= 2 records, so <= 2048 probes per tile).
// A second kernel concatenates the tiles' slots using the scanned tile counts, so
// the probes end up in ascending key order = the reference's AddHashEntry order.
#include "match_device.h"

namespace mums {

namespace {

constexpr int kGTile = 4096;
constexpr int kGRounds = kGTile / kBlock;
constexpr int kSlots = kGTile / 2;

__device__ __forceinline__ uint32_t blk_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = v;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    #pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint32_t x = s_w[w];
        pre += (w < wv) ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

template <int MG, typename K>
__global__ __launch_bounds__(kBlock) void probe_tile_kernel(const K* __restrict__ skey, const uint32_t* __restrict__ sidx,
                                                            uint64_t N, GenomeTable gt, MatchParams mp, int L,
                                                            uint32_t* __restrict__ tile_count,
                                                            uint32_t* __restrict__ slot_head,
                                                            uint32_t* __restrict__ slot_bucket,
                                                            DevCounters* __restrict__ ctr) {
    __shared__ uint16_t heads[kGTile];
    __shared__ uint32_t okb[kGTile];        // bucket | (ok << 31) per head (bucket < 2^31)
    __shared__ uint32_t wcnt[kGRounds][kBlock / 64];
    __shared__ uint32_t s_w[kBlock / 64];
    __shared__ uint32_t s_red[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kGTile;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    // 1) heads in stream order
    uint32_t hmask = 0;
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const uint64_t i = tile0 + (uint64_t)r * kBlock + threadIdx.x;
        bool head = false;
        if (i < N) head = (i == 0) || ((skey[i] >> 1) != (skey[i - 1] >> 1));
        hmask |= (head ? 1u : 0u) << r;
        const uint64_t bal = __ballot(head);
        if (lane == 0) wcnt[r][wv] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int r = 0; r < kGRounds; ++r)
            for (int w = 0; w < kBlock / 64; ++w) { const uint32_t c = wcnt[r][w]; wcnt[r][w] = acc; acc += c; }
        s_red[0] = acc;
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
        const bool head = (hmask >> r) & 1u;
        const uint64_t bal = __ballot(head);
        if (head) heads[wcnt[r][wv] + (uint32_t)__popcll(bal & lt)] = (uint16_t)(r * kBlock + threadIdx.x);
    }
    __syncthreads();
    const uint32_t H = s_red[0];

    // 2) one probe per lane
    uint32_t nrep = 0;
    for (uint32_t j = threadIdx.x; j < H; j += kBlock) {
        Mhe<MG> P;
        uint32_t gsz = 0;
        const bool ok = build_probe<MG, K>(skey, sidx, N, tile0 + heads[j], gt, mp, L, P, &gsz);
        nrep += gsz > (uint32_t)kRepeatLimit;
        okb[j] = ok ? (0x80000000u | bucket_of(P.offset, mp.table_size)) : 0u;
    }
    if (nrep) atomicAdd(&ctr->repeat_limit, (unsigned long long)nrep);
    __syncthreads();

    // 3) compact accepted probes in head order into this tile's slots
    uint32_t base = 0;
    const uint64_t sb = (uint64_t)blockIdx.x * kSlots;
    for (uint32_t c = 0; c < H; c += kBlock) {
        const uint32_t j = c + threadIdx.x;
        const uint32_t v = j < H ? okb[j] : 0u;
        const uint32_t ok = v >> 31;
        uint32_t tot;
        const uint32_t o = blk_excl_scan(ok, s_w, &tot);
        if (ok) {
            slot_head[sb + base + o] = (uint32_t)(tile0 + heads[j]);
            slot_bucket[sb + base + o] = v & 0x7FFFFFFFu;
        }
        base += tot;
    }
    if (threadIdx.x == 0) {
        tile_count[blockIdx.x] = base;
        atomicAdd(&ctr->groups, (unsigned long long)H);
    }
}

__global__ __launch_bounds__(kBlock) void probe_compact_kernel(const uint32_t* __restrict__ tile_count,
                                                               const uint32_t* __restrict__ tile_off,
                                                               const uint32_t* __restrict__ slot_head,
                                                               const uint32_t* __restrict__ slot_bucket,
                                                               uint32_t* __restrict__ probe_head,
                                                               uint32_t* __restrict__ probe_bucket) {
    const uint32_t n = tile_count[blockIdx.x];
    const uint64_t o = tile_off[blockIdx.x];
    const uint64_t sb = (uint64_t)blockIdx.x * kSlots;
    for (uint32_t k = threadIdx.x; k < n; k += kBlock) {
        probe_head[o + k] = slot_head[sb + k];
        probe_bucket[o + k] = slot_bucket[sb + k];
    }
}

}  // namespace

uint64_t group_tiles(uint64_t N) { return (N + kGTile - 1) / kGTile; }
uint64_t group_slot_count(uint64_t N) { return group_tiles(N) * kSlots; }

template <int MG, typename K>
hipError_t launch_probe_tiles(const K* skey, const uint32_t* sidx, uint64_t N, const GenomeTable& gt,
                              const MatchParams& mp, int L, uint32_t* tile_count, uint32_t* slot_head,
                              uint32_t* slot_bucket, void* counters, hipStream_t st) {
    const unsigned nb = (unsigned)group_tiles(N);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL((probe_tile_kernel<MG, K>), dim3(nb), dim3(kBlock), 0, st, skey, sidx, N, gt, mp, L,
                       tile_count, slot_head, slot_bucket, (DevCounters*)counters);
    return hipGetLastError();
}

hipError_t launch_probe_compact(uint64_t N, const uint32_t* tile_count, const uint32_t* tile_off,
                                const uint32_t* slot_head, const uint32_t* slot_bucket, uint32_t* probe_head,
                                uint32_t* probe_bucket, hipStream_t st) {
    const unsigned nb = (unsigned)group_tiles(N);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(probe_compact_kernel, dim3(nb), dim3(kBlock), 0, st, tile_count, tile_off, slot_head,
                       slot_bucket, probe_head, probe_bucket);
    return hipGetLastError();
}

#define MUMS_INST_PROBE(MG, K)                                                                                    \
    template hipError_t launch_probe_tiles<MG, K>(const K*, const uint32_t*, uint64_t, const GenomeTable&,       \
                                                  const MatchParams&, int, uint32_t*, uint32_t*, uint32_t*, void*, \
                                                  hipStream_t);
MUMS_INST_PROBE(4, uint32_t)
MUMS_INST_PROBE(8, uint32_t)
MUMS_INST_PROBE(16, uint32_t)
MUMS_INST_PROBE(32, uint32_t)
MUMS_INST_PROBE(4, uint64_t)
MUMS_INST_PROBE(8, uint64_t)
MUMS_INST_PROBE(16, uint64_t)
MUMS_INST_PROBE(32, uint64_t)

}  // namespace mums
