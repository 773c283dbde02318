// radix_seg.hip -- segmented stable LSD radix sort of packed 8-B seed records (row A5).
//
// Records are (ckey_low << 32 | global index) and already sit in their MSD bucket
// (top B key bits, seeds.hip); each pass sorts one 8-bit digit of ckey_low inside
// every bucket.  Replaces MemorySML::Create's std::sort of 16-B bmer records
// (MemorySML.cpp:54, bmer_lessthan SortedMerList.h:311-314) and the G-way list merge
// of MatchFinder::SearchRange (MatchFinder.cpp:236-333) in one stream.
//
// Tiles of 4096 records never straddle a bucket; the digit histogram of tile tb of
// bucket b lives at hist[tfirst_b*256 + d*ntiles_b + tb], so ONE exclusive scan over
// the whole histogram yields every (bucket, digit, tile) output offset.
// Per pass: upsweep (tile digit histogram), scan, downsweep (wave64 ballot match-any
// ranking, LDS reorder, digit-run-contiguous stores).
// HBM bytes per record per pass: upsweep 8, downsweep 8 + 8.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mums_internal.h"

namespace mums {

namespace {

constexpr int kTile = kSegTile;
constexpr int kRounds = kTile / kBlock;  // 16
constexpr int kWaves = kBlock / 64;
constexpr int kDigits = 256;
#ifndef MUMS_SORT_BLOCK
#define MUMS_SORT_BLOCK 768
#endif
#ifndef MUMS_SORT_TILE
#define MUMS_SORT_TILE 9216
#endif
#ifndef MUMS_SORT_NT
#define MUMS_SORT_NT 0      // bit 0: non-temporal record loads, bit 1: non-temporal stores
#endif
#ifndef MUMS_SORT_PERSIST
#define MUMS_SORT_PERSIST 0
#endif
constexpr int kSortBlock = MUMS_SORT_BLOCK;    // threads per onesweep block
constexpr int kSortTile = MUMS_SORT_TILE;      // records per onesweep tile (longer digit runs per store)
#ifndef MUMS_OS_LATEPUB
#define MUMS_OS_LATEPUB 0   // 1: publish the tile aggregate after ranking (no early per-digit atomics)
#endif
#ifndef MUMS_OS_NEXTHIST
#define MUMS_OS_NEXTHIST 0  // 1: pass p counts the pass-(p+1) digits (the histogram read covers digit 0 only)
#endif
#ifndef MUMS_OS_FUSED
#define MUMS_OS_FUSED 0     // 1: fold lstart into the per-wave bases and the output offsets
#endif
#ifndef MUMS_LOOKBACK
#define MUMS_LOOKBACK 4
#endif
#ifndef MUMS_OS_CTILES
#define MUMS_OS_CTILES 0    // 1: descriptors copied into claim order (one load per claim): measured 1.3 % slower per pass
#endif

#ifndef MUMS_OS_STATS
#define MUMS_OS_STATS 0     // 1 (development build): per-phase wall-clock sums of the onesweep blocks
#endif
#if MUMS_OS_STATS
// per claimed tile: 8 s_memrealtime stamps (100 MHz) of its block's phases, then the block id
// (plain stores: the host reduces them after every pass)
__device__ unsigned long long* g_os_stats;
#define OS_STAMP(k)                                                                  \
    do {                                                                             \
        if (tid == 0) ts[k] = __builtin_amdgcn_s_memrealtime();                      \
    } while (0)
#else
#define OS_STAMP(k) \
    do {            \
    } while (0)
#endif

constexpr int kLookback = MUMS_LOOKBACK;       // predecessor statuses fetched per look-back step
inline uint64_t ub_status(uint64_t ub, int npass) { return ub * kDigits * (uint64_t)npass; }

// bucket starts from the scanned MSD histogram: bstart[b] = scanned[b * T], bstart[nb] = n
__global__ void bucket_starts_kernel(const uint32_t* __restrict__ scanned, uint32_t T, int nb, uint64_t n,
                                     uint32_t* __restrict__ bstart, uint32_t* __restrict__ ntb) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    const uint64_t s = (b == nb) ? n : (uint64_t)scanned[(uint64_t)b * T];
    bstart[b] = (uint32_t)s;
    if (ntb && b < nb) {
        const uint64_t e = (b + 1 == nb) ? n : (uint64_t)scanned[(uint64_t)(b + 1) * T];
        ntb[b] = (uint32_t)((e - s + kTile - 1) / kTile);
    }
}

// tiles per bucket from bucket starts (tfirst[nb] = 0 so one scan gives the total)
__global__ void ntb_from_starts_kernel(const uint32_t* __restrict__ bstart, int nb, uint32_t tile,
                                       uint32_t* __restrict__ ntb) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    ntb[b] = (b == nb) ? 0u : (uint32_t)(((uint64_t)bstart[b + 1] - bstart[b] + tile - 1) / tile);
}

__global__ void single_bucket_kernel(uint64_t n, uint32_t* __restrict__ bstart) {
    if (threadIdx.x == 0) {
        bstart[0] = 0;
        bstart[1] = (uint32_t)n;
    }
}

__global__ void tiles_kernel(const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ tfirst, int nb,
                             uint64_t ub, uint32_t tile, SegTile* __restrict__ tiles,
                             uint32_t* __restrict__ ntiles_out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ub) return;
    const uint32_t total = tfirst[nb];
    if (t == 0) *ntiles_out = total;
    SegTile d{};
    if (t < total) {
        int lo = 0, hi = nb - 1;  // last bucket b with tfirst[b] <= t (buckets with 0 tiles skipped)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (tfirst[mid] <= t) lo = mid;
            else hi = mid - 1;
        }
        while (lo + 1 < nb && tfirst[lo + 1] <= t) ++lo;
        const uint32_t tb = (uint32_t)(t - tfirst[lo]);
        const uint32_t ntb = tfirst[lo + 1] - tfirst[lo];
        d.bstart = bstart[lo];
        d.bend = bstart[lo + 1];
        d.start = d.bstart + (uint64_t)tb * tile;
        const uint64_t rem = d.bend - d.start;
        d.count = (uint32_t)(rem < (uint64_t)tile ? rem : (uint64_t)tile);
        d.hbase = tfirst[lo] * kDigits;
        d.ntb = ntb;
        d.tb = tb;
        d.bucket = (uint32_t)lo;
    } else {
        d.count = 0;
        d.hbase = (uint32_t)(t * kDigits);
        d.ntb = 1;
        d.tb = 0;
    }
    tiles[t] = d;
}

// Claim order of the onesweep passes.  A tile waits only on the preceding tiles of
// its own MSD bucket, so the buckets are independent look-back chains.  Claiming
// tiles bucket-major would put every resident block on ONE chain (whose inclusive
// prefix advances one look-back round trip at a time); claiming them in
// (tile-in-bucket, bucket) order spreads the resident blocks over all chains.  A
// tile's predecessor still precedes it in this order, so every tile a block waits
// on was claimed earlier: forward progress is kept.
// pos(k, b) = sum_b' min(ntb_b', k) + #{b' < b : ntb_b' > k}.
__global__ __launch_bounds__(256) void claim_order_kernel(const uint32_t* __restrict__ tfirst, int nb, uint64_t ub,
                                                          SegTile* __restrict__ tiles) {
    __shared__ uint32_t s_n[1 << kMaxSegBucketBits];
    for (int b = threadIdx.x; b < nb; b += blockDim.x) s_n[b] = tfirst[b + 1] - tfirst[b];
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ub) return;
    const uint32_t total = tfirst[nb];
    if (t >= total) { tiles[t].order = (uint32_t)t; return; }
    const SegTile d = tiles[t];
    const uint32_t k = d.tb;
    uint32_t pos = 0;
    for (int b = 0; b < nb; ++b) {
        const uint32_t n = s_n[b];
        pos += (n < k ? n : k) + ((uint32_t)b < d.bucket && n > k ? 1u : 0u);
    }
    tiles[pos].order = (uint32_t)t;
}

// ctiles[c] = the descriptor of the c-th claimed tile (ctiles[c].order = its tile index): a
// claiming block then reads its tile with one load after the claim
__global__ __launch_bounds__(256) void claim_tiles_kernel(const SegTile* __restrict__ tiles, uint64_t ub,
                                                          SegTile* __restrict__ ctiles) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ub) return;
    const uint32_t t = tiles[c].order;
    SegTile d = tiles[t];
    d.order = t;
    ctiles[c] = d;
}

// XCD-grouped claim queues (default; MUMS_DEV_OS_XCD=0 turns them off): bucket b's tiles form queue
// b % 8, in (tile-in-bucket, bucket) order inside the queue; blocks b and b + 8 share an XCD
// (round-robin dispatch, MI355X_MICROARCH.md: a speed-only affinity), so a block claims from
// queue blockIdx % 8 first: consecutive tiles of a bucket -- whose digit runs abut in the
// output -- run on one XCD and their partial cache lines can merge in its L2.  A block whose
// queue is empty takes from the next queue: a tile's predecessors precede it in its queue, so
// they were claimed by running blocks (forward progress as in claim_order_kernel).
// xq[0..7] queue lengths, xq[8..16] queue offsets, xq[32 + off + i] the i-th tile of a queue;
// xd[off + i] its claim descriptor {tile, first record, count | bucket << 16, tile in bucket}: a
// claiming block reads its tile with ONE load after the claim's atomic (not the tile id, then
// the tile's SegTile: two dependent round trips at the start of every tile)
__global__ __launch_bounds__(256) void xcd_order_kernel(const uint32_t* __restrict__ tfirst, int nb, uint64_t ub,
                                                        const SegTile* __restrict__ tiles, uint32_t* __restrict__ xq,
                                                        uint4* __restrict__ xd) {
    __shared__ uint32_t s_n[1 << kMaxSegBucketBits];
    __shared__ uint32_t s_off[9];
    for (int b = threadIdx.x; b < nb; b += blockDim.x) s_n[b] = tfirst[b + 1] - tfirst[b];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t o = 0;
        for (int x = 0; x < 8; ++x) {
            uint32_t len = 0;
            for (int b = x; b < nb; b += 8) len += s_n[b];
            s_off[x] = o;
            if (blockIdx.x == 0) {
                xq[x] = len;
                xq[8 + x] = o;
            }
            o += len;
        }
        s_off[8] = o;
        if (blockIdx.x == 0) xq[16] = o;
    }
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ub || t >= tfirst[nb]) return;
    const SegTile d = tiles[t];
    const uint32_t k = d.tb;
    const int x = (int)(d.bucket & 7u);
    uint32_t pos = 0;
    for (int b = x; b < nb; b += 8) {
        const uint32_t n = s_n[b];
        pos += (n < k ? n : k) + ((uint32_t)b < d.bucket && n > k ? 1u : 0u);
    }
    xq[32 + s_off[x] + pos] = (uint32_t)t;
    xd[s_off[x] + pos] = make_uint4((uint32_t)t, (uint32_t)d.start, d.count | (d.bucket << 16), d.tb);
}

__global__ __launch_bounds__(kBlock) void seg_upsweep(const uint64_t* __restrict__ rec, const SegTile* __restrict__ tiles,
                                                      int shift, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kWaves][kDigits];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const SegTile d = tiles[blockIdx.x];
    for (int i = threadIdx.x; i < kWaves * kDigits; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t b0 = wv * (kTile / kWaves);
    #pragma unroll 4
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = b0 + r * 64 + lane;
        if (q < d.count) atomicAdd(&h[wv][(uint32_t)(rec[d.start + q] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    const int t = threadIdx.x;
    uint32_t s = 0;
    #pragma unroll
    for (int w = 0; w < kWaves; ++w) s += h[w][t];
    hist[(uint64_t)d.hbase + (uint64_t)t * d.ntb + d.tb] = s;
}

__global__ __launch_bounds__(kBlock) void seg_downsweep(const uint64_t* __restrict__ rin,
                                                        const SegTile* __restrict__ tiles, int shift,
                                                        const uint32_t* __restrict__ hist,
                                                        uint64_t* __restrict__ rout) {
    __shared__ uint64_t srec[kTile];
    __shared__ uint32_t wcnt[kWaves][kDigits];
    __shared__ uint32_t lstart[kDigits];
    __shared__ uint32_t gofs[kDigits];
    __shared__ uint32_t s_w[kWaves];
    const SegTile d = tiles[blockIdx.x];
    if (d.count == 0) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * kDigits; i += kBlock) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t q0 = wv * (kTile / kWaves);
    uint64_t key[kRounds];
    uint32_t rank[kRounds];
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
    }
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        const bool valid = q < d.count;
        const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<8>(dg, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][dg];
        if (valid && rk == 0) wcnt[wv][dg] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();
    {
        const int t = threadIdx.x;  // digit
        uint32_t acc = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) { const uint32_t c = wcnt[w][t]; wcnt[w][t] = acc; acc += c; }
        uint32_t v = acc;
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t x = __shfl_up(v, dd, 64);
            if (lane >= dd) v += x;
        }
        if (lane == 63) s_w[wv] = v;
        __syncthreads();
        uint32_t wpre = 0;
        #pragma unroll
        for (int w = 0; w < kWaves; ++w) wpre += (w < wv) ? s_w[w] : 0u;
        lstart[t] = wpre + v - acc;
        gofs[t] = hist[(uint64_t)d.hbase + (uint64_t)t * d.ntb + d.tb];
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        if (q < d.count) {
            const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
            srec[lstart[dg] + wcnt[wv][dg] + rank[r]] = key[r];
        }
    }
    __syncthreads();
    #pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t s = threadIdx.x + r * kBlock;
        if (s < d.count) {
            const uint64_t k = srec[s];
            const uint32_t dg = (uint32_t)(k >> shift) & 0xFFu;
            rout[(uint64_t)gofs[dg] + (s - lstart[dg])] = k;
        }
    }
}


// ---------------------------------------------------------------------------------
// Onesweep variant.  ghist[(b * npass + p) * 256 + d] = records of bucket b whose
// pass-p digit is d (one read of the data for all passes); dbase = per-bucket
// exclusive digit offsets + bucket start.  Each pass is then ONE launch: a tile
// ranks its records, publishes its per-digit count, looks back over the preceding
// tiles of its bucket for the exclusive prefix, and scatters.  Status words are one
// 32-bit {flag:2, count:30} granule per (tile, digit), stored and polled with
// agent-scope relaxed atomics (MI355X_MICROARCH.md "Valid forms": the data is the
// flag).  Tile ids come from an atomic counter in launch order, so every tile a
// block waits on is already resident: forward progress without a grid barrier.
// Spins are bounded; a timeout sets err bit 1 instead of hanging the device.
constexpr uint32_t kFlagAgg = 1u << 30;
constexpr uint32_t kFlagInc = 2u << 30;
constexpr uint32_t kValMask = (1u << 30) - 1;
constexpr int kGhistTilesPerBlock = 16;
#ifndef MUMS_GHIST_BATCH
#define MUMS_GHIST_BATCH 8
#endif
constexpr int kGhistBatch = MUMS_GHIST_BATCH;   // records per lane loaded as one batch

__global__ __launch_bounds__(kBlock) void seg_ghist_kernel(const uint64_t* __restrict__ rec,
                                                           const SegTile* __restrict__ tiles, uint64_t ntiles_ub,
                                                           int npass, uint32_t* __restrict__ ghist, int key_shift,
                                                           int nh, int runs) {
    __shared__ uint32_t h[4][kDigits];
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * kGhistTilesPerBlock;
    uint32_t cur_b = 0xFFFFFFFFu;
    for (int i = tid; i < 4 * kDigits; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    for (int k = 0; k < kGhistTilesPerBlock; ++k) {
        const uint64_t t = t0 + k;
        if (t >= ntiles_ub) break;
        const SegTile d = tiles[t];
        if (d.count == 0) break;
        if (d.bucket != cur_b) {
            if (cur_b != 0xFFFFFFFFu) {
                __syncthreads();
                for (int p = 0; p < nh; ++p) {
                    const uint32_t v = h[p][tid];
                    if (v) atomicAdd(&ghist[((uint64_t)cur_b * npass + p) * kDigits + tid], v);
                    h[p][tid] = 0;
                }
                __syncthreads();
            }
            cur_b = d.bucket;
        }
        // kGhistBatch loads in flight per lane before the LDS counting
        for (uint32_t q0 = 0; q0 < d.count; q0 += kBlock * kGhistBatch) {
            uint64_t kk[kGhistBatch];
            #pragma unroll
            for (int u = 0; u < kGhistBatch; ++u) {
                const uint32_t q = q0 + u * kBlock + tid;
                kk[u] = q < d.count ? rec[d.start + q] : 0ull;
            }
            if (runs) {   // uniform: runs of equal digits in neighbouring lanes add once per run
                const int lane = tid & 63;
                #pragma unroll
                for (int u = 0; u < kGhistBatch; ++u) {
                    const bool valid = q0 + u * kBlock + tid < d.count;   // a prefix of the wave's lanes
                    const uint64_t vm = __ballot(valid);
                    const uint64_t key = kk[u] >> key_shift;
                    for (int p = 0; p < nh; ++p) {
                        const uint32_t dg = (uint32_t)(key >> (8 * p)) & 0xFFu;
                        const uint32_t pd = __shfl_up(dg, 1, 64);
                        const bool head = valid && (lane == 0 || pd != dg);
                        const uint64_t hm = __ballot(head);
                        if (head) {
                            const uint64_t above = lane == 63 ? 0ull : (hm & (~0ull << (lane + 1)));
                            const int nxt = above ? __builtin_ctzll(above) : __popcll(vm);
                            atomicAdd(&h[p][dg], (uint32_t)(nxt - lane));
                        }
                    }
                }
            } else {
                #pragma unroll
                for (int u = 0; u < kGhistBatch; ++u) {
                    if (q0 + u * kBlock + tid >= d.count) break;
                    const uint64_t key = kk[u] >> key_shift;
                    for (int p = 0; p < nh; ++p) atomicAdd(&h[p][(uint32_t)(key >> (8 * p)) & 0xFFu], 1u);
                }
            }
        }
    }
    __syncthreads();
    if (cur_b != 0xFFFFFFFFu)
        for (int p = 0; p < nh; ++p) {
            const uint32_t v = h[p][tid];
            if (v) atomicAdd(&ghist[((uint64_t)cur_b * npass + p) * kDigits + tid], v);
        }
}

// one block per (bucket, pass): dbase = bstart[b] + exclusive scan over digits
__global__ __launch_bounds__(kBlock) void seg_dbase_kernel(const uint32_t* __restrict__ ghist,
                                                           const uint32_t* __restrict__ bstart, int npass,
                                                           uint32_t* __restrict__ dbase, int pass) {
    __shared__ uint32_t s_w[kWaves];
    // pass < 0: one block per (bucket, pass); else one block per bucket for that pass
    const uint64_t bp = pass < 0 ? (uint64_t)blockIdx.x : (uint64_t)blockIdx.x * npass + pass;
    const uint32_t b = (uint32_t)(bp / npass);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t v = ghist[bp * kDigits + threadIdx.x];
    uint32_t inc = v;
    #pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t x = __shfl_up(inc, dd, 64);
        if (lane >= dd) inc += x;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
    #pragma unroll
    for (int w = 0; w < kWaves; ++w) pre += (w < wv) ? s_w[w] : 0u;
    dbase[bp * kDigits + threadIdx.x] = bstart[b] + pre + inc - v;
}

template <int kIPT>
__device__ __forceinline__ void onesweep_load(const uint64_t* __restrict__ rin, const SegTile& d, uint32_t q0, int lane,
                                              uint64_t (&key)[kIPT]) {
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t q = q0 + r * 64 + lane;
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
    }
}

// One onesweep pass; each block claims one tile from an atomic counter (claim
// order = tiles[c].order, see claim_order_kernel), so every tile it waits on was
// claimed earlier by a resident block.  OB threads x kIPT records per tile; the first
// 256 threads also own one digit each for the look-back and the digit starts.
// kAlias: the per-wave digit counts live in the record exchange buffer (every lane folds
// its slot base into its ranks before the exchange), so a tile costs kT * 8 B + 4 KB of LDS.
// kGath (the line sort's last pass): instead of record k, gout[o] = low 32 bits of
// gsrc[low 32 bits of k] -- the permutation gather of the caller, done at the store
template <int OB, int kIPT, bool kAlias = false, bool kLate = false, bool kGath = false>
__global__ __launch_bounds__(OB) void seg_onesweep_kernel(const uint64_t* __restrict__ rin,
                                                          uint64_t* __restrict__ rout,
                                                          const SegTile* __restrict__ tiles, uint32_t nclaims,
                                                          int shift, int pass, int npass,
                                                          const uint32_t* __restrict__ dbase, uint32_t* status,
                                                          uint32_t* tile_counter, uint32_t* err,
                                                          uint32_t* __restrict__ ghist_next,
                                                          const uint32_t* __restrict__ xq,
                                                          const uint64_t* __restrict__ gsrc = nullptr,
                                                          uint32_t* __restrict__ gout = nullptr,
                                                          const uint4* __restrict__ xd = nullptr) {
    constexpr int kT = kIPT * OB;
    constexpr bool late = MUMS_OS_LATEPUB || kLate;
    constexpr int kW = OB / 64;
    static_assert(OB >= kDigits, "one thread per digit");
    static_assert(!kAlias || kW * kDigits * 4 <= kT * 8, "counts fit in the exchange buffer");
    __shared__ uint64_t srec[kT];
    __shared__ uint32_t wcnt_own[kAlias ? 1 : kW][kDigits];
    uint32_t (*wcnt)[kDigits] = kAlias ? reinterpret_cast<uint32_t (*)[kDigits]>(srec) : wcnt_own;
    __shared__ uint32_t lstart[kDigits];
    __shared__ uint32_t gofs[kDigits];
    __shared__ uint32_t s_w[kDigits / 64];
    __shared__ uint32_t s_tile;
    __shared__ uint32_t hcnt[kDigits];
    __shared__ uint32_t hnext[kDigits];   // next pass's digit counts (ghist_next != null)
    __shared__ uint4 s_desc;              // the claimed tile's descriptor (xd)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#if MUMS_OS_STATS
    unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    OS_STAMP(0);
    if (tid == 0) {
        if (xq) {   // XCD-grouped queues (xcd_order_kernel): s_tile = the tile itself
            uint32_t tt = 0xFFFFFFFFu;
            const uint32_t x = blockIdx.x & 7u;
            for (uint32_t a = 0; a < 8; ++a) {
                const uint32_t q = (x + a) & 7u;
                const uint32_t qo = xq[8 + q], ql = xq[q];   // issued with the atomic
                const uint32_t cc = atomicAdd(tile_counter + q, 1u);
                if (cc < ql) {
                    if (xd) {
                        const uint4 dd = xd[qo + cc];
                        s_desc = dd;
                        tt = dd.x;
                    } else {
                        tt = xq[32 + qo + cc];
                    }
                    break;
                }
            }
            s_tile = tt;
        } else {
            s_tile = atomicAdd(tile_counter, 1u);
        }
    }
    for (int i = tid; i < kW * kDigits; i += OB) (&wcnt[0][0])[i] = 0;
    if (tid < kDigits) { hcnt[tid] = 0; hnext[tid] = 0; }
    __syncthreads();
    const uint32_t c = __builtin_amdgcn_readfirstlane(s_tile);   // uniform: scalar descriptor loads
    if (xq ? c == 0xFFFFFFFFu : c >= nclaims) return;
#if MUMS_OS_CTILES
    const SegTile d = tiles[c];   // claim-ordered copy (claim_tiles_kernel)
    const uint32_t t = __builtin_amdgcn_readfirstlane(d.order);
#else
    const uint32_t t = xq ? c : __builtin_amdgcn_readfirstlane(tiles[c].order);
    SegTile d{};
    if (xd) {   // uniform: the descriptor the claim loaded
        const uint4 dd = s_desc;
        d.start = __builtin_amdgcn_readfirstlane(dd.y);
        d.count = __builtin_amdgcn_readfirstlane(dd.z & 0xFFFFu);
        d.bucket = __builtin_amdgcn_readfirstlane(dd.z >> 16);
        d.tb = __builtin_amdgcn_readfirstlane(dd.w);
    } else {
        d = tiles[t];
    }
#endif
    if (d.count == 0) return;
    OS_STAMP(1);
    const uint32_t q0 = wv * (kT / kW);
    uint64_t key[kIPT];
    uint32_t rank[kIPT];
    auto qof = [&](int r) -> uint32_t { return q0 + (uint32_t)r * 64u + (uint32_t)lane; };
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t q = qof(r);
#if MUMS_SORT_NT & 1
        key[r] = q < d.count ? __builtin_nontemporal_load(rin + d.start + q) : 0ull;   // read once per pass
#else
        key[r] = q < d.count ? rin[d.start + q] : 0ull;
#endif
    }
    if constexpr (!late) {
        // publish this tile's per-digit counts as soon as the keys are in: successors'
        // look-backs then rarely find an unpublished predecessor.  (Late: after the ranking,
        // from its per-wave counts -- for keys in runs of equal digits, whose per-record LDS
        // atomics here would serialise.)
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = qof(r);
            if (q < d.count) atomicAdd(&hcnt[(uint32_t)(key[r] >> shift) & 0xFFu], 1u);
        }
        __syncthreads();
        OS_STAMP(2);
        if (d.tb != 0 && tid < kDigits)
            __hip_atomic_store(status + (uint64_t)t * kDigits + tid, kFlagAgg | hcnt[tid], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (ghist_next) {   // uniform: the next pass's histogram rides on this pass's read
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = qof(r);
            if (q < d.count) atomicAdd(&hnext[(uint32_t)(key[r] >> (shift + 8)) & 0xFFu], 1u);
        }
    }
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t q = qof(r);
        const bool valid = q < d.count;
        const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
        uint32_t tot;
        const uint32_t rk = wave_match_rank<8>(dg, valid, &tot);
        uint32_t old = 0;
        if (valid) old = wcnt[wv][dg];
        if (valid && rk == 0) wcnt[wv][dg] = old + tot;
        rank[r] = old + rk;
    }
    __syncthreads();
    OS_STAMP(3);
    uint32_t v = 0, acc = 0;
    if (tid < kDigits) {
        const int dg = tid;  // digit
        #pragma unroll
        for (int w = 0; w < kW; ++w) { const uint32_t x = wcnt[w][dg]; wcnt[w][dg] = acc; acc += x; }
        // look back over the bucket's preceding tiles, then publish the inclusive prefix
        uint32_t* st = status + (uint64_t)t * kDigits + dg;
        if (late && d.tb != 0) __hip_atomic_store(st, kFlagAgg | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t prefix = 0;
        if (d.tb == 0) {
            __hip_atomic_store(st, kFlagInc | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            // windowed look-back: kLookback predecessor statuses per step as one batch of
            // independent loads; tiles before the bucket's first tile are never read
            // (the first tile always publishes an inclusive prefix).
            const int64_t tfirst = (int64_t)t - (int64_t)d.tb;
            int64_t j = (int64_t)t - 1;
            uint32_t spins = 0;
            bool done = false;
            while (!done) {
                uint32_t sv[kLookback];
                #pragma unroll
                for (int k = 0; k < kLookback; ++k)
                    sv[k] = (j - k >= tfirst) ? __hip_atomic_load(status + (uint64_t)(j - k) * kDigits + dg,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : kFlagInc;
                int used = 0;
                bool stall = false;
                #pragma unroll
                for (int k = 0; k < kLookback; ++k) {
                    if (done || stall) continue;
                    const uint32_t sx = sv[k];
                    if ((sx >> 30) == 0u) { stall = true; continue; }
                    prefix += sx & kValMask;
                    ++used;
                    if ((sx & kFlagInc) != 0u) done = true;
                }
                j -= used;
                if (stall && !done) {
                    if (++spins > (1u << 24)) { atomicOr(err, 2u); break; }
                    if (spins < 8) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(8);
                }
            }
            __hip_atomic_store(st, kFlagInc | ((prefix + acc) & kValMask), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        gofs[dg] = dbase[((uint64_t)d.bucket * npass + pass) * kDigits + dg] + prefix;
        // block-local digit starts
        v = acc;
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t x = __shfl_up(v, dd, 64);
            if (lane >= dd) v += x;
        }
        if (lane == 63) s_w[wv] = v;
    }
    __syncthreads();
    OS_STAMP(4);
    if (tid < kDigits) {
        uint32_t wpre = 0;
        #pragma unroll
        for (int w = 0; w < kDigits / 64; ++w) wpre += (w < wv) ? s_w[w] : 0u;
        lstart[tid] = wpre + v - acc;
#if MUMS_OS_FUSED
        // one LDS read per record in each scatter: per-wave LDS slot base and the
        // tile-slot -> output offset of every digit
        const uint32_t ls = wpre + v - acc;
        #pragma unroll
        for (int w = 0; w < kW; ++w) wcnt[w][tid] += ls;
        gofs[tid] -= ls;
#endif
    }
    __syncthreads();
    if constexpr (kAlias) {   // slots first: the exchange overwrites the counts
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
#if MUMS_OS_FUSED
            rank[r] += wcnt[wv][dg];
#else
            rank[r] += lstart[dg] + wcnt[wv][dg];
#endif
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kIPT; ++r)
            if (qof(r) < d.count) srec[rank[r]] = key[r];
    } else {
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t q = qof(r);
        if (q < d.count) {
            const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
#if MUMS_OS_FUSED
            srec[wcnt[wv][dg] + rank[r]] = key[r];
#else
            srec[lstart[dg] + wcnt[wv][dg] + rank[r]] = key[r];
#endif
        }
    }
    }
    __syncthreads();
    OS_STAMP(5);
    #pragma unroll
    for (int r = 0; r < kIPT; ++r) {
        const uint32_t sidx = tid + r * OB;
        if (sidx < d.count) {
            const uint64_t k = srec[sidx];
            const uint32_t dg = (uint32_t)(k >> shift) & 0xFFu;
#if MUMS_OS_FUSED
            const uint64_t o = (uint64_t)(uint32_t)(gofs[dg] + sidx);   // gofs holds out offset - lstart (mod 2^32)
#else
            const uint64_t o = (uint64_t)gofs[dg] + (sidx - lstart[dg]);
#endif
            if constexpr (kGath) {
                gout[o] = (uint32_t)gsrc[(uint32_t)k];
            } else {
#if MUMS_SORT_NT & 2
                __builtin_nontemporal_store(k, rout + o);
#else
                rout[o] = k;
#endif
            }
        }
    }
    if (ghist_next && tid < kDigits) {   // hnext complete: barriers since its atomics
        const uint32_t c = hnext[tid];
        if (c) atomicAdd(&ghist_next[((uint64_t)d.bucket * npass + pass + 1) * kDigits + tid], c);
    }
#if MUMS_OS_STATS
    OS_STAMP(6);
    __builtin_amdgcn_s_waitcnt(0);   // this wave's stores retired
    OS_STAMP(7);
    if (tid == 0) {
        unsigned long long* o = g_os_stats + (uint64_t)t * 10;
        for (int k = 0; k < 8; ++k) o[k] = ts[k];
        o[8] = blockIdx.x;
        o[9] = 1;
    }
#endif
}

// Persistent onesweep pass: a resident grid of blocks, each claiming tiles in claim
// order from the counter until none is left.  The next tile's records are loaded
// right after the current tile's look-back, so their HBM latency overlaps the current
// tile's LDS reorder and stores.  A block holds at most its current tile and the one
// after it; the earliest unfinished claim is always a current tile whose predecessors
// are all finished, so the look-back chain always progresses.
template <int OB, int kIPT>
__global__ __launch_bounds__(OB) __attribute__((amdgpu_waves_per_eu(4))) void seg_onesweep_persist_kernel(const uint64_t* __restrict__ rin,
                                                                  uint64_t* __restrict__ rout,
                                                                  const SegTile* __restrict__ tiles,
                                                                  uint32_t nclaims, int shift, int pass, int npass,
                                                                  const uint32_t* __restrict__ dbase,
                                                                  uint32_t* status, uint32_t* tile_counter,
                                                                  uint32_t* err) {
    constexpr int kT = kIPT * OB;
    constexpr int kW = OB / 64;
    static_assert(OB >= kDigits, "one thread per digit");
    __shared__ uint64_t srec[kT];
    __shared__ uint32_t wcnt[kW][kDigits];
    __shared__ uint32_t lstart[kDigits];
    __shared__ uint32_t gofs[kDigits];
    __shared__ uint32_t s_w[kDigits / 64];
    __shared__ uint32_t s_tile[2];
    __shared__ uint32_t hcnt[kDigits];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t q0 = wv * (kT / kW);
    if (tid == 0) s_tile[0] = atomicAdd(tile_counter, 1u);
    __syncthreads();
    uint32_t c = __builtin_amdgcn_readfirstlane(s_tile[0]);
    uint64_t key[kIPT];
    uint32_t rank[kIPT];
    SegTile d{};
    uint32_t t = 0;
    if (c < nclaims) {
        t = __builtin_amdgcn_readfirstlane(tiles[c].order);
        d = tiles[t];
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            key[r] = q < d.count ? rin[d.start + q] : 0ull;
        }
    }
    int par = 0;
    while (c < nclaims) {
        // claim the next tile now (its id is needed before the prefetch below)
        if (tid == 0) s_tile[par ^ 1] = atomicAdd(tile_counter, 1u);
        for (int i = tid; i < kW * kDigits; i += OB) (&wcnt[0][0])[i] = 0;
        if (tid < kDigits) hcnt[tid] = 0;
        __syncthreads();
        const uint32_t cn = __builtin_amdgcn_readfirstlane(s_tile[par ^ 1]);
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            if (q < d.count) atomicAdd(&hcnt[(uint32_t)(key[r] >> shift) & 0xFFu], 1u);
        }
        __syncthreads();
        if (d.tb != 0 && tid < kDigits)
            __hip_atomic_store(status + (uint64_t)t * kDigits + tid, kFlagAgg | hcnt[tid], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            const bool valid = q < d.count;
            const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
            uint32_t tot;
            const uint32_t rk = wave_match_rank<8>(dg, valid, &tot);
            uint32_t old = 0;
            if (valid) old = wcnt[wv][dg];
            if (valid && rk == 0) wcnt[wv][dg] = old + tot;
            rank[r] = old + rk;
        }
        __syncthreads();
        uint32_t v = 0, acc = 0;
        if (tid < kDigits) {
            const int dg = tid;
            #pragma unroll
            for (int w = 0; w < kW; ++w) { const uint32_t x = wcnt[w][dg]; wcnt[w][dg] = acc; acc += x; }
            uint32_t* st = status + (uint64_t)t * kDigits + dg;
            uint32_t prefix = 0;
            if (d.tb == 0) {
                __hip_atomic_store(st, kFlagInc | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const int64_t tfirst = (int64_t)t - (int64_t)d.tb;
                int64_t j = (int64_t)t - 1;
                uint32_t spins = 0;
                bool done = false;
                while (!done) {
                    uint32_t sv[kLookback];
                    #pragma unroll
                    for (int k = 0; k < kLookback; ++k)
                        sv[k] = (j - k >= tfirst) ? __hip_atomic_load(status + (uint64_t)(j - k) * kDigits + dg,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : kFlagInc;
                    int used = 0;
                    bool stall = false;
                    #pragma unroll
                    for (int k = 0; k < kLookback; ++k) {
                        if (done || stall) continue;
                        const uint32_t sx = sv[k];
                        if ((sx >> 30) == 0u) { stall = true; continue; }
                        prefix += sx & kValMask;
                        ++used;
                        if ((sx & kFlagInc) != 0u) done = true;
                    }
                    j -= used;
                    if (stall && !done) {
                        if (++spins > (1u << 24)) { atomicOr(err, 2u); break; }
                        if (spins < 8) __builtin_amdgcn_s_sleep(1);
                        else __builtin_amdgcn_s_sleep(8);
                    }
                }
                __hip_atomic_store(st, kFlagInc | ((prefix + acc) & kValMask), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            gofs[dg] = dbase[((uint64_t)d.bucket * npass + pass) * kDigits + dg] + prefix;
            v = acc;
            #pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t x = __shfl_up(v, dd, 64);
                if (lane >= dd) v += x;
            }
            if (lane == 63) s_w[wv] = v;
        }
        __syncthreads();
        if (tid < kDigits) {
            uint32_t wpre = 0;
            #pragma unroll
            for (int w = 0; w < kDigits / 64; ++w) wpre += (w < wv) ? s_w[w] : 0u;
            lstart[tid] = wpre + v - acc;
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t q = q0 + r * 64 + lane;
            if (q < d.count) {
                const uint32_t dg = (uint32_t)(key[r] >> shift) & 0xFFu;
                srec[lstart[dg] + wcnt[wv][dg] + rank[r]] = key[r];
            }
        }
        // prefetch the next tile's records into the key registers (now free)
        SegTile dn{};
        uint32_t tn = 0;
        if (cn < nclaims) {
            tn = __builtin_amdgcn_readfirstlane(tiles[cn].order);
            dn = tiles[tn];
            #pragma unroll
            for (int r = 0; r < kIPT; ++r) {
                const uint32_t q = q0 + r * 64 + lane;
                key[r] = q < dn.count ? rin[dn.start + q] : 0ull;
            }
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < kIPT; ++r) {
            const uint32_t sidx = tid + r * OB;
            if (sidx < d.count) {
                const uint64_t k = srec[sidx];
                const uint32_t dg = (uint32_t)(k >> shift) & 0xFFu;
                rout[(uint64_t)gofs[dg] + (sidx - lstart[dg])] = k;
            }
        }
        __syncthreads();   // srec / gofs / lstart are rewritten by the next tile
        c = cn;
        d = dn;
        t = tn;
        par ^= 1;
    }
}

// ---------------------------------------------------------------------------------
// Segment fix-up: the last step of the onesweep sort, in place of the pass over the
// lowest key digit.  After the passes over the higher digits the stream is sorted by
// (bucket, key bits above the lowest digit) and, inside such a "segment", by global
// index.  Stable-sorting every segment by its lowest digit completes the order
// (= the full LSD sort's).  A segment is mostly the copies of ONE seed key in the G
// genomes; it needs work only when it holds several keys whose digits decrease
// somewhere ("dirty").  So the step is one coalesced read of the stream plus sparse
// in-place writes, instead of a 16-B/record pass.
//
// The digit compared is (x >> dshift) & dmask and the segment prefix (x >> pshift) &
// pmask.  Under the default tolerances (repeat_tol 0, enum_tol 1) the probe of a masked
// key group does not depend on the order of its records (one record per genome), so the
// parity bit (key bit 0: the seed's orientation) is left out of the digit: the stream is
// then ordered by the masked key, the grouping key of SearchRange, and only segments
// holding two masked keys out of order are dirty.  seg_parity_fix restores the exact
// order (parity digit inside each masked-key group) for consumers that need it.
//
// A block owns the segments starting in its tile and sees kSfX records past the tile.
// Per window position the segment starts and the dirty pairs are ballot bitmaps in LDS;
// the lane holding the first dirty pair of an owned segment finds the segment's bounds
// in the bitmaps and lists its records; then one lane per listed record computes its
// stable rank inside the segment (segments of <= 64 records) and stores it.  Longer
// dirty segments and the owned segment running past the window go to the big list
// (segfix_big_kernel).  Writes stay inside owned segments, and other blocks read only
// the prefix of those records (the same for every record of a segment), so the
// in-place rewrite races with nothing.
constexpr int kSfTile = 2048;
constexpr int kSfX = 64;
constexpr int kSfIPT = (kSfTile + kSfX + 2 + kBlock - 1) / kBlock;   // window slots per thread (strided)
constexpr int kSfW = kSfIPT * kBlock;                               // window [t0 - 1, t1 + kSfX + 1) fits
constexpr int kSfWords = kSfW / 64;
constexpr int kSfReg = 16;    // dirty segments up to this size are ranked in registers
constexpr int kSfLds = 64;    // dirty segments up to this size are sorted in the block; longer: segfix_big_kernel

struct SfMode {
    int dshift;
    uint32_t dmask;
    int pshift;
    uint64_t pmask;
};
__device__ __forceinline__ uint64_t sf_prefix(uint64_t x, const SfMode& md) { return (x >> md.pshift) & md.pmask; }
__device__ __forceinline__ uint32_t sf_digit(uint64_t x, const SfMode& md) { return (uint32_t)(x >> md.dshift) & md.dmask; }

__device__ __forceinline__ void sf_push_big(uint32_t p, uint32_t* big_list, uint32_t* big_count, uint32_t cap,
                                            uint32_t* err) {
    const uint32_t i = atomicAdd(big_count, 1u);
    if (i < cap) big_list[i] = p;
    else atomicOr(err, 16u);
}

// start of the segment holding window slot r: the highest start bit <= r
__device__ __forceinline__ int sf_seg_start(const uint64_t* smask, const int16_t* lastw, int r) {
    const int wi = r >> 6, bi = r & 63;
    const uint64_t sm = smask[wi] & (bi == 63 ? ~0ull : ((2ull << bi) - 1));
    return sm ? wi * 64 + 63 - __builtin_clzll(sm) : (int)lastw[wi - 1];   // word 0 holds slot 0's start
}

__global__ __launch_bounds__(kBlock) void segfix_tile_kernel(uint64_t* rec, uint32_t n, SfMode md,
                                                             const uint32_t* __restrict__ bstart, int nb,
                                                             uint32_t* __restrict__ big_list,
                                                             uint32_t* __restrict__ big_count, uint32_t cap,
                                                             uint32_t* err, int force_big,
                                                             unsigned long long* dbg) {
    __shared__ uint64_t w[kSfW];
    __shared__ uint64_t smask[kSfWords];   // segment starts (bucket starts first)
    __shared__ uint64_t dmask[kSfWords];   // dirty pairs (position r: pair (r - 1, r))
    __shared__ uint64_t sdirty[kSfWords];  // at a segment start: the segment holds a dirty pair
    __shared__ int16_t lastw[kSfWords], nextw[kSfWords];
    __shared__ uint32_t jobs[kSfW / 2];    // dirty owned segments (>= 2 records each)
    __shared__ uint32_t s_njobs;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t t0 = blockIdx.x * kSfTile;
    const uint32_t t1 = min(t0 + (uint32_t)kSfTile, n);
    const uint32_t wbeg = t0 ? t0 - 1 : 0;
    const uint32_t wload = min(t1 + (uint32_t)kSfX + 1, n);
    const int wn = (int)(wload - wbeg);
    const long long c0 = clock64();
    const uint32_t bsv = tid <= nb ? bstart[tid] : 0u;   // issued with the record loads
    {
        uint64_t x[kSfIPT];   // all loads in flight before the first LDS store
        #pragma unroll
        for (int k = 0; k < kSfIPT; ++k) {
            const int r = tid + k * kBlock;
            x[k] = rec[wbeg + (uint32_t)(r < wn ? r : wn - 1)];
        }
        if (tid < kSfWords) { smask[tid] = 0; sdirty[tid] = 0; }
        if (tid == 0) s_njobs = 0;
        #pragma unroll
        for (int k = 0; k < kSfIPT; ++k) w[tid + k * kBlock] = x[k];
    }
    __syncthreads();
    const long long c1 = clock64();
    if (tid <= nb && bsv > wbeg && bsv < wload) atomicOr(&smask[(bsv - wbeg) >> 6], 1ull << ((bsv - wbeg) & 63));
    for (int b = tid + kBlock; b <= nb; b += kBlock) {
        const uint32_t p = bstart[b];
        if (p > wbeg && p < wload) atomicOr(&smask[(p - wbeg) >> 6], 1ull << ((p - wbeg) & 63));
    }
    __syncthreads();
    // slot r = k * 256 + wv * 64 + lane: bitmap word k * 4 + wv, bit lane
    uint32_t dk = 0;
    #pragma unroll
    for (int k = 0; k < kSfIPT; ++k) {
        const int r = tid + k * kBlock;
        bool st = false, dirty = false;
        if (r < wn) {
            st = r == 0 || ((smask[r >> 6] >> (r & 63)) & 1ull);
            if (!st) {
                const uint64_t x = w[r], y = w[r - 1];
                st = sf_prefix(x, md) != sf_prefix(y, md);
                dirty = !st && sf_digit(x, md) < sf_digit(y, md);
            }
        }
        const uint64_t sb = __ballot(st), db = __ballot(dirty);
        dk |= (dirty ? 1u : 0u) << k;
        if (lane == 0) { smask[k * 4 + wv] = sb; dmask[k * 4 + wv] = db; }   // after every read of word k*4+wv
    }
    __syncthreads();
    const long long c2 = clock64();
    if (dbg && tid == 0) {
        atomicAdd(dbg, (unsigned long long)(c1 - c0));
        atomicAdd(dbg + 1, (unsigned long long)(c2 - c1));
    }
    // per bitmap word: the last segment start at or before its end (prefix max) and the
    // first one at or after its beginning (suffix min): segment bounds in O(1) per slot
    if (wv == 0) {
        int ls = -1, fs = kSfW;
        if (lane < kSfWords) {
            const uint64_t sm = smask[lane];
            if (sm) { ls = lane * 64 + 63 - __builtin_clzll(sm); fs = lane * 64 + __builtin_ctzll(sm); }
        }
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const int a = __shfl_up(ls, dd, 64), c = __shfl_down(fs, dd, 64);
            if (lane >= dd) ls = max(ls, a);
            if (lane + dd < 64) fs = min(fs, c);
        }
        if (lane < kSfWords) { lastw[lane] = (int16_t)ls; nextw[lane] = (int16_t)fs; }
        const int q = __shfl(ls, kSfWords - 1, 64);   // the window's last segment start
        if (tid == 0 && wload < n) {   // ... whose segment runs past the window
            const uint32_t p = wbeg + (uint32_t)q;
            if (p >= t0 && p < t1) sf_push_big(p, big_list, big_count, cap, err);
        }
    }
    __syncthreads();
    // a dirty pair marks its segment's start
    #pragma unroll 1
    for (int k = 0; k < kSfIPT; ++k) {
        if (!((dk >> k) & 1u)) continue;
        const int r = tid + k * kBlock;
        const int s = sf_seg_start(smask, lastw, r);
        atomicOr(&sdirty[s >> 6], 1ull << (s & 63));
    }
    __syncthreads();
    // owned dirty segments -> jobs (the lane at the segment start), big ones -> big list
    #pragma unroll 1
    for (int k = 0; k < kSfIPT; ++k) {
        const int r = tid + k * kBlock;
        const int wi = k * (kBlock / 64) + wv;   // uniform in the wave
        if (!__ballot(r < wn)) break;
        const uint64_t sm = smask[wi];
        const uint64_t smb = sm & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
        const int s = smb ? wi * 64 + 63 - __builtin_clzll(smb) : (int)lastw[wi > 0 ? wi - 1 : 0];
        if (r >= wn || !((sdirty[s >> 6] >> (s & 63)) & 1ull)) continue;
        const uint32_t ps = wbeg + (uint32_t)s;
        if (ps < t0 || ps >= t1) continue;   // not owned
        const uint64_t sa = lane == 63 ? 0ull : (sm & (~0ull << (lane + 1)));
        int e = sa ? wi * 64 + __builtin_ctzll(sa) : (wi + 1 < kSfWords ? (int)nextw[wi + 1] : kSfW);
        if (e >= wn) {
            if (wload < n) continue;   // open: the big kernel sorts it
            e = wn;                    // the stream's last segment
        }
        const int m = e - s;
        if (m > kSfLds || (force_big == 1 && (ps & 63u) == 0u)) {   // force_big: test knob
            if (r == s) sf_push_big(ps, big_list, big_count, cap, err);
            continue;
        }
        if (r == s) {   // one job per segment: (start << 7 | size)
            if (dbg) { atomicAdd(dbg + 2, 1ull); atomicAdd(dbg + 3, (unsigned long long)m); }
            jobs[atomicAdd(&s_njobs, 1u)] = ((uint32_t)s << 7) | (uint32_t)m;
        }
    }
    __syncthreads();
    // one lane per dirty segment: up to kSfReg records ranked in registers, longer ones
    // (<= kSfLds) from LDS
    const uint32_t nj = force_big == 3 ? 0u : s_njobs;
    for (uint32_t j = tid; j < nj; j += kBlock) {
        const int s = (int)(jobs[j] >> 7), m = (int)(jobs[j] & 127u);
        const uint32_t ps = wbeg + (uint32_t)s;
        if (m <= kSfReg) {
            uint64_t y[kSfReg];
            uint32_t d[kSfReg];
            #pragma unroll
            for (int u = 0; u < kSfReg; ++u) {
                y[u] = w[min(s + u, kSfW - 1)];
                d[u] = u < m ? sf_digit(y[u], md) : 0xFFFFFFFFu;   // past the end: never smaller
            }
            #pragma unroll
            for (int i = 0; i < kSfReg; ++i) {
                uint32_t rank = 0;
                #pragma unroll
                for (int u = 0; u < kSfReg; ++u)
                    rank += (d[u] < d[i] || (d[u] == d[i] && u < i)) ? 1u : 0u;
                if (i < m && force_big != 2) rec[ps + rank] = y[i];
            }
        } else {
            for (int i = 0; i < m; ++i) {
                const uint64_t x = w[s + i];
                const uint32_t di = sf_digit(x, md);
                uint32_t rank = 0;
                for (int u = 0; u < m; ++u) {
                    const uint32_t du = sf_digit(w[s + u], md);
                    rank += (du < di || (du == di && u < i)) ? 1u : 0u;
                }
                if (force_big != 2) rec[ps + rank] = x;
            }
        }
    }
}

// Big-list segments (long repeats, N runs, and the segment running past a window): one
// block per segment finds its end, checks whether it is dirty, and if so sorts it stably
// by the digit through the scratch buffer (the sort's free ping-pong buffer).
__global__ __launch_bounds__(kBlock) void segfix_big_kernel(uint64_t* rec, uint64_t* scratch, uint32_t n, SfMode md,
                                                            const uint32_t* __restrict__ bstart, int nb,
                                                            const uint32_t* __restrict__ big_list,
                                                            const uint32_t* __restrict__ big_count, uint32_t cap) {
    __shared__ uint32_t base[256];
    __shared__ uint32_t wc[kBlock / 64][256];
    __shared__ uint32_t s_e, s_dirty;
    const int tid = threadIdx.x, wv = tid >> 6;
    const uint32_t cnt = min(*big_count, cap);
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        const uint32_t s = big_list[k];
        // end of the bucket holding s: first bucket start > s (bstart[nb] = n)
        int lo = 0, hi = nb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (bstart[mid] > s) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t bend = min(bstart[lo], n);
        if (tid == 0) { s_e = bend; s_dirty = 0; }
        base[tid] = 0;
        __syncthreads();
        const uint64_t ps = sf_prefix(rec[s], md);
        for (uint32_t q0 = s + 1; q0 < bend; q0 += kBlock) {
            const uint32_t q = q0 + tid;
            if (q < bend && sf_prefix(rec[q], md) != ps) atomicMin(&s_e, q);
            __syncthreads();
            if (s_e < q0 + kBlock) break;   // uniform: read after the barrier (later minima are larger)
        }
        const uint32_t e = s_e;
        for (uint32_t q = s + 1 + tid; q < e; q += kBlock)
            if (sf_digit(rec[q], md) < sf_digit(rec[q - 1], md)) s_dirty = 1u;
        __syncthreads();
        if (!s_dirty) continue;   // uniform
        for (uint32_t q = s + tid; q < e; q += kBlock) atomicAdd(&base[sf_digit(rec[q], md)], 1u);
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = s;
            for (int d = 0; d < 256; ++d) { const uint32_t c = base[d]; base[d] = acc; acc += c; }
        }
        __syncthreads();
        for (uint32_t c = s; c < e; c += kBlock) {
            const uint32_t q = c + tid;
            const bool valid = q < e;
            const uint64_t x = valid ? rec[q] : 0ull;
            const uint32_t d = sf_digit(x, md);
            #pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) wc[w][tid] = 0;
            __syncthreads();
            uint32_t tot;
            const uint32_t rk = wave_match_rank<8>(d, valid, &tot);
            if (valid && rk == 0) wc[wv][d] = tot;
            __syncthreads();
            if (valid) {
                uint32_t pre = 0;
                #pragma unroll
                for (int w = 0; w < kBlock / 64; ++w) pre += (w < wv) ? wc[w][d] : 0u;
                scratch[base[d] + pre + rk] = x;
            }
            __syncthreads();
            uint32_t add = 0;
            #pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) add += wc[w][tid];
            base[tid] += add;
            __syncthreads();
        }
        __threadfence();
        __syncthreads();
        for (uint32_t q = s + tid; q < e; q += kBlock) rec[q] = scratch[q];
        __syncthreads();
    }
}

}  // namespace

// MUMS_DEV_SEGFIX=1: the lowest digit of a sort of >= 2 digits is finished by the segment
// fix-up instead of an onesweep pass (=2: every dirty segment through segfix_big_kernel,
// for tests).  Off by default: on BASELINE config 3 the fix-up costs what the pass it
// replaces costs.
bool seg_segfix_enabled() {
    const char* e = getenv("MUMS_DEV_SEGFIX");
    return e && (e[0] == '1' || e[0] == '2' || e[0] == '3' || e[0] == '4');
}

static int seg_segfix_force_big() {   // 1: forced big path; 2 / 3: timing experiments (results wrong)
    const char* e = getenv("MUMS_DEV_SEGFIX");
    return (e && e[0] == '2') ? 1 : (e && e[0] == '3') ? 2 : (e && e[0] == '4') ? 3 : 0;
}

int seg_onesweep_launches(int key_bits) {
    const int npass = (key_bits + 7) / 8;
    return (npass >= 2 && seg_segfix_enabled()) ? npass - 1 : npass;
}

uint64_t seg_tiles_upper(uint64_t n, int msd_bits, uint32_t tile) { return (n + tile - 1) / tile + (1ull << msd_bits) + 1; }

size_t seg_tmp_bytes(uint64_t n, int msd_bits) {
    const uint64_t ub = seg_tiles_upper(n, msd_bits);
    const uint64_t nb = 1ull << msd_bits;
    const uint64_t h = ub * kDigits;
    return (h + 64) * 4 + (2 * nb + 130) * 4 + scan_tmp_bytes(h > nb ? h : nb) + 512;
}

// Regroup: dst[j] for j in [dst_off[c], dst_off[c] + len[c]) = src[src_off[c] + (j - dst_off[c])];
// chunks sorted by dst_off and tiling [0, n).  One block per 4096 destination records:
// the block's first chunk by binary search, then a short forward walk per element.
__global__ __launch_bounds__(256) void regroup_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                      const uint64_t* __restrict__ chunks, uint32_t nchunks,
                                                      uint64_t n) {
    __shared__ uint32_t s_c0;
    const uint64_t j0 = (uint64_t)blockIdx.x * 4096;
    if (threadIdx.x == 0) {
        uint32_t lo = 0, hi = nchunks - 1;   // last chunk with dst_off <= j0
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (chunks[3 * mid + 1] <= j0) lo = mid;
            else hi = mid - 1;
        }
        s_c0 = lo;
    }
    __syncthreads();
    uint32_t c = s_c0;
    for (uint64_t j = j0 + threadIdx.x; j < j0 + 4096 && j < n; j += 256) {
        while (c + 1 < nchunks && chunks[3 * (c + 1) + 1] <= j) ++c;
        dst[j] = src[chunks[3 * c] + (j - chunks[3 * c + 1])];
    }
}

hipError_t launch_regroup(const uint64_t* src, uint64_t* dst, const uint64_t* d_chunks, uint32_t nchunks, uint64_t n,
                          hipStream_t st) {
    if (n == 0 || nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(regroup_kernel, dim3((unsigned)((n + 4095) / 4096)), dim3(256), 0, st, src, dst, d_chunks,
                       nchunks, n);
    return hipGetLastError();
}

hipError_t seg_bucket_starts(const uint32_t* d_hist_scanned, uint32_t T, int msd_bits, uint64_t n, uint32_t* bstart,
                             hipStream_t st) {
    const int nb = 1 << msd_bits;
    if (msd_bits == 0) {
        hipLaunchKernelGGL(single_bucket_kernel, dim3(1), dim3(64), 0, st, n, bstart);
    } else {
        hipLaunchKernelGGL(bucket_starts_kernel, dim3((nb + 256) / 256), dim3(256), 0, st, d_hist_scanned, T, nb, n,
                           bstart, (uint32_t*)nullptr);
    }
    return hipGetLastError();
}

hipError_t build_seg_tiles_from_starts(const uint32_t* bstart, int msd_bits, uint64_t n, SegTile* d_tiles,
                                       uint32_t* d_ntiles, void* d_tmp, hipStream_t st, uint32_t tile) {
    const int nb = 1 << msd_bits;
    const uint64_t ub = seg_tiles_upper(n, msd_bits, tile);
    uint32_t* tfirst = (uint32_t*)d_tmp;
    void* stmp = (void*)(tfirst + nb + 64);
    hipLaunchKernelGGL(ntb_from_starts_kernel, dim3((nb + 256) / 256), dim3(256), 0, st, bstart, nb, tile, tfirst);
    // tfirst[b] = exclusive scan of tiles per bucket; tfirst[nb] = total
    hipError_t e = exclusive_scan_u32(tfirst, (uint64_t)nb + 1, stmp, nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tiles_kernel, dim3((unsigned)((ub + 255) / 256)), dim3(256), 0, st, bstart, tfirst, nb, ub,
                       tile, d_tiles, d_ntiles);
    hipLaunchKernelGGL(claim_order_kernel, dim3((unsigned)((ub + 255) / 256)), dim3(256), 0, st, tfirst, nb, ub,
                       d_tiles);
    return hipGetLastError();
}

// d_hist_scanned: the scanned MSD histogram [nb x T] (nullptr when msd_bits == 0).
hipError_t build_seg_tiles(const uint32_t* d_hist_scanned, uint32_t T, int msd_bits, uint64_t n, SegTile* d_tiles,
                           uint32_t* d_ntiles, uint32_t* bstart, void* d_tmp, hipStream_t st) {
    hipError_t e = seg_bucket_starts(d_hist_scanned, T, msd_bits, n, bstart, st);
    if (e != hipSuccess) return e;
    return build_seg_tiles_from_starts(bstart, msd_bits, n, d_tiles, d_ntiles, d_tmp, st);
}

// d_tmp layout: status [npass][ub][256] | ghist [nb][npass][256] | dbase [nb][npass][256]
// | counters [npass] (all zeroed per sort) | sort tiles [ub] | tile-build scratch
// scratch of build_seg_tiles_from_starts (tfirst + scan), rounded to 256 B
static size_t seg_build_tmp_bytes(uint64_t nb) { return ((nb + 128) * 4 + scan_tmp_bytes(nb + 1) + 4096 + 255) & ~(size_t)255; }

// big-list capacity of the segment fix-up: <= 1 open segment per tile, < n / 64 dirty
// segments of more than kSfLds records, + the forced test entries (starts at multiples of 64)
static uint64_t segfix_cap(uint64_t n) { return n / 32 + 2 * ((n + kSfTile - 1) / kSfTile + 2); }

// development A/B of the onesweep block shape (MUMS_DEV_OS_VARIANT, read once):
// 0 = <768 threads, 12 records> (9216-record tiles, the per-wave counts aliased into the
// exchange buffer: 76 KB, two blocks and 24 waves per CU, 79 VGPRs), 1-6 and 8 aliased too:
// 1 <512, 16> (8192), 2 <512, 12> and 3 <384, 16> (6144-record tiles, 52 KB: three blocks per
// CU), 4 <256, 16> and 5 <512, 8> (4096, 36 KB: four per CU), 6 <1024, 8> (8192, 32 waves per
// CU), 8 <640, 14> (8960); 7 = the round-2 shape <512, 16> with the counts in their own LDS
// (8192, 78 KB).  Measured on C3 in one call: 0 is 2.5 % faster per pass than 7 and 1;
// 6144- and 4096-record tiles (more blocks per CU) are 6-14 % slower: the digit runs a tile
// stores get shorter.
static int os_variant() {
    static const int v = [] {
        const char* e = getenv("MUMS_DEV_OS_VARIANT");
        const int x = e ? atoi(e) : 0;
        return x >= 0 && x <= 8 ? x : 0;
    }();
    return v;
}
// XCD-grouped claim queues (default since round 5: 3.31 -> 3.04 ms per C3 pass, same box,
// profiles/r05j_xcd_ab.txt); MUMS_DEV_OS_XCD=0 (read per call) restores the single queue
static bool os_xcd() {
    const char* e = getenv("MUMS_DEV_OS_XCD");
    return !(e && e[0] == '0');
}
// claim descriptors in the XCD queues (one dependent load per claim, default);
// MUMS_DEV_OS_XD=0 (read per call) reads the tile id, then its SegTile
static bool os_xd() {
    const char* e = getenv("MUMS_DEV_OS_XD");
    return !(e && e[0] == '0');
}
static int os_tile() {
    static const int t[9] = {kSortTile, 8192, 6144, 6144, 4096, 4096, 8192, 8192, 8960};
    return MUMS_SORT_PERSIST ? kSortTile : t[os_variant()];
}

size_t onesweep_tmp_bytes(uint64_t n, int msd_bits, int key_bits) {
    const uint64_t ub = seg_tiles_upper(n, msd_bits, os_tile());
    const int npass = (key_bits + 7) / 8;
    const uint64_t nb = 1ull << msd_bits;
    const size_t b = (ub * kDigits * (uint64_t)npass + 2 * nb * npass * kDigits + 256 + 64) * 4 +
                     2 * (ub * sizeof(SegTile) + 256) + seg_build_tmp_bytes(nb) + segfix_cap(n) * 4 +
                     256;   // + the claim-ordered copy, the fix-up's big list
    return seg_wide_sort_enabled() ? std::max(b, onesweep_wide_tmp_bytes(n, msd_bits, key_bits)) : b;
}

// segment fix-up launches: big_count[0..1] zeroed by the caller, big_list in d_list
static hipError_t launch_segfix(uint64_t* rec, uint64_t* scratch, uint64_t n, const SfMode& md, const uint32_t* d_bstart,
                                int nb, uint32_t* big_count, void* d_list, uint32_t* d_err, hipStream_t st) {
    const uint64_t tiles = (n + kSfTile - 1) / kSfTile;
    const uint32_t cap = (uint32_t)segfix_cap(n);
    uint32_t* big_list = (uint32_t*)d_list;
    unsigned long long* dbg = nullptr;
    const bool stats = getenv("MUMS_DEV_SEGFIX_STATS") != nullptr;
    if (stats) {   // development: per-phase cycles and job counts
        dbg = (unsigned long long*)(big_count + 2);   // 8-aligned (big_count = counters + 48 or d_tmp)
        (void)hipMemsetAsync(dbg, 0, 32, st);
    }
    hipLaunchKernelGGL(segfix_tile_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, st, rec, (uint32_t)n, md, d_bstart,
                       nb, big_list, big_count, cap, d_err, seg_segfix_force_big(), dbg);
    hipLaunchKernelGGL(segfix_big_kernel, dim3(256), dim3(kBlock), 0, st, rec, scratch, (uint32_t)n, md, d_bstart, nb,
                       big_list, big_count, cap);
    if (stats) {   // development: big-list length per fix-up
        uint32_t hc[2] = {0, 0};
        unsigned long long hd[4] = {0, 0, 0, 0};
        (void)hipMemcpyAsync(hc, big_count, 8, hipMemcpyDeviceToHost, st);
        (void)hipMemcpyAsync(hd, dbg, 32, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        fprintf(stderr, "segfix: n=%llu tiles=%llu dmask=%u big=%u forced=%u cyc/block load=%.0f flags=%.0f jobs=%llu job_recs=%llu\n",
                (unsigned long long)n, (unsigned long long)tiles, md.dmask, hc[0], hc[1], hd[0] / (double)tiles,
                hd[1] / (double)tiles, hd[2], hd[3]);
    }
    return hipGetLastError();
}

size_t seg_parity_fix_tmp_bytes(uint64_t n) { return 256 + segfix_cap(n) * 4 + 256; }

hipError_t seg_parity_fix(uint64_t* rec, uint64_t* scratch, uint64_t n, int key_bits, int msd_bits,
                          const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, hipStream_t st, int key_shift) {
    if (n == 0 || key_bits < 2) return hipSuccess;
    SfMode md;
    md.dshift = key_shift;
    md.dmask = 1u;
    md.pshift = key_shift + 1;
    md.pmask = (1ull << (key_bits - 1)) - 1;
    uint32_t* big_count = (uint32_t*)d_tmp;
    hipError_t e = hipMemsetAsync(big_count, 0, 64, st);
    if (e != hipSuccess) return e;
    return launch_segfix(rec, scratch, n, md, d_bstart, 1 << msd_bits, big_count, (char*)d_tmp + 256, d_err, st);
}

hipError_t seg_onesweep_sort(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, int msd_bits,
                             const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, int* out_buf, hipStream_t st,
                             hipEvent_t* ev_ds, int key_shift, bool mask_parity, bool key_runs,
                             const uint32_t* hist_in, const uint64_t* gsrc, uint32_t* gout) {
    const int nkd = (key_bits + 7) / 8;                  // key digits
    const bool segfix = nkd >= 2 && seg_segfix_enabled();
    const int npass = segfix ? nkd - 1 : nkd;            // onesweep launches (digits above the lowest)
    const int digit_shift = key_shift;                   // the lowest digit
    if (segfix) key_shift += 8;
    *out_buf = npass % 2;
    if (n == 0 || npass == 0) return hipSuccess;
    if (nkd > 4) return hipErrorInvalidValue;
    const uint64_t nb = 1ull << msd_bits;
    const int tile = os_tile();
    const uint64_t ub = seg_tiles_upper(n, msd_bits, tile);
    uint32_t* status = (uint32_t*)d_tmp;                       // [npass][ub][256]
    uint32_t* ghist = status + ub_status(ub, npass);           // [nb][npass][256]
    uint32_t* dbase = ghist + nb * npass * kDigits;            // [nb][npass][256]
    uint32_t* counters = dbase + nb * npass * kDigits;         // [npass] + ntiles
    const size_t zero_bytes = ((uint64_t)(counters - status) + 256) * 4;   // + the XCD queue counters
    SegTile* stiles = (SegTile*)((char*)d_tmp + ((zero_bytes + 255) & ~(size_t)255));
    SegTile* ctiles = (SegTile*)((char*)stiles + ((ub * sizeof(SegTile) + 255) & ~(size_t)255));
    void* btmp = (void*)((char*)ctiles + ((ub * sizeof(SegTile) + 255) & ~(size_t)255));
    hipError_t e = hipMemsetAsync(status, 0, zero_bytes, st);
    if (e != hipSuccess) return e;
    e = build_seg_tiles_from_starts(d_bstart, msd_bits, n, stiles, counters + 32, btmp, st, tile);
    if (e != hipSuccess) return e;
#if MUMS_OS_CTILES
    hipLaunchKernelGGL(claim_tiles_kernel, dim3((unsigned)((ub + 255) / 256)), dim3(256), 0, st, stiles, ub, ctiles);
    const SegTile* otiles = ctiles;   // what the onesweep launches read
    uint32_t* xq = nullptr;
#else
    const SegTile* otiles = stiles;
    // XCD-grouped claim queues (development A/B): the unused claim-ordered copy's room
    // (fewer than 8 MSD buckets: one queue is all there is)
    uint32_t* xq = (os_xcd() && nb >= 8 && !MUMS_SORT_PERSIST) ? (uint32_t*)ctiles : nullptr;
    // the queues' claim descriptors behind them (the claim-ordered copy's room: 48 B per tile)
    uint4* xqd = xq ? (uint4*)(((uintptr_t)(xq + 32 + ub) + 15) & ~(uintptr_t)15) : nullptr;
    const uint4* xd = os_xd() ? xqd : nullptr;
    if (xq)
        hipLaunchKernelGGL(xcd_order_kernel, dim3((unsigned)((ub + 255) / 256)), dim3(256), 0, st,
                           (const uint32_t*)btmp, (int)nb, ub, stiles, xq, xqd);
#endif
    const unsigned gblocks = (unsigned)((ub + kGhistTilesPerBlock - 1) / kGhistTilesPerBlock);
    // the histogram read counts digit 0 only when every later pass's digits are
    // counted by the pass before it (MUMS_OS_NEXTHIST, plain onesweep kernel)
    const bool nexthist = MUMS_OS_NEXTHIST && !MUMS_SORT_PERSIST;
    if (hist_in && nb == 1 && !segfix && !nexthist) {   // the producer counted every pass's digits
        e = hipMemcpyAsync(ghist, hist_in, (size_t)npass * kDigits * 4, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(seg_ghist_kernel, dim3(gblocks), dim3(kBlock), 0, st, recA, stiles, ub, npass, ghist,
                           key_shift, nexthist ? 1 : npass, key_runs ? 1 : 0);
    }
    if (nexthist)
        hipLaunchKernelGGL(seg_dbase_kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, ghist, d_bstart, npass, dbase,
                           0);
    else
        hipLaunchKernelGGL(seg_dbase_kernel, dim3((unsigned)(nb * npass)), dim3(kBlock), 0, st, ghist, d_bstart,
                           npass, dbase, -1);
#if MUMS_SORT_PERSIST
    // resident blocks of the persistent pass: occupancy x CUs of the current device
    uint64_t persist_grid = 0;
    {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, (const void*)seg_onesweep_persist_kernel<kSortBlock, kSortTile / kSortBlock>, kSortBlock, 0);
        persist_grid = (uint64_t)std::max(cus, 1) * (uint64_t)std::max(per, 1);
    }
#endif
#if MUMS_OS_STATS
    unsigned long long* os_dev = nullptr;   // development: the per-tile stamps of every pass
    (void)hipMalloc(&os_dev, ub * 80);
    (void)hipMemsetAsync(os_dev, 0, ub * 80, st);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_os_stats), &os_dev, sizeof(os_dev), 0, hipMemcpyHostToDevice);
#endif
    uint64_t* src = recA;
    uint64_t* dst = recB;
    for (int p = 0; p < npass; ++p) {
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p], st);
#if MUMS_SORT_PERSIST
        hipLaunchKernelGGL((seg_onesweep_persist_kernel<kSortBlock, kSortTile / kSortBlock>),
                           dim3((unsigned)std::min<uint64_t>(ub, persist_grid)), dim3(kSortBlock), 0, st, src, dst,
                           stiles, (uint32_t)ub, key_shift + 8 * p, p, npass, dbase,
                           status + (uint64_t)p * ub * kDigits, counters + p, d_err);
#else
        {
            uint32_t* gn = (nexthist && p + 1 < npass) ? ghist : (uint32_t*)nullptr;
            uint32_t* sp = status + (uint64_t)p * ub * kDigits;
            const int sh = key_shift + 8 * p;
            uint32_t* tc = xq ? counters + 128 + 8 * p : counters + p;
#define MUMS_OS_LAUNCH(OB, IPT, AL)                                                                               \
    hipLaunchKernelGGL((seg_onesweep_kernel<OB, IPT, AL>), dim3((unsigned)ub), dim3(OB), 0, st, src, dst, otiles, \
                       (uint32_t)ub, sh, p, npass, dbase, sp, tc, d_err, gn, xq, nullptr, nullptr, xd)
            if (key_runs && gout && p + 1 == npass) {   // the last pass stores gout[o] = gsrc[k]
                hipLaunchKernelGGL((seg_onesweep_kernel<kSortBlock, kSortTile / kSortBlock, true, true, true>),
                                   dim3((unsigned)ub), dim3(kSortBlock), 0, st, src, dst, otiles, (uint32_t)ub, sh, p,
                                   npass, dbase, sp, tc, d_err, gn, xq, gsrc, gout, xd);
            } else if (key_runs) {   // equal-digit runs: publish after the ranking (no per-record LDS atomics)
                hipLaunchKernelGGL((seg_onesweep_kernel<kSortBlock, kSortTile / kSortBlock, true, true>),
                                   dim3((unsigned)ub), dim3(kSortBlock), 0, st, src, dst, otiles, (uint32_t)ub, sh, p,
                                   npass, dbase, sp, tc, d_err, gn, xq, nullptr, nullptr, xd);
            } else
            switch (os_variant()) {
            case 1: MUMS_OS_LAUNCH(512, 16, true); break;
            case 2: MUMS_OS_LAUNCH(512, 12, true); break;
            case 3: MUMS_OS_LAUNCH(384, 16, true); break;
            case 4: MUMS_OS_LAUNCH(256, 16, true); break;
            case 5: MUMS_OS_LAUNCH(512, 8, true); break;
            case 6: MUMS_OS_LAUNCH(1024, 8, true); break;
            case 7: MUMS_OS_LAUNCH(512, 16, false); break;
            case 8: MUMS_OS_LAUNCH(640, 14, true); break;
            default: MUMS_OS_LAUNCH(kSortBlock, kSortTile / kSortBlock, true); break;
            }
#undef MUMS_OS_LAUNCH
        }
#endif
        e = hipGetLastError();
        if (e != hipSuccess) return e;
#if MUMS_OS_STATS
        {   // development: per-phase wall clock per tile (us) of this pass; per XCD (block % 8: the
            // real-time counters of different XCDs need not agree) the busy block slots
            (void)hipStreamSynchronize(st);
            std::vector<unsigned long long> hs(ub * 10);
            (void)hipMemcpy(hs.data(), os_dev, ub * 80, hipMemcpyDeviceToHost);
            double ph[7] = {0, 0, 0, 0, 0, 0, 0}, tot = 0;
            unsigned long long lo[8], hi[8];
            double busy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int x = 0; x < 8; ++x) { lo[x] = ~0ull; hi[x] = 0; }
            uint64_t nt = 0;
            for (uint64_t i = 0; i < ub; ++i) {
                const unsigned long long* o = &hs[i * 10];
                if (!o[9]) continue;
                ++nt;
                for (int k = 1; k < 8; ++k) ph[k - 1] += (double)(o[k] - o[k - 1]);
                tot += (double)(o[7] - o[0]);
                const int x = (int)(o[8] & 7);
                lo[x] = std::min(lo[x], o[0]);
                hi[x] = std::max(hi[x], o[7]);
                busy[x] += (double)(o[7] - o[0]);
            }
            const double d = nt ? (double)nt * 100.0 : 1.0;
            double bs = 0, wl = 0;
            for (int x = 0; x < 8; ++x)
                if (hi[x] > lo[x]) { bs += busy[x] / (double)(hi[x] - lo[x]); wl = std::max(wl, (double)(hi[x] - lo[x])); }
            fprintf(stderr, "os_stats n=%llu pass=%d tiles=%llu us/tile: claim %.2f load+count %.2f rank %.2f lookback %.2f "
                    "lstart+exch %.2f stores %.2f drain %.2f | tile %.2f us, XCD wall %.1f us, busy block slots %.1f\n",
                    (unsigned long long)n, p, (unsigned long long)nt, ph[0] / d, ph[1] / d, ph[2] / d, ph[3] / d,
                    ph[4] / d, ph[5] / d, ph[6] / d, tot / d, wl / 100.0, bs);
            (void)hipMemset(os_dev, 0, ub * 80);
        }
#endif
        if (nexthist && p + 1 < npass)
            hipLaunchKernelGGL(seg_dbase_kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, ghist, d_bstart, npass,
                               dbase, p + 1);
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p + 1], st);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
#if MUMS_OS_STATS
    (void)hipStreamSynchronize(st);
    (void)hipFree(os_dev);
#endif
    if (segfix) {   // src holds the stream sorted above the lowest digit; dst is free scratch
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * npass], st);
        SfMode md;
        md.dshift = mask_parity ? digit_shift + 1 : digit_shift;
        md.dmask = mask_parity ? 0x7Fu : 0xFFu;
        md.pshift = digit_shift + 8;
        md.pmask = (1ull << (key_bits - 8)) - 1;
        e = launch_segfix(src, dst, n, md, d_bstart, (int)nb, counters + 48, (char*)btmp + seg_build_tmp_bytes(nb),
                          d_err, st);
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * npass + 1], st);
    }
    return hipSuccess;
}

hipError_t seg_radix_sort(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, const SegTile* d_tiles,
                          uint64_t ntiles_ub, void* d_tmp, int* out_buf, hipStream_t st, hipEvent_t* ev_ds) {
    const int passes = (key_bits + 7) / 8;
    *out_buf = passes % 2;  // 0: result in recA, 1: in recB
    if (n == 0 || passes == 0) return hipSuccess;
    const uint64_t h = ntiles_ub * kDigits;
    uint32_t* hist = (uint32_t*)d_tmp;
    void* stmp = (void*)(hist + h + 64);
    uint64_t* src = recA;
    uint64_t* dst = recB;
    for (int p = 0; p < passes; ++p) {
        const int shift = 32 + 8 * p;
        hipLaunchKernelGGL(seg_upsweep, dim3((unsigned)ntiles_ub), dim3(kBlock), 0, st, src, d_tiles, shift, hist);
        hipError_t e = exclusive_scan_u32(hist, h, stmp, nullptr, st);
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p], st);
        hipLaunchKernelGGL(seg_downsweep, dim3((unsigned)ntiles_ub), dim3(kBlock), 0, st, src, d_tiles, shift, hist,
                           dst);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (ev_ds) (void)hipEventRecord(ev_ds[2 * p + 1], st);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    return hipSuccess;
}

}  // namespace mums
