// mums_internal.h -- shared declarations of the gfx950 multi-MUM pipeline.
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   * genome g's ASCII bytes (caller- or context-owned), n_g bytes
//   * ckey[N]   : compact canonical spaced-seed key per seed-mer, indexed by the
//                 global seed-mer index i = base_g + p (p = 0-based position in
//                 genome g, 0 <= p < m_g = n_g - L + 1).  ckey = (v << 1) | parity,
//                 v = the 2w-bit canonical seed value (top 2w bits of
//                 GetDnaSeedMer, SortedMerList.cpp:764-769), parity = 1 iff the
//                 reverse complement was chosen.  uint32 when 2w+1 <= 32, else uint64.
//   * skey/sidx : (ckey, i) pairs radix-sorted by ckey (stable) = the G
//                 SortedMerLists merged into one key-ordered stream
//                 (MemorySML.cpp:45-60 + MatchFinder.cpp:172-340).
//   * probes    : one per accepted masked-key group, as the sorted index of the
//                 group head, bucket-sorted (stable) for the per-bucket replay.
//   * entries   : MatchHashEntry pool, int64 [len, offset, start_0..start_{G-1}].
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mums {

constexpr int kMaxG = 32;            // genomes per context (register arrays in the replay)
constexpr int kRepeatLimit = 1000;   // MER_REPEAT_LIMIT, MatchFinder.cpp:166
constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)

// Per-run constants shared by the kernels (passed by value).
struct SeedSpec {
    uint64_t pattern;
    int L;                  // seed length   (getSeedLength, SeedMasks.h:335)
    int w;                  // seed weight   (getSeedWeight, SeedMasks.h:363)
    int nruns;              // maximal runs of care positions in the pattern
    int run_start[32];      // first base offset of each run (0 = first base)
    int run_len[32];        // bases in the run
    int run_dst[32];        // bit shift of the run inside the 2w-bit seed value
};

struct GenomeTable {
    int G;
    uint64_t n[kMaxG];      // sequence lengths
    uint64_t m[kMaxG];      // SMLLength = n - L + 1 (0 if n < L)
    uint64_t base[kMaxG + 1];  // global seed-mer index base; base[G] = N
};

struct MatchParams {
    uint32_t repeat_tol;    // MemHash.h:31
    uint32_t enum_tol;      // MemHash.h:32
    uint32_t table_size;    // MemHash.h:30
    int masked;             // MaskedMemHash::HashMatch semantics
    uint64_t seq_mask;      // MaskedMemHash::SetMask
};

// device-side counters, zeroed at the start of every run
struct DevCounters {
    unsigned long long groups;        // distinct masked keys
    unsigned long long repeat_limit;  // groups above MER_REPEAT_LIMIT
    unsigned long long collisions;    // MemHash::m_collision_count
    unsigned long long entries;       // MemHash::m_mem_count (pool cursor)
    uint32_t err;                     // bit 0: '-' seen in a genome
    uint32_t pad;
    uint32_t nprobes;                 // accepted probes (scan total)
    uint32_t nmatches;                // output matches (scan total)
};

// genome of a global seed-mer index (G <= 32: linear scan is cheapest)
__device__ __forceinline__ int genome_of(const GenomeTable& gt, uint64_t i) {
    int g = 0;
    #pragma unroll 1
    for (int k = 1; k < gt.G; ++k) g += (i >= gt.base[k]) ? 1 : 0;
    return g;
}

// ---- host-side launchers (one per translation unit) -------------------------
struct Workspace;

hipError_t launch_seed_keys(const SeedSpec& ss, const GenomeTable& gt, const char* const* d_ascii,
                            void* d_ckey, bool key64, uint32_t* d_err, hipStream_t st);

// exclusive scan of n uint32 values in place; d_tmp needs scan_tmp_bytes(n)
size_t scan_tmp_bytes(uint64_t n);
hipError_t exclusive_scan_u32(uint32_t* d_data, uint64_t n, void* d_tmp, uint32_t* d_total,
                              hipStream_t st);

// stable LSD radix sort of keys over bit range [0, bits); values are the
// implicit indices 0..n-1 when vals_in == nullptr.  Returns which buffer holds
// the result (0 = A, 1 = B).
size_t radix_tmp_bytes(uint64_t n);
// ev_ds (optional): 2 events per pass recorded around each downsweep launch.
template <typename K>
hipError_t radix_sort(const K* keys_in, const uint32_t* vals_in, uint64_t n, int bits,
                      K* kA, uint32_t* vA, K* kB, uint32_t* vB, void* d_tmp, int* out_buf,
                      hipStream_t st, hipEvent_t* ev_ds = nullptr);

// groups.hip
uint64_t group_tiles(uint64_t N);
uint64_t group_slot_count(uint64_t N);
template <int MG, typename K>
hipError_t launch_probe_tiles(const K* skey, const uint32_t* sidx, uint64_t N, const GenomeTable& gt,
                              const MatchParams& mp, int L, uint32_t* tile_count, uint32_t* slot_head,
                              uint32_t* slot_bucket, void* counters, hipStream_t st);
hipError_t launch_probe_compact(uint64_t N, const uint32_t* tile_count, const uint32_t* tile_off,
                                const uint32_t* slot_head, const uint32_t* slot_bucket, uint32_t* probe_head,
                                uint32_t* probe_bucket, hipStream_t st);

// replay.hip
hipError_t launch_bucket_ranges(const uint32_t* sb, uint64_t P, uint32_t* bstart, uint32_t* bend, hipStream_t st);
template <int MG, typename K>
hipError_t launch_replay(const K* skey, const uint32_t* sidx, uint64_t N, const GenomeTable& gt,
                         const MatchParams& mp, int L, const uint32_t* heads, const uint32_t* bstart,
                         const uint32_t* bend, uint32_t* tbl, int64_t* pool, const K* ckey, uint32_t* tsize,
                         void* ctr, hipStream_t st);
hipError_t launch_emit(const uint32_t* tsize, const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl,
                       const int64_t* pool, int G, uint32_t table_size, uint64_t* out_len, int64_t* out_s,
                       hipStream_t st);

}  // namespace mums
