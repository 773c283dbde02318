// mums_internal.h -- shared declarations of the gfx950 multi-MUM pipeline.
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   * genome g's ASCII bytes (caller- or context-owned), n_g bytes
//   * packed[]  : 2-bit packed genomes, the reference SortedMerList::sequence layout
//                 (translate32, SortedMerList.cpp:425-460), genome g at word woff[g]
//   * the merged key-sorted stream of all seed-mers (the G SortedMerLists of
//     MemorySML.cpp:45-60 merged as MatchFinder::SearchRange walks them,
//     MatchFinder.cpp:172-340), in one of two forms:
//       packed path (2w+1 <= 43): uint64 records (ckey_low << 32 | i), grouped by the
//                 top B = 2w+1-32 ckey bits (MSD buckets; B = 0 for w <= 15)
//       pair path  (larger w)   : (ckey, i) pairs, ckey uint32/uint64
//     where ckey = (v << 1) | parity, v = canonical 2w-bit spaced seed, and
//     i = base_g + position is the global seed-mer index (stable: ties by i).
//   * probes    : one per accepted masked-key group in ascending key order,
//                 (head index | group size << 32) + hash bucket, then bucket-sorted.
//   * entries   : MatchHashEntry pool, int64 [len, offset, start_0..start_{G-1}].
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "restart_plan.h"

namespace mums {

constexpr int kMaxG = 64;            // genomes per context (MaskedMemHash's 64-bit match number)
constexpr int kRepeatLimit = 1000;   // MER_REPEAT_LIMIT, MatchFinder.cpp:166
constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
#ifndef MUMS_SEED_TILE
#define MUMS_SEED_TILE 4096
#endif
constexpr int kSeedTile = MUMS_SEED_TILE;  // positions per key-kernel workgroup
#ifndef MUMS_SEG_TILE
#define MUMS_SEG_TILE 4096
#endif
constexpr int kSegTile = MUMS_SEG_TILE; // records per sort / group tile
constexpr int kLocalIPT = 16;        // records per lane of the LDS-resident local sort (local_sort.hip)
constexpr int kMaxMsdBits = 11;      // packed path: 2w+1 <= 32 + 11
constexpr int kMaxSegBucketBits = 12; // segmented sorts: buckets of a merge (sharded 33-bit records at w21: 12 MSD bits)

// Per-run constants shared by the kernels (passed by value).
constexpr int kMaxSeedRuns = 16;     // runs of care positions in a seed of length <= 32

struct SeedSpec {
    uint64_t pattern;
    int L;                  // seed length   (getSeedLength, SeedMasks.h:335)
    int w;                  // seed weight   (getSeedWeight, SeedMasks.h:363)
    int nruns;              // maximal runs of care positions in the pattern
    int run_start[32];      // first base offset of each run (0 = first base)
    int run_len[32];        // bases in the run
    int run_dst[32];        // bit shift of the run inside the 2w-bit seed value
    // device form: run r of the 64-bit window lands at its seed bits as
    // ((sh >= 0 ? mer >> sh : mer << -sh) & mask); sh = 64 - 2(start + len) - dst
    int run_sh[kMaxSeedRuns];
    uint64_t run_mask[kMaxSeedRuns];
};

struct GenomeTable {
    int G;
    uint64_t n[kMaxG];          // sequence lengths
    uint64_t m[kMaxG];          // SMLLength = n - L + 1 (0 if n < L)
    uint64_t base[kMaxG + 1];   // global seed-mer index base; base[G] = N
    uint64_t woff[kMaxG + 1];   // word offset of genome g in the packed array
    uint32_t tfirst[kMaxG + 1]; // first key-kernel tile of genome g (tiles cover n_g bytes)
    // coarse genome lookup (genome_lookup_init): gl[i >> gl_shift] = the genome of index
    // i's bucket start; every genome is at least 2^gl_shift seed-mers long, so a bucket meets
    // at most two genomes and g = gl[.] + (i >= base[gl[.] + 1]).  gl_n = 0: off.
    uint32_t gl_shift;
    uint32_t gl_n;
    uint8_t gl[256];
};

// the coarse lookup table of gt (bases set; off when a genome is empty or the table would
// need more than 256 buckets)
inline void genome_lookup_init(GenomeTable& gt) {
    gt.gl_n = 0;
    gt.gl_shift = 0;
    const uint64_t N = gt.base[gt.G];
    if (gt.G < 2 || N == 0 || N >= (1ull << 32)) return;
    if (getenv("MUMS_DEV_NO_GL")) return;   // development A/B: the compare-and-select lookup
    uint64_t mn = ~0ull;
    for (int g = 0; g < gt.G; ++g) mn = gt.m[g] < mn ? gt.m[g] : mn;
    if (mn == 0) return;
    const int sh = 63 - __builtin_clzll(mn);
    const uint64_t nb = ((N - 1) >> sh) + 1;
    if (nb > 256) return;
    int g = 0;
    for (uint64_t s = 0; s < nb; ++s) {
        const uint64_t i = s << sh;
        while (g + 1 < gt.G && gt.base[g + 1] <= i) ++g;
        gt.gl[s] = (uint8_t)g;
    }
    gt.gl_shift = (uint32_t)sh;
    gt.gl_n = (uint32_t)nb;
}

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
    uint32_t ntiles;                  // segmented tiles in use
    uint32_t nprobes;                 // accepted probes (scan total)
    uint32_t nmatches;                // output matches (scan total)
    uint32_t ngroups;                 // distinct masked keys (scan total of per-tile counts)
    uint32_t nchains;                 // seed chains among the probes (chains.hip)
    uint32_t max_bucket;              // probes in the fullest hash bucket
    uint32_t scratch32;               // one-word device results read back by the host (compat_split)
    unsigned long long walk_words;    // 64-column hit words evaluated by chain_walk_kernel
    unsigned long long walk_items;    // walks chain_walk_kernel finished
    unsigned long long walk_wins;     // 28-B packed windows those words loaded (present components)
    unsigned long long short_words;   // the same for chain_walk_short_kernel (one lane per walk)
    unsigned long long short_items;   // walks it took from the queue
    unsigned long long short_wins;
    unsigned long long log_n;         // insertion events recorded for SetMatchLog (replay.hip)
};

// A tile of the segmented (per-MSD-bucket) sort/group passes.  Tiles never
// straddle a bucket; hist index of (digit d) = hbase + d * ntb + tb.
struct SegTile {
    uint64_t start;     // first record
    uint64_t bstart;    // bucket range [bstart, bend)
    uint64_t bend;
    uint32_t count;     // records in this tile (0 = unused)
    uint32_t hbase;     // tfirst_b * 256
    uint32_t ntb;       // tiles in this bucket
    uint32_t tb;        // index of this tile within the bucket
    uint32_t bucket;    // MSD bucket id
    uint32_t order;     // onesweep claim order: the c-th claimed block sorts tile tiles[c].order
};

// Stable wave64 "match any" on a kBits-bit digit: *peers_out = popcount of the lanes
// (valid ones) holding the same digit, returned value = how many of them sit in lower
// lanes.  Per digit bit: a 1-bit signed extract (0 / all ones), one ballot, and
// peers &= ~(X ^ ext) on each 32-bit half (one v_bitop3 each); the rank is two mbcnt ops.
template <int kBits>
__device__ __forceinline__ uint32_t wave_match_rank(uint32_t dg, bool valid, uint32_t* peers_out) {
    const uint64_t v = __ballot(valid);
    uint32_t pl = (uint32_t)v, ph = (uint32_t)(v >> 32);
    #pragma unroll
    for (int b = 0; b < kBits; ++b) {
        const uint32_t ms = (uint32_t)__builtin_amdgcn_sbfe((int32_t)dg, b, 1);   // all ones when set
        const uint64_t x = __ballot(ms != 0u);
        // p & ~(x ^ m): LUT index (p << 2 | x << 1 | m) -> bits 4 and 7
        pl = __builtin_amdgcn_bitop3_b32(pl, (uint32_t)x, ms, 0x90);
        ph = __builtin_amdgcn_bitop3_b32(ph, (uint32_t)(x >> 32), ms, 0x90);
    }
    *peers_out = (uint32_t)__builtin_popcount(pl) + (uint32_t)__builtin_popcount(ph);
    return __builtin_amdgcn_mbcnt_hi(ph, __builtin_amdgcn_mbcnt_lo(pl, 0u));
}

// ParallelMemHash compat records' group key (compat.hip, chunked.hip): masked-ckey bits 1-30
// and the chunk's parity, from key2 = chunk << kbits | ckey
__device__ __forceinline__ uint64_t compat_gid(uint64_t k, int kbits) {
    return ((k >> 1) & 0x3FFFFFFFull) | (((k >> kbits) & 1ull) << 30);
}

// genome of a global seed-mer index (G <= 64: a linear scan is cheapest)
__device__ __forceinline__ int genome_of(const GenomeTable& gt, uint64_t i) {
    int g = 0;
    #pragma unroll 1
    for (int k = 1; k < gt.G; ++k) g += (i >= gt.base[k]) ? 1 : 0;
    return g;
}

__host__ __device__ inline uint64_t packed_words(uint64_t n) { return (2 * n) / 32 + (((2 * n) % 32) ? 1 : 0) + 2; }

// ---- host-side launchers ------------------------------------------------------------
// seeds.hip: pack + keys.  mode 0: write ckey[] (pair path, key64 selects width);
// mode 1: MSD histogram hist[b * T + t] of the top msd_bits of ckey (packed path).
hipError_t launch_seed_pack(const SeedSpec& ss, const GenomeTable& gt, const char* const* d_ascii,
                            uint32_t* d_packed, int mode, bool key64, void* d_ckey, int msd_bits,
                            uint32_t* d_hist, uint32_t ntiles, uint32_t* d_err, hipStream_t st);
// packed path: scatter records into MSD buckets (offsets = scanned hist)
// side_bits > 0 (msd_bits 8, 2w+1 = 40 + side_bits): the key bits [32, 32 + side_bits) of every
// record go to d_side at the record's position (msd_split below)
hipError_t launch_seed_scatter(const SeedSpec& ss, const GenomeTable& gt, const uint32_t* d_packed, int msd_bits,
                               const uint32_t* d_hist_scanned, uint32_t ntiles, uint64_t* d_rec, hipStream_t st,
                               uint8_t* d_side = nullptr, int side_bits = 0);
// chunked mode (> 2^32 seed-mers), 33-bit record indices: only MSD digits [dlo, dlo + nbc)
// (d_cbase null), or every digit d at d_cbase[d >> mb] + its offset inside its chunk
hipError_t launch_seed_scatter_chunk(const SeedSpec& ss, const GenomeTable& gt, const uint32_t* d_packed, int msd_bits,
                                     const uint32_t* d_hist_slice, uint32_t ntiles, uint32_t dlo, uint32_t nbc,
                                     uint64_t* d_rec, hipStream_t st, const uint64_t* d_cbase = nullptr, int mb = 0,
                                     uint8_t* d_side = nullptr, int side_bits = 0);
// msdsplit.hip: every parent bucket (2^parent_bits, starts bstart_in) partitioned stably by
// its records' S-bit side digit -> 2^(parent_bits + S) buckets (starts bstart_out)
size_t msd_split_tmp_bytes(uint64_t n, int parent_bits);
hipError_t msd_split(const uint64_t* rin, const uint8_t* side, uint64_t* rout, uint64_t n, int parent_bits, int S,
                     const uint32_t* bstart_in, uint32_t* bstart_out, void* d_tmp, hipStream_t st);
// key of every position of one genome: ref_form = GetDnaSeedMer's left-aligned 64-bit mer
// (mums_copy_seed_keys), else the 2w+1-bit ckey (same order; one genome's SML sort)
hipError_t launch_keys_of_genome(const SeedSpec& ss, const uint32_t* d_words, uint64_t m, uint64_t* d_out,
                                 hipStream_t st, bool ref_form = true);

// scan.hip: exclusive scan of n uint32 values in place; d_tmp needs scan_tmp_bytes(n)
size_t scan_tmp_bytes(uint64_t n);
hipError_t exclusive_scan_u32(uint32_t* d_data, uint64_t n, void* d_tmp, uint32_t* d_total, hipStream_t st);

// radix_sort.hip: stable LSD radix sort of keys over bit range [0, bits); values are
// the implicit indices 0..n-1 when vals_in == nullptr.  ev_ds (optional): 2 events per
// pass around each downsweep launch.
size_t radix_tmp_bytes(uint64_t n);
template <typename K>
hipError_t radix_sort(const K* keys_in, const uint32_t* vals_in, uint64_t n, int bits,
                      K* kA, uint32_t* vA, K* kB, uint32_t* vB, void* d_tmp, int* out_buf,
                      hipStream_t st, hipEvent_t* ev_ds = nullptr);

// radix_seg.hip: segmented tiles + stable LSD sort of packed records on bits
// [32, 32 + key_bits) inside each MSD bucket.
uint64_t seg_tiles_upper(uint64_t n, int msd_bits, uint32_t tile = kSegTile);
size_t seg_tmp_bytes(uint64_t n, int msd_bits);
// chunks[3c .. 3c+2] = {src_off, dst_off, len}, sorted by dst_off, tiling [0, n)
hipError_t launch_regroup(const uint64_t* src, uint64_t* dst, const uint64_t* d_chunks, uint32_t nchunks, uint64_t n,
                          hipStream_t st);
hipError_t seg_bucket_starts(const uint32_t* d_hist_scanned, uint32_t T, int msd_bits, uint64_t n, uint32_t* bstart,
                             hipStream_t st);
hipError_t build_seg_tiles_from_starts(const uint32_t* bstart, int msd_bits, uint64_t n, SegTile* d_tiles,
                                       uint32_t* d_ntiles, void* d_tmp, hipStream_t st, uint32_t tile = kSegTile);
hipError_t build_seg_tiles(const uint32_t* d_hist_scanned, uint32_t T, int msd_bits, uint64_t n, SegTile* d_tiles,
                           uint32_t* d_ntiles, uint32_t* d_bstart, void* d_tmp, hipStream_t st);
hipError_t seg_radix_sort(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, const SegTile* d_tiles,
                          uint64_t ntiles_ub, void* d_tmp, int* out_buf, hipStream_t st,
                          hipEvent_t* ev_ds = nullptr);
// onesweep variant (n < 2^30): one histogram read for all passes, then one launch per
// pass with decoupled look-back between consecutive tiles of a bucket.
size_t onesweep_tmp_bytes(uint64_t n, int msd_bits, int key_bits);
// key_shift: first key bit of the records (32; 33 in the chunked mode)
hipError_t seg_onesweep_sort(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, int msd_bits,
                             const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, int* out_buf, hipStream_t st,
                             hipEvent_t* ev_ds = nullptr, int key_shift = 32, bool mask_parity = false,
                             bool key_runs = false, const uint32_t* hist_in = nullptr,
                             const uint64_t* gsrc = nullptr, uint32_t* gout = nullptr);
// gsrc / gout (key_runs only): the last pass writes gout[o] = low 32 bits of gsrc[low 32 bits of
// the record] instead of the record (a permutation gather at the store; the records of that
// pass are not written)
// hist_in: one bucket's digit histograms of every pass (npass x 256), counted by the records'
// producer: no histogram read of the records
// key_runs: the keys come in runs of equal digits (the line sort's hashes in x order): the
// histogram adds once per run and the passes publish their counts after the ranking
// mask_parity: the segment fix-up leaves key bit 0 (the parity / orientation bit) out of
// the last digit, so equal masked keys keep index order; seg_parity_fix then sorts every
// masked-key group of such a stream by that bit (d_tmp: seg_parity_fix_tmp_bytes(n))
size_t seg_parity_fix_tmp_bytes(uint64_t n);
hipError_t seg_parity_fix(uint64_t* rec, uint64_t* scratch, uint64_t n, int key_bits, int msd_bits,
                          const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, hipStream_t st, int key_shift = 32);
// onesweep launches of seg_onesweep_sort for key_bits (the lowest digit of a >= 2-digit
// key is finished by the segment fix-up unless MUMS_DEV_SEGFIX=0)
int seg_onesweep_launches(int key_bits);
// radix_wide.hip (MUMS_DEV_SORT3 > 0): three 10-bit passes over key bits [1, key_bits) with
// the parity bit left unsorted (default tolerances; the 8-bit MSD scatter leaves 31 key bits)
bool seg_wide_sort_enabled();
int seg_wide_passes(int key_bits);
size_t onesweep_wide_tmp_bytes(uint64_t n, int msd_bits, int key_bits);
hipError_t seg_onesweep_sort_wide(uint64_t* recA, uint64_t* recB, uint64_t n, int key_bits, int msd_bits,
                                  const uint32_t* d_bstart, void* d_tmp, uint32_t* d_err, int* out_buf,
                                  hipStream_t st, hipEvent_t* ev_ds, int key_shift = 32);

// groups.hip
uint64_t group_slot_count(uint64_t ntiles);
// probe-stage workgroups (= tile_count entries) for ntiles tiles (packed records: split tiles)
uint64_t group_blocks(uint64_t ntiles, bool packed);
template <int MG, typename View>
hipError_t launch_probe_tiles(View v, const SegTile* tiles, uint64_t ntiles, uint64_t N, const GenomeTable& gt,
                              const MatchParams& mp, int L, uint32_t* tile_count, uint64_t* slot_info,
                              uint32_t* slot_bucket, void* counters, hipStream_t st);
hipError_t launch_probe_compact(uint64_t nblocks, const uint32_t* tile_count, const uint32_t* tile_off,
                                const uint64_t* slot_info, const uint32_t* slot_bucket, uint64_t* probe_info,
                                uint32_t* probe_bucket, hipStream_t st, bool packed);
// the bucket partition of the probes as packed records (bucket << 32 | probe) and back
hipError_t launch_bucket_records(const uint32_t* b, uint64_t P, uint64_t* rec, hipStream_t st);
hipError_t launch_bucket_split(const uint64_t* rec, uint64_t P, uint32_t* b, uint32_t* ids, hipStream_t st);
// probes (key order) -> materialized rows (MatProbes, match_device.h)
template <int MG, typename View>
// lkey / fsk (optional): each probe's line key (chain_lkey_slot) and first-genome start;
// with lhash the line sort's first records (x << 32 | k) go to lkey and the line hashes to
// lhash (chain_line_slots)
hipError_t launch_materialize(View v, const uint64_t* probe_info, uint64_t P, const GenomeTable& gt,
                              const MatchParams& mp, int L, int64_t* rows, hipStream_t st, uint64_t* lkey = nullptr,
                              uint32_t* fsk = nullptr, uint32_t* lhash = nullptr, int32_t* rows32 = nullptr);
// rows32 (MG a multiple of 4 up to 16, fsk given): the rows as int32 starts instead
// (MatProbes::rows32); fsk[P] |= 1 when a start or the recomputed offset does not fit
// hash bucket of every row (d_bounds == nullptr) or its owning rank (bucket ranges)
hipError_t launch_row_buckets(const int64_t* rows, uint64_t P, int G, uint32_t table_size, const uint32_t* d_bounds,
                              uint32_t nranks, uint32_t* out, hipStream_t st);
hipError_t launch_gather_rows(const int64_t* src, const uint32_t* perm, uint64_t P, int G, int64_t* dst,
                              hipStream_t st);
// sharded FindMatches with chains labelled on the probes' own rank (mums_shard_chain_*):
// chain destinations (the rank of the chain's first probe), an inverse permutation, every
// exported row's entry index inside its destination block, and the exported entries with
// their first probe's index inside the destination's row block
// a sharded rank's merged records (local MSD buckets, starts d_bst[0..nb]) as (full key,
// 32-bit index) pairs for the group scans of pairwise.hip
hipError_t launch_rec_pairs(const uint64_t* rec, uint64_t n, const uint32_t* d_bst, uint32_t nb, uint32_t kfirst,
                            int kb_rec, uint64_t* key, uint32_t* idx, hipStream_t st);
// the same for 33-bit records (above 2^32 seed-mers): 64-bit indices
hipError_t launch_rec_pairs33(const uint64_t* rec, uint64_t n, const uint32_t* d_bst, uint32_t nb, uint32_t kfirst,
                              int kb_rec, uint64_t* key, uint64_t* idx, hipStream_t st);
hipError_t launch_chain_dest(const uint32_t* fk, uint64_t nch, const uint32_t* pdest, uint32_t* cdest, hipStream_t st);
hipError_t launch_inverse_perm(const uint32_t* perm, uint64_t n, uint32_t* inv, hipStream_t st);
hipError_t launch_chain_tags(const uint32_t* chain_of, const uint32_t* perm, const uint32_t* sdest, uint64_t P,
                             const uint32_t* cinv, const uint32_t* cstart, uint32_t* tags, hipStream_t st);
hipError_t launch_chain_entries_out(const int64_t* pool, const uint32_t* fk, const uint32_t* cperm,
                                    const uint32_t* scdest, uint64_t nch, int G, const uint32_t* pinv,
                                    const uint32_t* rstart, int64_t* eout, uint32_t* fout, hipStream_t st);
// the kept-probe export (groups.hip): per probe its destination (pdest when the owner's replay
// needs it, nranks + pdest when it collides), the first sorted position of every destination,
// and per exported entry its first sent row inside its destination's row block
hipError_t launch_kept_dest(const int64_t* rows, uint64_t P, int G, const uint32_t* chain_of, const uint32_t* cinv,
                            const uint2* thr, const uint32_t* fk, const uint32_t* pdest, uint32_t nranks, uint32_t* dest,
                            hipStream_t st);
hipError_t launch_dest_first(const uint32_t* sdest, uint64_t P, uint32_t* first, hipStream_t st);
hipError_t launch_entry_first(const uint32_t* scdest, uint64_t nch, const uint32_t* rcount, const uint32_t* perm,
                              const uint32_t* sdest, uint64_t K, const uint32_t* chain_of, const uint32_t* cinv,
                              const uint32_t* rstart, uint32_t* efirst, hipStream_t st);
// flat tiles over [0, N) for the pair path (one bucket)
hipError_t launch_flat_tiles(uint64_t N, SegTile* d_tiles, hipStream_t st);

// replay.hip
hipError_t launch_bucket_ranges(const uint32_t* sb, uint64_t P, uint32_t* bstart, uint32_t* bend, uint32_t* d_max,
                                hipStream_t st);
// the replay from the probes in key order (rows v, chain_of, fk = each chain's first probe):
// kept probes (chain-first / suspicious) bucket-sorted, summarised and replayed; the bucket
// vectors in *tbl_out at bases *base_out (allocated through alloc)
template <int MG, typename View>
hipError_t launch_replay_kept(View v, const GenomeTable& gt, const MatchParams& mp, int L, uint64_t P,
                              const int64_t* pool, const uint32_t* chain_of, const uint32_t* fk, uint32_t nch,
                              void* d_tmp, void* d_radix_tmp, void* d_scan_tmp, uint32_t lds_cap, uint32_t* tsize,
                              void* ctr, uint64_t* dbg, hipStream_t st, uint64_t* mlog, uint32_t** tbl_out,
                              const uint32_t** base_out, void* (*alloc)(void*, size_t), void* alloc_ctx,
                              const uint32_t* jl = nullptr);
// chains.hip: chain labelling of the probes (key order) before the replay
// context accessors for the multi-GPU orchestration (shard_comm.hip; mums_capi.hip)
}  // namespace mums
struct mums_ctx;
namespace mums {
hipStream_t ctx_stream(mums_ctx* ctx);
int ctx_device(mums_ctx* ctx);
int ctx_table_genomes(mums_ctx* ctx, uint32_t* table_size, uint32_t* genomes);
uint32_t ctx_repeat_tol(mums_ctx* ctx);
bool ctx_merge_chunked(mums_ctx* ctx);   // the last shard merge ran in key chunks
bool ctx_tie_all(mums_ctx* ctx);         // every run of equal keys in std::sort order (repeat / enum tol)
// ParallelMemHash compat over ranks (shard_comm.hip compat_shard_run; mums_capi.hip)
bool ctx_pcompat(mums_ctx* ctx);
// the shard layout of a compat context: owned genomes [*first, *first + *nown) of lens
int ctx_compat_layout(mums_ctx* ctx, uint32_t* first, uint32_t* nown, std::vector<uint64_t>* lens);
// the compat search of chunk range rank / ranks over all genomes (device ASCII) on the
// context's rank sub-context
int ctx_compat_rank_find(mums_ctx* ctx, const char* const* d_ascii, const uint64_t* lens, int G, uint32_t rank,
                         uint32_t ranks, int stage);
// the rank's table: per-bucket counts (table_size words) and, with d_rows, its rows in bucket order
int ctx_compat_rank_export(mums_ctx* ctx, uint64_t* bucket_counts, int64_t* d_rows, uint64_t* M);
// re-add W sources' rows (rank order; source s holds counts[s * nb + j] rows of bucket j of this
// owner's nb buckets, in bucket order) into this context's MatchList
int ctx_compat_rank_merge(mums_ctx* ctx, const int64_t* d_rows, uint32_t W, const uint64_t* counts, uint32_t nb);

// overlaps.hip: EliminateOverlaps (Aligner.cpp:62-176) on a device MatchList
struct EoWork {
    void *K = nullptr, *V = nullptr, *V2 = nullptr, *fl = nullptr, *fr = nullptr, *Lpos = nullptr, *Rpos = nullptr;
    void *bound = nullptr, *segA = nullptr, *segB = nullptr, *act = nullptr, *heap = nullptr, *piv = nullptr;
    void *nsw = nullptr, *scratch = nullptr, *plen = nullptr, *ps = nullptr, *nm_key = nullptr, *nm_id = nullptr;
    void *nk2 = nullptr, *nv2 = nullptr, *nk3 = nullptr, *nv3 = nullptr, *radix = nullptr, *ctr = nullptr;
    uint64_t cap_n = 0, cap_pool = 0, cap_new = 0, pool_n = 0, n_final = 0;
    unsigned long long hbuf[8] = {};
    EoWork() = default;
    EoWork(const EoWork&) = delete;
    EoWork& operator=(const EoWork&) = delete;
    ~EoWork();
    void release();
};
// the result stays in w (pool + ids) until eo_gather writes it out (*M_out matches)
hipError_t eliminate_overlaps_device(EoWork& w, const uint64_t* d_len, const int64_t* d_s, uint64_t M, int G,
                                     uint64_t* M_out, hipStream_t st);
hipError_t eo_gather(EoWork& w, int G, uint64_t* d_len_out, int64_t* d_s_out, hipStream_t st);
// libstdc++ std::sort replay of ids 0..n-1 by d_keys (test entry point); depth_override >= 0
// forces __introsort_loop's depth limit
hipError_t eo_sort_ids(EoWork& w, const uint64_t* d_keys, uint32_t n, int depth_override, uint32_t* d_ids_out,
                       hipStream_t st);

size_t chain_tmp_bytes(uint64_t P, uint32_t Tb, int G);
// chunked FindMatches: chain ids of a slice shifted past the slices before it, then the
// per-slice chain entries merged by content (chain_of remapped, *d_nchains = merged count)
hipError_t launch_add_offset(uint32_t* a, uint64_t n, uint32_t off, hipStream_t st);
size_t chain_merge_tmp_bytes(uint64_t n);
// the bucket owner's answer to the sharded kept-probe export (replay.hip): the n received chain
// entries merged into pool_out (*h_nchains chains), thr[e] = {next_s of entry e's chain, 1 when e
// is the chain's first received entry}; d_tmp: chain_thr_tmp_bytes(n), d_radix_tmp:
// radix_tmp_bytes(n + 1), d_scan_tmp: scan_tmp_bytes(n)
size_t chain_thr_tmp_bytes(uint64_t n);
hipError_t launch_chain_thresholds(const int64_t* entries, uint64_t n, const GenomeTable& gt, const MatchParams& mp,
                                   int64_t* pool_out, void* d_tmp, void* d_radix_tmp, void* d_scan_tmp,
                                   uint32_t* d_nchains, uint32_t* h_nchains, uint2* thr, hipStream_t st);
// fk_out[merged chain] = min of fk_loc over its per-slice chains
hipError_t launch_chain_merge(const int64_t* pool_loc, uint64_t n, int G, uint32_t* chain_of, uint64_t P,
                              int64_t* pool_out, void* d_tmp, void* d_radix_tmp, void* d_scan_tmp, uint32_t* d_nchains,
                              hipStream_t st, const uint32_t* fk_loc, uint32_t* fk_out);
// radix scratch of launch_chains / launch_chains_stream for P probes (the line sort)
size_t chain_radix_tmp_bytes(uint64_t P);
template <int MG, typename View>
hipError_t launch_chains(View v, const uint64_t* probe_info, uint64_t P, const GenomeTable& gt, const MatchParams& mp,
                         const SeedSpec& ss, const uint32_t* packed, void* d_chain_tmp, void* d_scan_tmp,
                         void* d_radix_tmp, uint32_t* chain_of, int64_t* pool, uint32_t* d_nchains, hipStream_t st,
                         void* ctr, hipEvent_t* ev_walk, uint32_t* fk, uint32_t kbase, bool lkey_ready = false,
                         uint32_t* jl = nullptr);
// jl (3 P words, optional): per line position j the chain, the probe (key order) and its
// first-genome start -- the replay's keep pass then reads them in line order and chain_of
// (a random scatter) is not written (chain_of may be null)
// where launch_chains(d_chain_tmp, P probes, G) reads the line keys from: a producer that
// writes them there (launch_materialize) lets launch_chains skip its key pass (lkey_ready)
uint64_t* chain_lkey_slot(void* d_chain_tmp, uint64_t P, int G);
// whether launch_chains orders the lines by the onesweep records (given DevCounters); then a
// producer writes (x << 32 | k) and the line hashes into chain_line_slots instead
bool chain_line_records(uint64_t P, const GenomeTable& gt);
void chain_line_slots(void* d_chain_tmp, uint64_t P, int G, uint64_t** rec, uint32_t** lhash);
hipError_t launch_emit(const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl, const int64_t* pool, int G,
                       uint32_t table_size, uint64_t M, uint64_t* out_len, int64_t* out_s, hipStream_t st);

// sml_tools.hip: SeedOccurrenceList and MatchList filters
size_t occ_tmp_bytes(uint64_t m);
hipError_t launch_seed_occurrence(const uint64_t* sk, const uint32_t* sv, uint64_t m, uint64_t n, int L, void* d_tmp,
                                  float* out, hipStream_t st);
hipError_t launch_unpack(const uint32_t* words, uint64_t n, char* out, hipStream_t st);
size_t filter_tmp_bytes(uint64_t M);
hipError_t launch_match_filter(const uint64_t* len, const int64_t* s, uint64_t M, int G, uint32_t mult,
                               uint64_t min_len, void* d_tmp, uint32_t* d_kept, uint64_t* len2, int64_t* s2,
                               hipStream_t st);

// pairwise.hip: PairwiseMatchFinder probe rows (PairwiseMatchFinder.cpp:37-73)
template <typename View>
hipError_t launch_pairwise_count(View v, uint64_t N, const GenomeTable& gt, uint32_t* npairs, void* ctr,
                                 hipStream_t st);
template <typename View>
hipError_t launch_pairwise_emit(View v, uint64_t N, const GenomeTable& gt, int L, const uint32_t* npairs,
                                const uint32_t* off, int64_t* rows, hipStream_t st);

// chunked.hip: records per MSD digit (chunked mode, > 2^32 seed-mers)
hipError_t launch_digit_totals(const uint32_t* hist, uint32_t ndigits, uint32_t T, unsigned long long* out,
                               hipStream_t st);

// MemHash with enumeration tolerance > 1 (any: slot kernels up to 8, group walks above):
// AddHashEntry calls per group, their rows
template <typename View>
hipError_t launch_enum_count(View v, uint64_t N, const GenomeTable& gt, const MatchParams& mp, uint32_t* ncalls,
                             void* ctr, hipStream_t st);
template <typename View>
hipError_t launch_enum_emit(View v, uint64_t N, const GenomeTable& gt, const MatchParams& mp, int L,
                            const uint32_t* ncalls, const uint32_t* off, int64_t* rows, hipStream_t st);

// pairwise.hip: a chunked-mode chunk (RecViewT<33>, nb + 1 bucket starts, bucket j = implicit
// digit digit0 + j) as (full ckey, 64-bit index) pairs for the enumeration kernels
hipError_t launch_chunk_pairs(const uint64_t* rec, uint64_t n, const uint32_t* bstart, uint32_t nb, uint64_t digit0,
                              uint64_t* key, uint64_t* idx, hipStream_t st);

// compat.hip: ParallelMemHash chunk-compat mode (ParallelMemHash.cpp:42-121)
hipError_t launch_genome_keys(uint64_t* ckey, uint64_t N, const GenomeTable& gt, int kbits, hipStream_t st);
hipError_t launch_compat_breaks(const uint64_t* sk, const GenomeTable& gt, uint64_t kmask, int mx, uint64_t chunk,
                                uint64_t* cs, uint64_t* bm, uint32_t cap, uint32_t* d_nch, uint32_t* err,
                                hipStream_t st);
hipError_t launch_compat_find(const uint64_t* sk, const GenomeTable& gt, uint64_t kmask, int mx, int L, uint64_t* cs,
                              const uint64_t* bm, uint32_t nch, hipStream_t st);
hipError_t launch_compat_chunk_keys(const uint64_t* sk, const uint32_t* sv, uint64_t N, const GenomeTable& gt,
                                    int kbits, const uint64_t* cs, uint32_t nch, uint64_t* key2, uint32_t* val2,
                                    uint64_t* ck, hipStream_t st);
hipError_t launch_compat_cands(const uint64_t* key2, uint64_t N, uint64_t* list, unsigned long long* cnt, uint64_t cap,
                               hipStream_t st);
hipError_t launch_compat_fire(const restart::PlanData& d, const uint64_t* key2, uint64_t N, int kbits,
                              const uint64_t* cand, uint64_t C, const uint64_t* cs, uint32_t nch, uint32_t* out,
                              uint64_t* cend, uint64_t* cons, hipStream_t st);
// out[j] = in[j] & mask (the genome-major SML keys without the genome bits)
hipError_t launch_compat_strip(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t mask, hipStream_t st);
hipError_t launch_compat_recs(const uint64_t* key2, const uint32_t* idx, uint64_t n, int kbits, uint64_t* rec,
                              uint32_t* clash, uint32_t* scratch, void* scan_tmp, bool force_scan, uint64_t* list,
                              unsigned long long* cnt, uint64_t cap, hipStream_t st);
hipError_t launch_compat_split(const uint64_t* sk, const GenomeTable& gt, const uint64_t* cs, uint32_t nch,
                               uint32_t* out, hipStream_t st);
hipError_t launch_compat_probe_chunks(const uint64_t* probe_info, uint64_t P, const uint64_t* key2, int kbits,
                                      uint32_t nch, uint32_t* pfirst, hipStream_t st);
hipError_t launch_compat_drop(const uint64_t* k_in, const uint32_t* v_in, uint64_t N, const uint64_t* rlo,
                              const uint64_t* rhi, const uint64_t* rpre, uint32_t R, uint64_t* k_out, uint32_t* v_out,
                              hipStream_t st);
hipError_t launch_compat_merge(uint32_t* tsize, const uint32_t* bstart, uint32_t* tbl, const int64_t* pool, int G,
                               uint32_t Tb, unsigned long long* collisions, const uint32_t* tscan, uint64_t total,
                               uint32_t* first_fail, hipStream_t st);
hipError_t launch_compat_merge_from(uint32_t* tsize, const uint32_t* bstart, uint32_t* tbl, const int64_t* pool, int G,
                                    uint32_t nb, const uint32_t* first_fail, unsigned long long* collisions,
                                    hipStream_t st);
// [first, last) records of the chunk-major stream (key2 sorted) in chunks [c0, c1): out[0..1]
hipError_t launch_compat_chunk_span(const uint64_t* key2, uint64_t n, int kbits, uint32_t c0, uint32_t c1,
                                    uint64_t* out, hipStream_t st);

// compat_ranks.hip: the ranks' compat tables re-added rank after rank at the bucket owners
// (pool rows int64 [len, offset, s_0 .. s_{G-1}]; per-bucket offsets nb + 1 words)
hipError_t launch_rank_rows(const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl, const int64_t* pool,
                            int G, uint32_t Tb, uint64_t M, int64_t* rows, hipStream_t st);
hipError_t launch_rank_lb(const int64_t* pool, int G, uint32_t nA, const uint32_t* offA, const uint32_t* offB,
                          uint32_t nb, uint32_t nB, uint32_t* lbA, uint32_t* nd, uint32_t* bad, hipStream_t st);
hipError_t launch_rank_place(const int64_t* pool, int G, uint32_t nA, const uint32_t* offA, const uint32_t* offB,
                             uint32_t nb, uint32_t nB, const uint32_t* lbA, const uint32_t* ndp, uint32_t* catoff,
                             uint32_t* tsize, uint32_t* tblcat, hipStream_t st);
hipError_t launch_rank_check(const int64_t* pool, int G, const uint32_t* catoff, const uint32_t* tsize, uint32_t nb,
                             uint32_t ncat, const uint32_t* tblcat, uint32_t* bad, hipStream_t st);
hipError_t launch_rank_exact_init(uint32_t nA, const uint32_t* offA, const uint32_t* offB, const uint32_t* catoff,
                                  uint32_t nb, uint32_t ncat, const uint32_t* bad, uint32_t* tblcat, uint32_t* tsize,
                                  uint32_t* first_fail, hipStream_t st);
hipError_t launch_rank_gather(const int64_t* pool, int G, const uint32_t* catoff, const uint32_t* tsize, uint32_t nb,
                              uint32_t ncat, const uint32_t* tblcat, const uint32_t* newoff, int64_t* out,
                              hipStream_t st);
hipError_t launch_rank_list(const int64_t* rows, int G, uint64_t M, uint64_t* out_len, int64_t* out_s, hipStream_t st);

// restart.hip: MER_REPEAT_LIMIT restart (MatchFinder.cpp:253-277) / start points
// (MemHash.cpp:117-127) as a fix-up of the merged stream
struct RsStream {
    int kind;                  // 0: packed records, 1: (u32 ckey, idx) pairs, 2: (u64 ckey, idx) pairs
    const uint64_t* rec;       // kind 0
    const uint32_t* bstart;    // kind 0: 2^B + 1 MSD bucket starts
    int B, kbits;              // kind 0: MSD bits, 2w+1
    const void* key;           // kind 1/2
    const uint32_t* idx;
};
struct RestartWs {             // workspace carved from one device buffer
    uint64_t* ckf;             // full ckey per stream record
    uint64_t* ck;              // ckeys genome-major (the G SortedMerLists)
    uint32_t* gen;             // genome per stream record
    uint32_t* inv;             // genome-major slot per stream record
    uint32_t *kA, *kB, *vA, *vB;
    uint64_t* dm;              // SMLLength per genome
    uint64_t* dbase;           // first genome-major slot per genome
    void* tmp;
    size_t bytes;
};
RestartWs restart_ws_layout(void* base, uint64_t n, int G);
size_t restart_ws_bytes(uint64_t n, int G);
hipError_t launch_restart_smls(const RsStream& s, uint64_t n, const GenomeTable& gt, const RestartWs& w,
                               hipStream_t st);
hipError_t launch_restart_cands(const RestartWs& w, uint64_t n, uint64_t* d_list, unsigned long long* d_cnt,
                                uint64_t cap, hipStream_t st);
// d_pre: 3 * C * G uint64 + C int; d_S: G start points in / last phase's out
hipError_t launch_restart_plan(const RestartWs& w, int G, const uint64_t* d_cand, uint64_t C, uint64_t* d_pre,
                               uint64_t* d_S, restart::PlanOut* d_out, hipStream_t st);
// the sharded mode's distributed plan (PlanData with off / n / prv / nxt; cbad: C flags)
hipError_t launch_restart_dpre(const restart::PlanData& d, const uint64_t* d_cand, uint64_t C, uint64_t* d_pre,
                               unsigned* cbad, hipStream_t st);
hipError_t launch_restart_dplan(const restart::PlanData& d, const uint64_t* d_cand, uint64_t C, const uint64_t* d_pre,
                                const unsigned* cbad, uint64_t* d_S, restart::PlanOut* d_out, hipStream_t st);
// live records (SML index >= start point of their key's phase) compacted in order into
// dst (records, or keys + dst_idx); kind 0 also writes the new bucket starts
// LogProgress tie groups (w.ck / w.dm / w.dbase): ord[i * G ..] = head order of the genomes
// gu[i] at masked key gk[i] in phase gp[i] (start points Sall[gp * G ..]), -1 padded
hipError_t launch_tie_heads(const RestartWs& w, int G, const uint64_t* gk, const uint64_t* gu, const uint32_t* gp,
                            const uint64_t* Sall, uint64_t ng, int* ord, hipStream_t st);
hipError_t launch_restart_compact(const RsStream& s, uint64_t n, int G, const RestartWs& w, const uint64_t* d_rkey,
                                  uint64_t R, const uint64_t* d_rS, const uint64_t* d_S0, void* dst_a, uint32_t* dst_idx,
                                  uint32_t* dst_bstart, uint32_t* d_total, hipStream_t st);

// bucket starts through a compaction's exclusive scan: out[b] = pos[bstart[b]], b <= nb
hipError_t launch_map_starts(const uint32_t* bstart, uint32_t nb, const uint32_t* pos, uint32_t* out, hipStream_t st);

// chunked.hip: MER_REPEAT_LIMIT restarts / start points over the resident chunked stream
struct CrStream {
    const uint64_t* rec;       // N sorted records (key_low << ib | index), MSD digit implicit
    const uint64_t* dstart;    // 2^B + 1 global MSD digit starts
    uint32_t nd;               // 2^B
    uint64_t N;
    uint32_t kb = 31, ib = 33; // key bits / index bits per record (chunked mode: 31 / 33)
};
uint64_t cr_blocks(uint64_t N);
// gcnt: G x (cr_blocks(N) + 1) per-genome block counts, exclusive-scanned per genome
hipError_t launch_cr_counts(const CrStream& s, const GenomeTable& gt, uint32_t* gcnt, void* d_scan_tmp, hipStream_t st);
// the SMLs as (genome << kbits | ckey, index) pairs at gt.base[g] + SML index (compat.hip's input)
hipError_t launch_cr_partition(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int kbits, uint64_t* sk,
                               uint32_t* sv, uint64_t* ck, hipStream_t st);
// ParallelMemHash's chunk-major stream (key2 = chunk << kbits | ckey, index) as a stable
// partition of the sorted stream by chunk (cs: nch x G chunk starts); cnt: cr_chunk_part_cnt_words
// u32 scratch; only when cr_chunk_part_fits
size_t cr_chunk_part_cnt_words(uint64_t N, uint32_t nch);
bool cr_chunk_part_fits(uint64_t N, uint32_t nch);
hipError_t launch_cr_chunk_part(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* cs,
                                uint32_t nch, int kbits, uint32_t* cnt, void* d_scan_tmp, uint64_t* key2, uint32_t* idx,
                                hipStream_t st);
// The same stream as compat_recs' packed records in one pass (no key2 / index arrays) when every
// block boundary of the sorted stream is closed under the chunk-major order; ws: cr_direct_ws_bytes.
// *flags (host, after a stream sync) = 0: rec holds all N records; else the reason the caller
// takes the partition + compat_recs path (1 open boundary, 2 group-key clash, 4 a masked-key run
// above MER_REPEAT_LIMIT, 8 too many chunks in one unit).
// ParallelMemHash chunk starts cs[k * G + g] (k = 1 .. nch - 1; row 0 the caller's) from the
// sorted stream when no break walks back; *flags (4 B device) 0 = cs complete and no chunk start
// splits an equal-key run, else the caller builds the genome-major SMLs (compat.hip kernels)
hipError_t launch_compat_fast_chunks(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int mx,
                                    uint64_t chunk, int L, uint32_t nch, uint64_t* cs, uint32_t* flags, hipStream_t st);
// k2 (N u64) and sc (N bytes): scratch of the units that hold chunk starts or open boundaries.
size_t cr_direct_ws_bytes(uint64_t N);
hipError_t launch_cr_compat_direct(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* cs,
                                   uint32_t nch, int kbits, uint64_t* rec, uint64_t* k2, uint8_t* sc, void* ws,
                                   uint32_t* flags, hipStream_t st);
hipError_t launch_cr_ck(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, uint64_t* ck, hipStream_t st,
                        const uint64_t* lbase = nullptr);
// masked key of genome g's SML index e for every query g << 56 | e (gscan from launch_cr_counts)
hipError_t launch_cr_query(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* q, uint64_t nq,
                           uint64_t* out, hipStream_t st);
// the same from genome-major SMLs (ck[base[g] + e])
hipError_t launch_cr_ck_query(const uint64_t* ck, const GenomeTable& gt, const uint64_t* q, uint64_t nq, uint64_t* out,
                              hipStream_t st);
hipError_t launch_cr_cands(const CrStream& s, uint64_t* list, unsigned long long* cnt, uint64_t cap, hipStream_t st);
hipError_t launch_cr_runs(const uint64_t* ck, const GenomeTable& gt, const uint64_t* sp, uint64_t rows, uint64_t* runs,
                          unsigned long long* nr, uint64_t cap, hipStream_t st);
hipError_t launch_cr_kpos(const CrStream& s, const GenomeTable& gt, int g, uint64_t* K, hipStream_t st);
// repeat tolerance: genome g's records in flagged runs (tie replay slot flags ts, ids V) take
// the std::sort order's ids
// sharded repeat tolerance: pair flags of a rank's SML parts at out[gofs[g] + i]; ids from
// V[vofs[g] + i] (~0 keeps the id)
hipError_t launch_cr_pair_flags(const uint64_t* ck, int G, const uint64_t* lbase, const uint64_t* gofs, uint64_t n,
                                uint32_t* out, hipStream_t st);
hipError_t launch_cr_tie_vals(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, const uint64_t* vofs,
                              const uint32_t* V, uint64_t* rec, hipStream_t st);
hipError_t launch_cr_tie_all(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, int g, const uint32_t* ts,
                             const uint32_t* V, uint64_t* rec, hipStream_t st);
// a sharded rank's part of every SML (global indices [goff[g], goff[g] + gn[g]) at ck[lbase[g] ..]):
// straddled runs {g, lo, hi} (global indices) of the start points sp (rows x G), and the id
// rewrite of its runs from V[vofs[q] ..]
hipError_t launch_cr_druns(const uint64_t* ck, int G, const uint64_t* lbase, const uint64_t* goff, const uint64_t* gn,
                           const uint64_t* sp, uint64_t rows, uint64_t* runs, unsigned long long* nr, uint64_t cap,
                           hipStream_t st);
hipError_t launch_cr_dtie_write(const CrStream& s, const GenomeTable& gt, const uint64_t* runs, uint64_t nrun,
                                const uint64_t* ck, const uint64_t* lbase, const uint64_t* goff, const uint32_t* V,
                                const uint64_t* vofs, uint64_t* rec, hipStream_t st);
hipError_t launch_cr_tie_write(const CrStream& s, const GenomeTable& gt, int g, const uint64_t* runs, uint64_t nrun,
                               const uint64_t* ck, const uint32_t* V, uint64_t* rec, hipStream_t st);
hipError_t launch_cr_live_compact(const CrStream& s, const GenomeTable& gt, const uint32_t* gscan, uint64_t lo,
                                  uint64_t hi, const uint64_t* rkey, uint64_t R, const uint64_t* rS, const uint64_t* S0,
                                  uint32_t* live, uint32_t* pos, void* d_scan_tmp, uint64_t* dst,
                                  const uint32_t* bstart, uint32_t nb, uint32_t* dst_bstart, uint32_t* d_total,
                                  hipStream_t st, const uint64_t* goff = nullptr);

// smlsort.hip: the std::sort order of equal seed mers in every SortedMerList
// (MemorySML.cpp:54) for flagged runs.  Slot space = genome-major SML slots (= global
// seed-mer indices); flags: pf[t] = 1 when sorted slots t, t + 1 form a pair of a run that
// matters.  Usage: tie_set_genomes, tie_clear_flags, tie_mark_all / tie_mark_starts, K filled
// with the keys in position order (tie_scatter_keys), tie_prepare, tie_replay, then tie_writeback /
// tie_slots_out.
struct TieWs {
    uint64_t n;
    int G;
    uint64_t smax;                 // segment capacity per level
    uint32_t* pf;                  // pair flags (n + 1)
    uint32_t* ts;                  // exclusive scan of the slot flags (n + 1)
    uint64_t* K;                   // keys at the slots
    uint32_t* V;                   // seed-mer ids at the slots
    uint32_t *fl, *fr, *Lpos, *Rpos;
    uint8_t* bound;                // partition / genome bounds (leaf pass)
    void *segA, *segB, *heap;
    uint32_t *act, *off, *nsw, *ctr;
    uint64_t* piv;
    uint64_t *dbase, *dm;          // G + 1 slot bases, SML lengths
    void* tmp;
    size_t bytes;
};
TieWs tie_ws_layout(void* base, uint64_t n, int G);
size_t tie_ws_bytes(uint64_t n, int G);
hipError_t tie_set_genomes(const TieWs& w, const uint64_t* base, const uint64_t* m, hipStream_t st);
hipError_t tie_clear_flags(const TieWs& w, hipStream_t st);
hipError_t tie_mark_all(const TieWs& w, const uint64_t* ck, hipStream_t st);
// d_sp: rows x G start points (SML indices per genome)
hipError_t tie_mark_starts(const TieWs& w, const uint64_t* ck, const uint64_t* d_sp, uint64_t rows, hipStream_t st);
// K[global index of stream record j] = ckf[j] (rec: packed records, else idx)
hipError_t tie_scatter_keys(const TieWs& w, const uint64_t* ckf, const uint64_t* rec, const uint32_t* idx,
                            hipStream_t st);
// slot flags scanned; *flagged = slots of flagged runs (0: nothing to replay)
hipError_t tie_prepare(const TieWs& w, uint64_t* flagged, hipStream_t st);
hipError_t tie_replay(const TieWs& w, hipStream_t st);
// stream record j of a flagged run takes the id at its SML slot inv[j] (rec or idx)
hipError_t tie_writeback(const TieWs& w, uint64_t* rec, uint32_t* idx, const uint32_t* inv, hipStream_t st);
hipError_t tie_slots_out(const TieWs& w, uint32_t* out, hipStream_t st);

}  // namespace mums
