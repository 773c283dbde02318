/*
 * mums.h -- C ABI of the MI355X-native multi-MUM seed finder (libmums_hip.so).
 *
 * This is the drop-in boundary for libMems' MemHash / MaskedMemHash hot path
 * (koadman/libMems 1.6.1).  Each entry point names the reference interface it
 * replaces (paths relative to /root/reference/libMems/).  Plain pointers and
 * sizes only; no C++ exceptions cross this boundary: every call returns a
 * status code (MUMS_OK == 0) and mums_last_error() carries the message that
 * the reference would have thrown or printed.
 *
 * Threading (MemHash.h:38, Aligner.h:198 TLS<MemHash>): a context is used by
 * one host thread at a time; distinct contexts are independent and may be
 * used concurrently from different host threads.
 *
 * Coordinates (AbstractMatch.h:27, MemHash.cpp:176-177): match starts are
 * 1-based, signed (negative = reverse complement relative to the first
 * present genome), 0 = NO_MATCH.  Result order is the reference's
 * bucket-major MatchList order (MemHash.h:182-203).
 */
#ifndef MUMS_H
#define MUMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MUMS_ABI_VERSION 6

enum mums_status {
    MUMS_OK = 0,
    MUMS_E_INVALID = -1,      /* bad argument / inconsistent state (gnException InvalidData)        */
    MUMS_E_NOMEM = -2,        /* device allocation failed                                           */
    MUMS_E_HIP = -3,          /* HIP runtime error                                                  */
    MUMS_E_GAP = -4,          /* '-' in a genome: SortedMerList.cpp:433-437 throws "Gap in genome"  */
    MUMS_E_UNSUPPORTED = -5,  /* a feature outside the implemented scope (see mums_last_error)      */
    MUMS_E_NODEVICE = -6      /* no HIP device: the product path never falls back to the CPU        */
};

/* Run stages for mums_find_stage(). */
enum mums_stage {
    MUMS_STAGE_SEEDS = 1,     /* pack + keys + sort + merge/accept + probe build ("sorted+matched") */
    MUMS_STAGE_ALL = 2        /* + extension, bucket replay, MatchList materialisation (FindMatches)*/
};

typedef struct mums_ctx mums_ctx;

typedef struct mums_stats {
    uint64_t seedmers;          /* N = sum over genomes of SMLLength (SortedMerList.cpp:288-295)     */
    uint64_t groups;            /* distinct masked keys                                               */
    uint64_t probes;            /* accepted seed probes handed to AddHashEntry                        */
    uint64_t mem_count;         /* MemHash::MemCount()  (MemHash.h:94)                                */
    uint64_t collision_count;   /* MemHash::MemCollisionCount() (MemHash.h:97)                        */
    uint64_t repeat_limit_groups; /* groups larger than MER_REPEAT_LIMIT (MatchFinder.cpp:166)        */
    uint64_t nonempty_buckets;  /* hash buckets holding >= 1 entry                                    */
    double   ms_keys;           /* device time per phase of the last run (HIP events)                 */
    double   ms_sort;
    double   ms_groups;
    double   ms_buckets;
    double   ms_replay;
    double   ms_output;
    double   ms_total;
    /* dominant-kernel instrumentation (mums_set_profiling(ctx, 1)): HIP events
     * around every downsweep launch of the seed-key radix sort, on the
     * context's stream; bytes = algorithmic HBM bytes of those launches. */
    double   ms_dominant;
    uint64_t dominant_launches;
    uint64_t dominant_bytes;
    uint64_t key_bytes;         /* 4 (2w+1 <= 32) or 8 */
    uint64_t sort_passes;
    double   ms_chains;         /* seed-chain labelling before the replay (ExtendMatch results)        */
    uint64_t chains;            /* seed chains among the probes                                        */
    uint64_t chunks;            /* ParallelMemHash compat: SML chunks searched (ParallelMemHash.cpp:75-83) */
    uint64_t restarts;          /* MER_REPEAT_LIMIT restarts of the merge (MatchFinder.cpp:253-277)      */
    /* FindMatches' dominant kernel, chain_walk_kernel (ABI 5): HIP events around its launches
     * (mums_set_profiling), the 64-column hit words it evaluated, the walks it finished and
     * its algorithmic bytes: 28-B packed windows per word and present component + per walk
     * the probe row ((G + 1) x 8 B) and the queue item (24 B). */
    double   ms_chain_walks;
    uint64_t chain_walk_words;
    uint64_t chain_walks;
    uint64_t chain_walk_bytes;
    /* the same for chain_walk_short_kernel (ABI 6): every queued walk's first kWalkBudget
     * words, one lane per walk; the walks it hands on are counted again above. */
    double   ms_short_walks;
    uint64_t short_walk_words;
    uint64_t short_walks;
    uint64_t short_walk_bytes;
} mums_stats;

/* MemHash::MemHash (MemHash.cpp:33-49); device = HIP ordinal. */
int  mums_ctx_create(int device, mums_ctx** out);
/* MemHash::~MemHash */
int  mums_ctx_destroy(mums_ctx* ctx);
/* Optional: run on a caller-provided hipStream_t (default: a private stream). */
int  mums_set_stream(mums_ctx* ctx, void* hip_stream);

/* Seed pattern (SeedMasks.h getSeed, SortedMerList::Create seed argument,
 * SortedMerList.cpp:786-824).  0 = choose getDefaultSeedWeight() from the
 * mean genome length at find time (MatchList.h:351-357). */
int  mums_set_seed(mums_ctx* ctx, uint64_t pattern);
/* MemHash::SetRepeatTolerance / SetEnumerationTolerance (MemHash.h:125-144)
 * and MemHash::SetTableSize (MemHash.cpp:95-102). */
int  mums_set_params(mums_ctx* ctx, uint32_t repeat_tol, uint32_t enum_tol, uint32_t table_size);
/* MaskedMemHash (MaskedMemHash.h:25-40): masked=1 selects MaskedMemHash::HashMatch
 * semantics; seq_mask = MaskedMemHash::SetMask (genome 0 = most significant bit). */
int  mums_set_mask(mums_ctx* ctx, int masked, uint64_t seq_mask);
/* ParallelMemHash (ParallelMemHash.h:29-48, FindMatches ParallelMemHash.cpp:42-103):
 * enable=1 reproduces its chunked search -- SML chunks of chunk_size mers of the
 * longest SML cut by MatchFinder::GetBreakpoint (MatchFinder.cpp:89-126), searched
 * one by one, thread tables merged by MergeTable (:105-121) -- so the MatchList is
 * the (patched) OpenMP reference's.  chunk_size 0 = the
 * reference's CHUNK_SIZE 200000 (:51).  enable=0 = serial MemHash (default). */
int  mums_set_parallel_compat(mums_ctx* ctx, int enable, uint64_t chunk_size);
/* PairwiseMatchFinder (PairwiseMatchFinder.h:23-33): a MemHash whose EnumerateMatches
 * (PairwiseMatchFinder.cpp:37-73) hashes every pair of genomes occurring once in a seed
 * group instead of one multi-genome seed.  enable=0 = MemHash. */
int  mums_set_pairwise(mums_ctx* ctx, int enable);

/* MatchFinder::AddSequence (MatchFinder.cpp:59-87) for a host ASCII genome
 * (copied to HBM).  Genome ids are assigned in call order. */
int  mums_add_genome(mums_ctx* ctx, const char* ascii, uint64_t n);
/* Same for a device-resident ASCII genome (not copied; must outlive the find). */
int  mums_add_genome_device(mums_ctx* ctx, const void* d_ascii, uint64_t n);
/* The device copy of genome g this context holds (its ASCII in HBM, n bases): a deferred
 * SortedMerList (SortedMerList::Create, SortedMerList.cpp:786-824, recorded but not built;
 * mums::HipSML in mums_memhash.hpp) hands its genome to a MemHash context this way, through
 * mums_add_genome_device, without a host copy.  Valid until the context is cleared. */
int  mums_genome_device(mums_ctx* ctx, uint32_t genome, const void** d_ascii, uint64_t* n);
/* MemHash::Clear / ClearSequences (MemHash.cpp:80-93): drops genomes and results. */
int  mums_clear(mums_ctx* ctx);

/* MemHash::FindMatchesFromPosition (MemHash.cpp:117-127) -> FindMatchSeeds(start_points)
 * (MatchFinder.cpp:137-164): the merge of the next finds starts at SML index
 * start_points[g] of genome g (count = genome count; count 0 = from 0, FindMatches).
 * Single-context MemHash / MaskedMemHash / PairwiseMatchFinder only. */
int  mums_set_start_points(mums_ctx* ctx, const uint64_t* start_points, uint32_t count);
/* MatchFinder::SetOffsetLog (MatchFinder.h:81; written MatchFinder.cpp:152-162): the start
 * points after every MER_REPEAT_LIMIT restart of the last find, one row of genome-count
 * entries per restart.  *rows = row count, *seq_count = entries per row (may be NULL);
 * out (cap_rows rows) may be NULL to query. */
int  mums_get_offset_log(mums_ctx* ctx, uint64_t* out, uint64_t cap_rows, uint64_t* rows, uint32_t* seq_count);
/* MemHash::FindMatches(MatchList&) (MemHash.cpp:109-115) / CreateMatches (:104-107).
 * SearchRange's MER_REPEAT_LIMIT restart (MatchFinder.cpp:253-277) is reproduced
 * (mums_stats.restarts) in the single-context, chunked (> 2^32 seed-mers) and sharded
 * modes. */
int  mums_find(mums_ctx* ctx);
/* Run only up to a stage (benchmarks); MUMS_STAGE_ALL == mums_find. */
int  mums_find_stage(mums_ctx* ctx, int stage);

/* MemHash::GetMatchList (MemHash.h:182-203): number of matches and genomes. */
int  mums_result_count(mums_ctx* ctx, uint64_t* count, uint32_t* seq_count);
/* lengths[count]; starts[count * seq_count] row-major (match-major). */
int  mums_result_copy(mums_ctx* ctx, uint64_t* lengths, int64_t* starts);

/* MemHash::MemTableCount (MemHash.h:100; mem_table_count, MemHash.cpp:245): entries
 * inserted per hash bucket of the last FindMatches; counts[table_size]. */
int  mums_mem_table_count(mums_ctx* ctx, uint32_t* counts, uint32_t table_size);
/* MemCount / MemCollisionCount (MemHash.h:94-97) + per-phase device timings. */
int  mums_get_stats(mums_ctx* ctx, mums_stats* out);
/* Record HIP events around each dominant-kernel launch (adds a few us per run). */
int  mums_set_profiling(mums_ctx* ctx, int enable);
/* Message of the last failing call on this context ("" if none). */
const char* mums_last_error(mums_ctx* ctx);

/* ---- row A1-A5 helpers (seed table, keys, SortedMerList) ------------------ */
/* getSeed(weight, rank) (SeedMasks.h:298-321); SOLID_SEED == INT32_MAX. */
int64_t  mums_get_seed(int weight, int seed_rank);
/* getDefaultSeedWeight (SeedMasks.h:389-401). */
uint32_t mums_default_seed_weight(uint64_t avg_len);
/* GetDnaSeedMer for every position of genome g after mums_find_stage(>=SEEDS):
 * out[p] = canonical key (SortedMerList.cpp:764-769, 64-bit left-aligned form). */
int  mums_copy_seed_keys(mums_ctx* ctx, uint32_t genome, uint64_t* out, uint64_t cap);
/* Same for positions [first, first + count) only (sampling genomes of billions of bases). */
int  mums_copy_seed_keys_range(mums_ctx* ctx, uint32_t genome, uint64_t first, uint64_t count, uint64_t* out);
/* MemorySML::Create (MemorySML.cpp:45-60): SML positions of genome g sorted by
 * full key, equal keys in libstdc++ std::sort(bmer_lessthan) order. */
int  mums_build_sml(mums_ctx* ctx, uint32_t genome, uint32_t* positions, uint64_t cap);
/* SeedOccurrenceList::construct (SeedOccurrenceList.h:22-61) + smoothFrequencies
 * (:71-87) over genome's SortedMerList: freq[p] (float32, n entries) = mean masked-key
 * frequency of the seeds covering position p (getFrequency, :64-67). */
int  mums_seed_occurrence(mums_ctx* ctx, uint32_t genome, float* freq, uint64_t cap);
/* GenericMatchList::MultiplicityFilter / LengthFilter (MatchList.h:636-664) applied to
 * the context's last MatchList in place (order kept). */
int  mums_multiplicity_filter(mums_ctx* ctx, uint32_t multiplicity);
/* DNAFileSML (format version 5, DNAFileSML.h:58-62) writer, FileSML::Create's file
 * (FileSML.cpp:316-374): SMLHeader + 2-bit sequence words + SML positions, for genome g
 * of a context whose seed stage ran.  Readable by FileSML::LoadFile (FileSML.cpp:46-110)
 * so LoadSMLs callers (MatchList.h:261-349) reuse GPU-built SMLs. */
int  mums_write_sml(mums_ctx* ctx, uint32_t genome, const char* path, const char* description);
/* FileSML::LoadFile (FileSML.cpp:46-110) of such a file: its sequence becomes the next
 * genome of the context; *seed_out = the file's seed pattern (may be NULL). */
int  mums_add_genome_sml(mums_ctx* ctx, const char* path, uint64_t* seed_out);
int  mums_length_filter(mums_ctx* ctx, uint64_t min_length);
/* MemHash::SetMatchLog (MemHash.h:149): the reference writes every inserted entry to the
 * log stream as it inserts it (MemHash.cpp:238-241: `len\ts0\t...` per line, the order of
 * the AddHashEntry calls that inserted them).  Enable before mums_find; afterwards
 * mums_match_log_copy returns those entries in that order (*count first: lengths / starts
 * NULL).  ParallelMemHash compat (the patched 2-argument AddHashEntry of SURVEY.md B.3,
 * one OpenMP thread): per chunk its thread-table inserts in call order, then MergeTable's
 * inserts (ParallelMemHash.cpp:105-121) in bucket order -- every entry appears twice. */
int  mums_set_match_log(mums_ctx* ctx, int enable);
int  mums_match_log_copy(mums_ctx* ctx, uint64_t* lengths, int64_t* starts, uint64_t capacity, uint64_t* count);
/* MatchFinder::LogProgress (MatchFinder.h:80, MatchFinder.cpp:55-56,296-309): the reference
 * writes "N%.." to the log stream each time its merge crosses a whole percent of the mers
 * (counted per 10 000-mer buffer refill, a newline every ten).  Enable before mums_find; the
 * seed stage then restates that text (MER_REPEAT_LIMIT restarts and start points included;
 * single context and chunked mode with packed records, i.e. seed weight <= 21; ParallelMemHash
 * compat: every chunk's SearchRange in chunk order, the count set once for the whole loop,
 * ParallelMemHash.cpp:56-61) and mums_progress_log_copy returns it (*length = its size; text
 * NUL-terminated, may be NULL). */
int  mums_set_progress_log(mums_ctx* ctx, int enable);
int  mums_progress_log_copy(mums_ctx* ctx, char* text, uint64_t capacity, uint64_t* length);
/* EliminateOverlaps (libMems/Aligner.cpp:62-176, declared Aligner.h:239) on the context's
 * MatchList in place: per genome, std::sort by SingleStartComparator (AbstractMatch.h:324-351,
 * libstdc++ tie order reproduced), crop / delete the smaller of every overlapping pair,
 * append the cut-off overlaps without that genome (multiplicity > 1).  Same result and
 * order as the reference on the same MatchList. */
int  mums_eliminate_overlaps(mums_ctx* ctx);
/* The caller's MatchList (count x seq_count signed starts, NO_MATCH = 0, lengths) becomes
 * the context's result, for mums_eliminate_overlaps / the filters on lists that did not
 * come from this context's FindMatches (Aligner.cpp:920 gap_list, :1580 mlist). */
int  mums_load_matches(mums_ctx* ctx, uint32_t seq_count, uint64_t count, const uint64_t* lengths,
                       const int64_t* starts);
/* Test entry point: ids[0..n) = the permutation libstdc++ std::sort leaves on keys with
 * operator< (depth_override >= 0 forces the introsort depth limit; -1 = 2*lg(n)). */
int  mums_debug_std_sort(mums_ctx* ctx, const uint64_t* keys, uint64_t n, int depth_override, uint32_t* ids);

/* ---- sharded seed stage across GPUs -----------------------
 * Replaces the single-process G-way merge of MatchFinder::SearchRange
 * (MatchFinder.cpp:172-340) over the G SortedMerLists (MemorySML::Create,
 * MemorySML.cpp:45-60) when the genomes live on different GPUs; the result is
 * the same key-ordered stream of accepted probes as mums_find_stage(SEEDS).
 * One context per rank; the caller moves the records between ranks (RCCL
 * all-to-all over xGMI, libmems_amd/shard.py).
 *   1. mums_shard_layout: all G genome lengths; this context owns genomes
 *      [first_genome, first_genome + #mums_add_genome calls).
 *   2. mums_shard_keys: keys of the owned genomes as 8-B records
 *      (ckey_low << 32 | global seed-mer index), stably bucketed by the top
 *      msd_bits key bits into d_records; bucket_counts[2^msd_bits].
 *   3. exchange: bucket range [first_bucket, first_bucket + nbuckets) of every
 *      source rank goes to its owner rank, sources in rank order.
 *   4. mums_shard_merge: the received records (source-major: each source's
 *      buckets in order; counts[nsources][nbuckets]) -> sort -> groups ->
 *      probes of this key range; stats via mums_get_stats. */
int  mums_shard_layout(mums_ctx* ctx, uint32_t genomes_total, uint32_t first_genome, const uint64_t* lengths);
/* msd_bits of the exchange and the number of records mums_shard_keys will write. */
/* Position-sharded layout (BASELINE config 5 on 8 GPUs): the context's
 * one genome is the ASCII of genome `genome`'s bases [pos_begin, pos_end + L - 1) (L = seed
 * length, clipped at the genome end) and this rank owns its SML positions [pos_begin,
 * pos_end); records carry global seed-mer indices (33-bit above 2^32 seed-mers).  Seed
 * stage only (mums_shard_keys / mums_shard_merge). */
int  mums_shard_slice(mums_ctx* ctx, uint32_t genomes_total, const uint64_t* lengths, uint32_t genome,
                      uint64_t pos_begin, uint64_t pos_end);
int  mums_shard_msd_bits(mums_ctx* ctx, uint32_t* msd_bits, uint64_t* local_records);
int  mums_shard_keys(mums_ctx* ctx, uint64_t* d_records, uint64_t capacity, uint64_t* bucket_counts);
int  mums_shard_merge(mums_ctx* ctx, const uint64_t* d_records, uint32_t nsources, uint32_t first_bucket,
                      uint32_t nbuckets, const uint64_t* counts);
/* ---- sharded MER_REPEAT_LIMIT restart (MatchFinder::SearchRange, MatchFinder.cpp:253-277;
 * GetBreakpoint, :89-126) and FindMatchesFromPosition start points (MemHash.cpp:117-127;
 * FindMatchSeeds, MatchFinder.cpp:137-164), between mums_shard_merge and the probe /
 * FindMatches steps.  A restart moves the start points of every later key, i.e. of records
 * held by other ranks, and its plan reads whole SortedMerLists (FindMer, the head-order
 * walk), so one planner rank plans on the whole merged stream:
 *   1. mums_shard_restart_pending: > 0 when this rank's key range holds a group above
 *      MER_REPEAT_LIMIT or start points are set (mums_set_start_points: one per genome of
 *      the shard layout); when any rank reports one, the steps below are required;
 *   2. mums_shard_stream: this rank's merged stream (device records, count), gathered onto
 *      the planner in rank order (= key order);
 *   3. mums_shard_restart_plan (planner): d_stream = the gathered streams (ids of the runs a
 *      start point falls into are rewritten in place, std::sort order, MemorySML.cpp:54),
 *      counts = the keys stage's per-rank bucket counts [nranks][2^msd_bits], the key
 *      ranges; writes one block per rank into d_out (capacity >= 8 * (N + nranks *
 *      (2^msd_bits + 4)) bytes), block_bytes[r]; the restart log via mums_get_offset_log;
 *   4. mums_shard_restart_apply (every rank): its block + the planner's restart log ->
 *      the live records replace the stream and the groups stage runs again. */
int  mums_shard_restart_pending(mums_ctx* ctx, uint64_t* pending);
int  mums_shard_stream(mums_ctx* ctx, const void** d_records, uint64_t* n);
int  mums_shard_restart_plan(mums_ctx* ctx, uint64_t* d_stream, uint32_t nranks, const uint64_t* counts,
                             const uint32_t* first_bucket, const uint32_t* nbuckets, void* d_out,
                             uint64_t capacity_bytes, uint64_t* block_bytes);
int  mums_shard_restart_apply(mums_ctx* ctx, const void* d_block, uint64_t restarts, const uint64_t* offset_log);
/* The same restart planned where the records are (mums_shard_run's default; the gathered
 * plan above stays the fallback).  Rank r holds SML indices [off_r[g], off_r[g] + n_r[g])
 * of every genome g (off_r = the counts of lower ranks), so every SML read of the plan
 * (restart_plan.h) is answered locally, with the last key of genome g below the range and
 * the first above it as neighbours; a read beyond those flags the plan undecidable.
 *   1. mums_shard_restart_counts: this rank's SML parts (local genome-major keys), info =
 *      [n[G], first key[G], last key[G], status] (status 1: use the gathered plan);
 *   2. mums_shard_restart_prepare: every rank's info (all-gathered, rank order) -> offsets,
 *      neighbours, the per-candidate precompute (cand_precompute); S0 = the start points;
 *   3. mums_shard_restart_step, one rank after the other: the plan over this rank's
 *      candidates with the running start points S (in/out), its restart count and the
 *      undecidable flag (any rank: every rank falls back before anything is changed);
 *      mums_shard_restart_log copies its restarts (keys, start points R x G);
 *   4. mums_shard_restart_runs: the runs of equal keys that the start points of every phase
 *      (S0 + all ranks' restarts, in key order) fall into on this rank, {g, lo, hi} global;
 *   5. mums_shard_restart_ties (rank g % world for genome g): std::sort order of genome g's
 *      runs (smlsort.hip) from the all-gathered packed genomes; the positions of run q's
 *      slots to d_out + vofs[q];
 *   6. mums_shard_restart_finish: this rank's runs take those positions as ids; the live
 *      records (SML index >= its phase's start point) replace the stream, groups again.
 * mums_shard_restart_info: [path (1 local plan, 2 gathered plan), candidates, restarts,
 * device bytes the restart allocated on this rank]. */
int  mums_shard_restart_counts(mums_ctx* ctx, uint64_t* info);
int  mums_shard_restart_prepare(mums_ctx* ctx, uint32_t nranks, uint32_t rank, const uint64_t* all_info,
                                uint64_t* S0);
int  mums_shard_restart_step(mums_ctx* ctx, uint64_t* S, uint64_t* restarts, uint64_t* undecidable);
int  mums_shard_restart_log(mums_ctx* ctx, uint64_t* rkey, uint64_t* rS);
int  mums_shard_restart_runs(mums_ctx* ctx, uint64_t restarts, const uint64_t* rkey, const uint64_t* rS,
                             uint64_t* runs, uint64_t capacity, uint64_t* nruns);
int  mums_shard_restart_ties(mums_ctx* ctx, const uint32_t* d_packed_all, const uint64_t* runs, uint64_t nruns,
                             const uint64_t* vofs, uint32_t* d_out);
int  mums_shard_restart_finish(mums_ctx* ctx, uint64_t restarts, const uint64_t* rkey, const uint64_t* rS,
                               const uint64_t* runs, uint64_t nruns, const uint32_t* d_pos, const uint64_t* vofs);
int  mums_shard_restart_info(mums_ctx* ctx, uint64_t* info);
/* Repeat tolerance in the sharded mode (MemHash.cpp:139-162: the first copies of a genome in
 * SortedMerList order, so every run of equal keys in std::sort order, MemorySML.cpp:54), run
 * by mums_shard_run after step 3 above:
 *   mums_shard_tie_flags: this rank's pair flags of its SML parts (u32 per record: slot i of
 *     genome g flags i, i + 1 equal), genome g's at d_out + gofs[g];
 *   mums_shard_tie_replay (rank g % world): genome g's flags from every rank (nparts parts in
 *     rank order at d_flags + flag_off[r], lens[r] slots) -> the std::sort order replayed on
 *     the keys of the all-gathered packed genome -> ids (position in the genome, ~0 outside
 *     every run) of part r at d_out + out_off[r];
 *   mums_shard_tie_apply: this rank's records take the ids at d_ids + vofs[g] + SML slot. */
int  mums_shard_tie_flags(mums_ctx* ctx, const uint64_t* gofs, uint32_t* d_out);
int  mums_shard_tie_replay(mums_ctx* ctx, const uint32_t* d_packed_all, uint32_t genome, uint32_t nparts,
                           const uint32_t* d_flags, const uint64_t* flag_off, const uint64_t* lens, uint32_t* d_out,
                           const uint64_t* out_off);
int  mums_shard_tie_apply(mums_ctx* ctx, const uint32_t* d_ids, const uint64_t* vofs);
/* Accepted probes of the last seed stage, in AddHashEntry call order
 * (MemHash::EnumerateMatches -> AddHashEntry, MemHash.cpp:139-162, 209-251):
 * hash bucket ((offset % T) + T) % T and the smallest global seed-mer index of
 * the probe's key group (its identity; checking aid, host-side gather). */
int  mums_probe_count(mums_ctx* ctx, uint64_t* count);
/* ---- sharded FindMatches, after mums_shard_merge on every rank ---
 * Replaces the single-process AddHashEntry replay (MemHash::AddHashEntry,
 * MemHash.cpp:209-251; ExtendMatch, MatchFinder.h:218-374; GetMatchList,
 * MemHash.h:182-203) when the probes of one MemHash live on several GPUs.  Rank r owns
 * the hash buckets [bounds[r], bounds[r+1]); the ranks' key ranges are in rank order,
 * so every bucket's probes arrive in the reference's AddHashEntry order and the
 * ranks' outputs concatenated in rank order are the bucket-major MatchList.
 *   1. mums_shard_bucket_counts: probes of this rank per hash bucket (host, table_size);
 *   2. mums_shard_probe_rows: this rank's probes (key order) as rows of G+1 int64
 *      {signed starts (SetDirection), CalculateOffset} into d_rows, stably grouped by
 *      destination rank; counts[r] rows go to rank r;
 *   3. the caller exchanges the rows (all-to-all, sources in rank order) and assembles
 *      all genomes' 2-bit packed words (mums_shard_packed_info / _copy: this rank's
 *      slice [word_offset, word_offset + nwords) of the total_words array);
 *   4. mums_shard_find: chain labelling + replay of the received rows; results via
 *      mums_result_count / mums_result_copy (this rank's buckets, bucket-major). */
int  mums_shard_bucket_counts(mums_ctx* ctx, uint64_t* counts);
int  mums_shard_probe_rows(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_rows,
                           uint64_t capacity_rows, uint64_t* counts);
int  mums_shard_packed_info(mums_ctx* ctx, uint64_t* word_offset, uint64_t* nwords, uint64_t* total_words);
int  mums_shard_packed_copy(mums_ctx* ctx, uint32_t* d_dst);
int  mums_shard_find(mums_ctx* ctx, const int64_t* d_rows, uint64_t nrows, const uint32_t* d_packed_all);
/* The same FindMatches with the chains labelled where the probes are (mums_shard_run's
 * default): on related genomes most probes share one hash bucket (the main
 * diagonal's offset, MemHash.cpp:213), so the bucket owner would label nearly every chain.
 *   mums_shard_chain_label: after the merge (and restarts) the rank labels the chains of its
 *     own probes (its key range, key order; MatchFinder::ExtendMatch, MatchFinder.h:218-374)
 *     against the all-gathered packed genomes; *nchains = chain entries labelled.
 *   mums_shard_chain_export: rows (as mums_shard_probe_rows) + per row its chain entry's index
 *     inside the destination's entry block (d_tags) + the entries (G + 2 int64 each, d_entries)
 *     with their first probe's index inside the destination's row block (d_first), grouped by
 *     destination rank (row_counts / entry_counts per rank; a chain goes where its bucket does).
 *   mums_shard_find_labelled: on the bucket owner, the received blocks in source-rank order
 *     (src_rows / src_entries: the blocks' sizes); equal entries from several ranks merge, then
 *     the replay and the MatchList of the owned buckets.
 *   mums_shard_chain_info: info[4] = {probes labelled, chains, label time in us, rows the rank
 *     replayed as bucket owner in its last sharded FindMatches}.
 *
 * Kept-probe export (what mums_shard_run does by default; MUMS_DEV_SHARD_ALL_ROWS=1 sends every
 * row as above).  The owner's replay needs only each chain's first AddHashEntry call and the
 * suspicious calls (first-genome start at or past the chain's next_s: the only ones whose
 * lower_bound over the bucket vector can miss their chain entry, MemHash.cpp:209-251,
 * MatchHashEntry.h:121-143); every other call collides with its chain entry.
 *   mums_shard_chain_entries: after mums_shard_chain_label, the rank's chain entries (G + 2 int64)
 *     grouped by the rank owning their hash bucket (bounds as above; entry_counts per rank).
 *   mums_shard_entry_thresholds: on the bucket owner, the received entries in source-rank order:
 *     equal entries merge; d_thr[2e] = next_s of entry e's chain (the smallest first-genome start
 *     >= its own among the other chains of its bucket and genome set, ~0 when none), d_thr[2e+1]
 *     = 1 when e is the chain's first entry in source order (that rank holds the chain's first
 *     AddHashEntry call).  The answers go back to the sources in the same order.
 *   mums_shard_kept_export: with the owner's answers for the rank's own entries (the order of
 *     mums_shard_chain_entries), the rows the replay needs (grouped by destination, key order,
 *     with tags as mums_shard_chain_export), per entry its first sent row inside its
 *     destination's row block (d_first; the block's end when none), and per destination the
 *     probes not sent (dropped_counts: collisions).
 *   mums_shard_find_kept: mums_shard_find_labelled on the kept rows (the entries of
 *     mums_shard_chain_entries, d_first of mums_shard_kept_export); dropped = the calls of the
 *     owned buckets the sources did not send, counted as collisions (MemCollisionCount). */
int  mums_shard_chain_label(mums_ctx* ctx, const uint32_t* d_packed_all, uint64_t* nchains);
int  mums_shard_chain_export(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_rows, uint32_t* d_tags,
                             uint64_t capacity_rows, int64_t* d_entries, uint32_t* d_first, uint64_t capacity_entries,
                             uint64_t* row_counts, uint64_t* entry_counts);
int  mums_shard_find_labelled(mums_ctx* ctx, const int64_t* d_rows, const uint32_t* d_tags, uint64_t nrows,
                              const int64_t* d_entries, const uint32_t* d_first, uint64_t nentries, uint32_t nsrc,
                              const uint64_t* src_rows, const uint64_t* src_entries, const uint32_t* d_packed_all);
int  mums_shard_chain_info(mums_ctx* ctx, uint64_t* info);
int  mums_shard_chain_entries(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_entries,
                              uint64_t capacity_entries, uint64_t* entry_counts);
int  mums_shard_entry_thresholds(mums_ctx* ctx, const int64_t* d_entries, uint64_t nentries, uint32_t* d_thr);
int  mums_shard_kept_export(mums_ctx* ctx, uint32_t nranks, const uint32_t* d_thr, int64_t* d_rows, uint32_t* d_tags,
                            uint64_t capacity_rows, uint32_t* d_first, uint64_t* row_counts, uint64_t* dropped_counts);
int  mums_shard_find_kept(mums_ctx* ctx, const int64_t* d_rows, const uint32_t* d_tags, uint64_t nrows,
                          const int64_t* d_entries, const uint32_t* d_first, uint64_t nentries, uint32_t nsrc,
                          const uint64_t* src_rows, const uint64_t* src_entries, uint64_t dropped,
                          const uint32_t* d_packed_all);
int  mums_probe_copy(mums_ctx* ctx, uint32_t* buckets, uint64_t* ref_index, uint64_t capacity);

/* ---- multi-GPU MemHash through the ABI ----------
 * One communicator per rank: RCCL over xGMI for one process per GPU
 * (mums_comm_unique_id on rank 0, broadcast by the caller, mums_comm_init_rank on every
 * rank) or for one process driving several GPUs (mums_comm_init_all, then one host
 * thread per device); mums_comm_init_local: ranks that are threads of this process,
 * host-staged (testing the orchestration on one GPU).  mums_shard_run(ctx, comm, stage)
 * runs the whole sharded pipeline of a rank whose context was set up with
 * mums_shard_layout / mums_shard_slice and its genomes: keys, all-gather of bucket counts,
 * key ranges (mums_shard_key_ranges), all-to-allv of the records, merge; with
 * MUMS_STAGE_ALL also the probe rows' all-to-allv, the packed genomes' all-gather and the
 * chain labelling + replay of this rank's hash buckets (results via mums_result_*, the
 * ranks' lists in rank order = the bucket-major MatchList). */
typedef struct mums_comm mums_comm;
int  mums_comm_unique_id(void* id, uint64_t bytes);   /* ncclGetUniqueId, 128 bytes */
int  mums_comm_init_rank(mums_comm** comm, int device, int world, int rank, const void* id);
int  mums_comm_init_all(mums_comm** comms, int ndev, const int* devices);
int  mums_comm_init_local(mums_comm** comms, int nranks, const int* devices);
/* The caller's own transport (MPI, gloo, a job launcher's sockets ...): two host-side
 * collectives, called on every rank in the same order; return 0 on success.  Device data
 * is staged through host memory by the library.
 *   allgather_u64: recv[r * n + i] = rank r's send[i]
 *   alltoallv    : send holds one byte block per peer in rank order (send_bytes[p] bytes
 *                  for peer p), recv the blocks from every peer in rank order (recv_bytes[p]) */
typedef struct mums_comm_ops {
    int (*allgather_u64)(void* user, const uint64_t* send, uint64_t n, uint64_t* recv);
    int (*alltoallv)(void* user, const void* send, const uint64_t* send_bytes, void* recv,
                     const uint64_t* recv_bytes);
} mums_comm_ops;
int  mums_comm_init_host(mums_comm** comm, int device, int world, int rank, const mums_comm_ops* ops, void* user);
void mums_comm_destroy(mums_comm* comm);
const char* mums_comm_last_error(mums_comm* comm);
/* info[4] = {probe rows sent, bytes sent, probe rows received, bytes received} by this rank in
 * its last sharded FindMatches (rows, tags, chain entries, thresholds and first-row indices). */
int mums_comm_exchange_info(mums_comm* comm, uint64_t* info);
/* the balanced contiguous key (or hash-bucket) ranges of the exchange: rank r gets
 * [first[r], first[r] + count[r]) (host only, no device needed) */
int  mums_shard_key_ranges(const uint64_t* totals, uint32_t nbuckets, uint32_t world, uint32_t* first,
                           uint32_t* count);
int  mums_shard_run(mums_ctx* ctx, mums_comm* comm, int stage);

int  mums_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MUMS_H */
