/*
 * mums_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of libMems' MemHash / MaskedMemHash multi-MUM seed-finding
 * path (koadman/libMems 1.6.1), used as the parity checker for the HIP
 * implementation in libmems_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product path never
 * links or calls it.
 *
 * Pinning: the reference is not buildable in this image without stand-ins
 * for libGenome / libMUSCLE / boost, so it is not compiled here.  This
 * restatement is pinned to the known-answer vectors recorded in
 * SURVEY.md Appendix C (outputs of the reference itself: match counts and
 * md5 of the MatchList text for 9 generator configurations); see
 * tests/test_oracle_pinning.py and tests/golden/.
 */
#ifndef MUMS_ORACLE_H
#define MUMS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- seed patterns (SeedMasks.h) ---- */
int64_t  oracle_get_seed(int weight, int seed_rank);          /* SeedMasks.h:298-321 */
int      oracle_seed_length(int64_t seed);                    /* SeedMasks.h:335-350 */
int      oracle_seed_weight(int64_t seed);                    /* SeedMasks.h:363-373 */
unsigned oracle_default_seed_weight(uint64_t avg_len);        /* SeedMasks.h:389-401 */

/* ---- encoding (SortedMerList.cpp) ---- */
/* 2-bit pack, returns number of words written ( ceil(2n/32)+2 ); -1 on '-' */
int64_t  oracle_pack(const char* seq, uint64_t n, uint32_t* out_words);
/* canonical spaced-seed key (GetDnaSeedMer) for every position 0..n-L  */
int      oracle_seed_keys(const char* seq, uint64_t n, uint64_t seed, uint64_t* out_keys);
/* MemorySML::Create: positions sorted by full 64-bit key (ties: position asc) */
int      oracle_build_sml(const char* seq, uint64_t n, uint64_t seed, uint32_t* out_pos);
/* SeedOccurrenceList::construct + smoothFrequencies: n float32 frequencies */
int      oracle_seed_occurrence(const char* seq, uint64_t n, uint64_t seed, float* out);

/* ---- MemHash::FindMatches ---- */
typedef struct oracle_params {
    uint64_t seed;             /* spaced seed pattern                          */
    uint32_t repeat_tol;       /* MemHash::SetRepeatTolerance, default 0       */
    uint32_t enum_tol;         /* MemHash::SetEnumerationTolerance, default 1  */
    uint32_t table_size;       /* MemHash::SetTableSize, default 40000         */
    int      masked;           /* 1 = MaskedMemHash::HashMatch semantics       */
    uint64_t seq_mask;         /* MaskedMemHash::SetMask (0 = no filter)       */
    int      gnseqi_end_neg1;  /* 1: GNSEQI_END == UINT64_MAX (maxlen -1 in    *
                                *    ExtendMatch); 0: INT64_MAX                 */
    int      seeds_only;       /* 1: stop after probe construction (keys, SML  *
                                *    sort, merge, accept, probe + bucket): the  *
                                *    "sorted+matched" scope of the bench metric */
    int      parallel_compat;  /* 1: ParallelMemHash::FindMatches chunking +    *
                                *    MergeTable (ParallelMemHash.cpp:42-121);    *
                                *    2: same chunks, one MergeTable at the end   *
                                *    (checking aid for the GPU's model)          */
    uint64_t chunk_size;       /* its CHUNK_SIZE (0 = 200000, :51)              */
    int      pairwise;         /* 1: PairwiseMatchFinder::EnumerateMatches      *
                                *    (PairwiseMatchFinder.cpp:37-73)             */
    const uint64_t* start_points; /* MemHash::FindMatchesFromPosition start SML  *
                                *    indices (MemHash.cpp:117-127); NULL = 0     */
} oracle_params;

typedef struct oracle_result oracle_result;

oracle_result* oracle_find_matches(int G, const char* const* seqs, const uint64_t* lens,
                                   const oracle_params* prm);
/* MergeTable of tables given as rows in bucket order, table after table */
oracle_result* oracle_merge_tables(int G, uint32_t table_size, const uint64_t* lens, const int64_t* starts,
                                   const uint64_t* nrows, uint32_t ntables);
uint64_t oracle_result_count(const oracle_result* r);
int      oracle_result_seqcount(const oracle_result* r);
/* lengths[count], starts[count*G] (row-major, signed 1-based, 0 = NO_MATCH) */
void     oracle_result_copy(const oracle_result* r, uint64_t* lengths, int64_t* starts);
uint64_t oracle_result_mem_count(const oracle_result* r);
uint64_t oracle_result_collision_count(const oracle_result* r);
uint64_t oracle_result_max_group(const oracle_result* r);
uint64_t oracle_result_probe_count(const oracle_result* r);
int      oracle_result_probe_log(const oracle_result* r, uint32_t* buckets, uint64_t* ref);
uint64_t oracle_result_seedmers(const oracle_result* r);
uint64_t oracle_result_chunks(const oracle_result* r);     /* compat: chunks searched */
uint64_t oracle_result_restarts(const oracle_result* r);   /* MER_REPEAT_LIMIT restarts */
const char* oracle_result_progress(const oracle_result* r); /* LogProgress text (serial MemHash path) */
int      oracle_result_match_log(const oracle_result* r, uint64_t* lengths, int64_t* starts); /* SetMatchLog order */
uint64_t oracle_result_match_log_count(const oracle_result* r);   /* its lines */
int      oracle_result_offset_log(const oracle_result* r, uint64_t* out); /* restarts x G start points */
void     oracle_result_free(oracle_result* r);
/* OpenMP driver of the same restatement (the bench's CPU baseline on the host cores):
 * per-genome SMLs in parallel, the merge split by key range, the hash buckets replayed
 * in parallel; bit-identical to oracle_find_matches (falls back to it for restarting
 * merges, start points and the compat mode).  threads <= 0: the OpenMP default. */
oracle_result* oracle_find_matches_omp(int G, const char* const* seqs, const uint64_t* lens,
                                       const oracle_params* prm, int threads);
int      oracle_omp_threads(void);
/* AddHashEntry replay of probe rows {starts[G], offset} (sharded FindMatches checks). */
oracle_result* oracle_replay_rows(int G, const char* const* seqs, const uint64_t* lens, const oracle_params* prm,
                                  const int64_t* rows, uint64_t nrows);

/* ---- synthetic genomes (SURVEY.md Appendix C generator) ---- */
/* fills G buffers of n bytes each (caller allocates G*n bytes, genome-major) */
/* EliminateOverlaps (Aligner.cpp:62-176) over a MatchList {len, starts[G]}; returns the
   new count, *len_out / *s_out malloc'd (free with oracle_free) -- eliminate_overlaps.c */
uint64_t oracle_eliminate_overlaps(int G, uint64_t M, const uint64_t* len_in, const int64_t* s_in,
                                   uint64_t** len_out, int64_t** s_out);
/* libstdc++ std::sort of ids by key[id] (SingleStartComparator order); depth override for tests */
void     oracle_std_sort_ids(uint32_t* ids, uint64_t n, const uint64_t* key);
void     oracle_std_sort_depth_override(int depth);
/* SML tie order: 1 = libstdc++ std::sort (the reference, default), 0 = by position */
void     oracle_set_sml_tie_rule(int rule);
int      oracle_get_sml_tie_rule(void);
/* SML tie order: 1 = libstdc++ std::sort (the reference, default), 0 = by position */
void     oracle_set_sml_tie_rule(int rule);
int      oracle_get_sml_tie_rule(void);
void     oracle_free(void* p);
void     oracle_generate(int G, uint64_t n, double p, uint64_t rng_seed, char* out);

#ifdef __cplusplus
}
#endif
#endif
