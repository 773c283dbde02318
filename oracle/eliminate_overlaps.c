/* TEST INFRASTRUCTURE ONLY -- CPU restatement of libMems' EliminateOverlaps
 * (libMems/Aligner.cpp:62-176), the MatchList step right after MemHash::FindMatches in
 * both aligners (Aligner.cpp:920,1211,1580,2220).  Only tests/ use it.
 *
 * Matches are value records {len, starts[G]} (Match = UngappedLocalAlignment<
 * HybridAbstractMatch<> >, Match.h:26): LeftEnd(s) = |start| (HybridAbstractMatch.h:217-225),
 * Multiplicity = defined starts (:54-60), CropStart(a): len -= a, positive starts += a;
 * CropEnd(a): len -= a, negative starts -= a (UngappedLocalAlignment.h:138-152,
 * HybridAbstractMatch.h:271-290), SetStart(s, 0) drops genome s (:163-204).
 *
 * The MatchList is a vector of pointers sorted per genome with std::sort and
 * SingleStartComparator (AbstractMatch.h:324-351: undefined < defined, then LeftEnd), so
 * the order of equal keys is the one libstdc++'s introsort leaves.  sort_ids restates
 * that algorithm literally (GCC bits/stl_algo.h / stl_heap.h: __introsort_loop with
 * _S_threshold 16 and depth 2*lg(n), __move_median_to_first, __unguarded_partition,
 * __partial_sort = heap select + sort_heap, __final_insertion_sort); tests pin it against
 * the real std::sort of this toolchain (tests/eo_model.cpp).  Parity of EliminateOverlaps
 * itself is unpinned by reference fixtures (the reference has none and Aligner.cpp needs
 * libGenome / MUSCLE to build).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mums_oracle.h"
#include "std_sort.h"

typedef struct {
    int G;
    uint64_t n, cap;
    int64_t* len;
    int64_t* s;   /* n x G */
} pool_t;

static int64_t pool_add(pool_t* p) {
    if (p->n == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 1024;
        p->len = (int64_t*)realloc(p->len, p->cap * sizeof(int64_t));
        p->s = (int64_t*)realloc(p->s, p->cap * (uint64_t)p->G * sizeof(int64_t));
    }
    return (int64_t)p->n++;
}

static int64_t labs64(int64_t x) { return x < 0 ? -x : x; }

/* ---- libstdc++ std::sort over ids, comp(a, b) = key[a] < key[b] (std_sort.h) ----------- */
static int depth_override = -1;

void oracle_std_sort_ids(uint32_t* ids, uint64_t n, const uint64_t* key) {
    ss_std_sort(key, ids, n, depth_override >= 0 ? depth_override : -1);
}

void oracle_std_sort_depth_override(int depth) { depth_override = depth; }

/* ---- EliminateOverlaps (Aligner.cpp:62-176) ----------------------------------------- */
static int mult(const pool_t* p, int64_t id) {
    int m = 0;
    for (int g = 0; g < p->G; ++g) m += p->s[id * p->G + g] != 0;
    return m;
}
static void crop_start(pool_t* p, int64_t id, int64_t a) {
    p->len[id] -= a;
    for (int g = 0; g < p->G; ++g)
        if (p->s[id * p->G + g] > 0) p->s[id * p->G + g] += a;
}
static void crop_end(pool_t* p, int64_t id, int64_t a) {
    p->len[id] -= a;
    for (int g = 0; g < p->G; ++g)
        if (p->s[id * p->G + g] < 0) p->s[id * p->G + g] -= a;
}
static int64_t copy_match(pool_t* p, int64_t id) {
    const int64_t c = pool_add(p);
    p->len[c] = p->len[id];
    memcpy(p->s + c * p->G, p->s + id * p->G, (size_t)p->G * sizeof(int64_t));
    return c;
}

uint64_t oracle_eliminate_overlaps(int G, uint64_t M, const uint64_t* len_in, const int64_t* s_in,
                                   uint64_t** len_out, int64_t** s_out) {
    pool_t P = {G, 0, 0, NULL, NULL};
    uint32_t* ml = (uint32_t*)malloc((M + 1) * sizeof(uint32_t));
    for (uint64_t i = 0; i < M; ++i) {
        const int64_t id = pool_add(&P);
        P.len[id] = (int64_t)len_in[i];
        memcpy(P.s + id * G, s_in + i * G, (size_t)G * sizeof(int64_t));
        ml[i] = (uint32_t)id;
    }
    uint64_t n = M;
    const uint32_t DEL = 0xFFFFFFFFu;
    if (n >= 2) {   /* if( ml.size() < 2 ) return; */
        for (int seqI = 0; seqI < G; ++seqI) {
            uint64_t* key = (uint64_t*)malloc(P.n * sizeof(uint64_t));
            for (uint64_t id = 0; id < P.n; ++id) key[id] = (uint64_t)labs64(P.s[id * G + seqI]);
            oracle_std_sort_ids(ml, n, key);
            free(key);
            uint32_t* newm = NULL;
            uint64_t nnew = 0, capnew = 0, deleted = 0;
            int64_t matchI = 0, nextI;
            for (; matchI != (int64_t)n; matchI++)
                if (P.s[(int64_t)ml[matchI] * G + seqI] != 0) break;
            for (; matchI < (int64_t)n; matchI++) {
                if (ml[matchI] == DEL) continue;
                for (nextI = matchI + 1; nextI < (int64_t)n; nextI++) {
                    if (ml[nextI] == DEL) continue;
                    int deleted_matchI = 0;
                    const int64_t I = ml[matchI], J = ml[nextI];
                    const int64_t startI = P.s[I * G + seqI], lenI = P.len[I];
                    const int64_t startJ = P.s[J * G + seqI];
                    int64_t diff = labs64(startJ) - labs64(startI) - lenI;
                    if (diff < 0) {
                        diff = -diff;
                        int64_t nm;
                        const int mJ = mult(&P, J), mI = mult(&P, I);
                        if (mJ > mI || (mJ == mI && P.len[J] > P.len[I])) {   /* matchI is smaller */
                            nm = copy_match(&P, I);
                            if (diff >= lenI) {
                                ml[matchI] = DEL;
                                matchI--;
                                deleted_matchI = 1;
                                deleted++;
                            } else if (startI > 0) {
                                crop_end(&P, I, diff);
                                crop_start(&P, nm, P.len[nm] - diff);
                            } else {
                                crop_start(&P, I, diff);
                                crop_end(&P, nm, P.len[nm] - diff);
                            }
                        } else {   /* nextI is smaller */
                            nm = copy_match(&P, J);
                            if (diff >= P.len[J]) {
                                ml[nextI] = DEL;
                                deleted++;
                            } else if (startJ > 0) {
                                crop_start(&P, J, diff);
                                crop_end(&P, nm, P.len[nm] - diff);
                            } else {
                                crop_end(&P, J, diff);
                                crop_start(&P, nm, P.len[nm] - diff);
                            }
                        }
                        P.s[nm * G + seqI] = 0;   /* new_match->SetStart( seqI, 0 ) */
                        if (mult(&P, nm) > 1 && P.len[nm] > 0) {
                            if (nnew == capnew) {
                                capnew = capnew ? 2 * capnew : 256;
                                newm = (uint32_t*)realloc(newm, capnew * sizeof(uint32_t));
                            }
                            newm[nnew++] = (uint32_t)nm;
                        }
                        if (deleted_matchI) break;
                    } else {
                        break;   /* there are no more overlaps */
                    }
                }
            }
            uint64_t w = n;
            if (deleted > 0) {
                w = 0;
                for (uint64_t k = 0; k < n; ++k)
                    if (ml[k] != DEL) ml[w++] = ml[k];
            }
            ml = (uint32_t*)realloc(ml, (w + nnew + 1) * sizeof(uint32_t));
            for (uint64_t k = 0; k < nnew; ++k) ml[w + k] = newm[k];
            n = w + nnew;
            free(newm);
        }
    }
    *len_out = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    *s_out = (int64_t*)malloc((n + 1) * (uint64_t)G * sizeof(int64_t));
    for (uint64_t k = 0; k < n; ++k) {
        (*len_out)[k] = (uint64_t)P.len[ml[k]];
        memcpy(*s_out + k * G, P.s + (uint64_t)ml[k] * G, (size_t)G * sizeof(int64_t));
    }
    free(ml);
    free(P.len);
    free(P.s);
    return n;
}

void oracle_free(void* p) { free(p); }
