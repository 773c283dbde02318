/*
 * mums_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker; see mums_oracle.h).
 *
 * Plain-C restatement of the libMems 1.6.1 MemHash hot path.  Every function
 * names the reference file:line it follows (paths relative to libMems/).
 * Nothing here is shipped in, linked into, or called by the product path.
 */
#include "mums_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "std_sort.h"

/* ------------------------------------------------------------------------- */
/* Seed pattern table: SeedMasks.h:44-260 (low words; the high words are 0). */
/* Rows are weights 0..31, columns seed ranks 0..5; 0 = "no seed".           */
/* ------------------------------------------------------------------------- */
static const uint32_t k_seed_table[32][6] = {
    {0}, {0}, {0},
    {0xb, 0, 0, 0, 0, 0},                                   /* w3  */
    {0x3b, 0, 0, 0, 0, 0},                                  /* w4  */
    {0x6b, 0x139, 0x193, 0x6b, 0, 0},                       /* w5  */
    {0x58D, 0x653, 0x1AB, 0xdb, 0, 0},                      /* w6  */
    {0x1953, 0x588d, 0x688b, 0x17d, 0x164d, 0},             /* w7  */
    {0x3927, 0x1CA7, 0x6553, 0xb6d, 0, 0},                  /* w8  */
    {0x7497, 0x1c927, 0x72a7, 0x6fb, 0x16ed, 0},            /* w9  */
    {0x1d297, 0x3A497, 0xE997, 0x6D5B, 0, 0},               /* w10 */
    {0x7954f, 0x75257, 0x1c9527, 0x5bed, 0x5b26d, 0},       /* w11 */
    {0x7954f, 0x3D32F, 0x768B7, 0x5B56D, 0, 0},             /* w12 */
    {0x792a4f, 0x1d64d7, 0x1d3597, 0x1b7db, 0x75ad7, 0},    /* w13 */
    {0x1e6acf, 0xF59AF, 0x3D4CAF, 0x35AD6B, 0, 0},          /* w14 */
    {0x7ac9af, 0x7b2a6f, 0x79aacf, 0x16df6d, 0x6b5d6b, 0},  /* w15 */
    {0xf599af, 0xEE5A77, 0x7CD59F, 0xEB5AD7, 0, 0},         /* w16 */
    {0x6dbedb, 0, 0, 0, 0, 0},                              /* w17 */
    {0x3E6B59F, 0x3EB335F, 0x7B3566F, 0, 0, 0},             /* w18 */
    {0x7b974ef, 0x7d6735f, 0x1edd74f, 0, 0, 0},             /* w19 */
    {0x1F59B35F, 0x3EDCEDF, 0xFAE675F, 0, 0, 0},            /* w20 */
    {0x7ddaddf, 0xaeb3f, 0x7eb76bf, 0, 0, 0},               /* w21 */
    {0x003fffff, 0, 0, 0, 0, 0},                            /* w22 */
    {0x007fffff, 0, 0, 0, 0, 0},
    {0x00ffffff, 0, 0, 0, 0, 0},
    {0x01ffffff, 0, 0, 0, 0, 0},
    {0x03ffffff, 0, 0, 0, 0, 0},
    {0x07ffffff, 0, 0, 0, 0, 0},
    {0x0fffffff, 0, 0, 0, 0, 0},
    {0x1fffffff, 0, 0, 0, 0, 0},
    {0x3fffffff, 0, 0, 0, 0, 0},
    {0x7fffffff, 0, 0, 0, 0, 0},                            /* w31 */
};

/* getSolidSeed: SeedMasks.h:270-281 */
static int64_t solid_seed(int weight) { return (int64_t)((((uint64_t)1) << weight) - 1); }

/* getSeed: SeedMasks.h:298-321 (SOLID_SEED == INT_MAX, :263) */
int64_t oracle_get_seed(int weight, int seed_rank) {
    if (seed_rank == INT_MAX) return solid_seed(weight);
    if (weight > 31) return solid_seed(32);
    if (seed_rank > 5) return solid_seed(weight);
    if (weight < 0 || k_seed_table[weight][seed_rank] == 0) return solid_seed(weight);
    return (int64_t)k_seed_table[weight][seed_rank];
}

/* getSeedLength: SeedMasks.h:335-350 */
int oracle_seed_length(int64_t seed) {
    int right = -1, left = -1;
    uint64_t s = (uint64_t)seed;
    for (int b = 0; b < 64; ++b, s >>= 1)
        if (s & 1) { left = b; if (right == -1) right = b; }
    return left != -1 ? left - right + 1 : 0;
}

/* getSeedWeight: SeedMasks.h:363-373 */
int oracle_seed_weight(int64_t seed) {
    int w = 0;
    uint64_t s = (uint64_t)seed;
    for (int b = 0; b < 64; ++b, s >>= 1) w += (int)(s & 1);
    return w;
}

/* getDefaultSeedWeight: SeedMasks.h:389-401 */
unsigned oracle_default_seed_weight(uint64_t avg_len) {
    unsigned m = (unsigned)ceil((log((double)avg_len) / log(2.0)) / 1.5);
    if (!(m & 1)) ++m;
    m = m < 5 ? 0 : m;
    if (avg_len == 0) m = 0;
    return m > 31 ? 31 : m;
}

/* ------------------------------------------------------------------------- */
/* Encoding: BasicDNATable SortedMerList.cpp:29-47, translate32 :425-460,     */
/* SetSequence :306-317 (ceil(2n/32) + 2 words; pad words zeroed here, they   */
/* are uninitialised in the reference but always masked off).                */
/* ------------------------------------------------------------------------- */
static uint8_t dna_code(unsigned char c) {
    switch (c) {
    case 'c': case 'C': case 'b': case 'B': case 'y': case 'Y': return 1;
    case 'g': case 'G': case 's': case 'S': case 'k': case 'K': return 2;
    case 't': case 'T': return 3;
    default: return 0;
    }
}

static uint64_t packed_words(uint64_t n) { return (2 * n) / 32 + (((2 * n) % 32) ? 1 : 0) + 2; }

int64_t oracle_pack(const char* seq, uint64_t n, uint32_t* out) {
    uint64_t nw = packed_words(n);
    memset(out, 0, nw * sizeof(uint32_t));
    for (uint64_t i = 0; i < n; ++i) {
        if (seq[i] == '-') return -1;  /* SortedMerList.cpp:433-437 throws */
        out[i / 16] |= (uint32_t)dna_code((unsigned char)seq[i]) << (30 - 2 * (i % 16));
    }
    return (int64_t)nw;
}

typedef struct sml_ctx {
    const uint32_t* words;
    uint64_t n;          /* sequence length                 */
    uint64_t seed;       /* pattern                         */
    int L, w;            /* seed length / weight            */
    uint64_t mer_mask;   /* top 2L bits  (SetMerMaskSize)   */
    uint64_t seed_mask;  /* top 2w bits                     */
} sml_ctx;

static uint64_t top_mask(int chars) {  /* SetMerMaskSize: SortedMerList.cpp:271-282 */
    return chars >= 32 ? ~(uint64_t)0 : (~(uint64_t)0) << (64 - 2 * chars);
}

/* GetMer: SortedMerList.cpp:321-342 */
static uint64_t get_mer(const sml_ctx* c, uint64_t pos) {
    uint64_t wi = (pos * 2) / 32, bit = (pos * 2) % 32;
    uint64_t m = ((uint64_t)c->words[wi] << 32) | c->words[wi + 1];
    if (bit > 0) m = (m << bit) | (c->words[wi + 2] >> (32 - bit));
    return m & c->mer_mask;
}

/* GetSeedMer: SortedMerList.cpp:726-762 (mer_transition at :744 never fires, L<=32) */
static uint64_t get_seed_mer(const sml_ctx* c, uint64_t pos) {
    uint64_t mer = get_mer(c, pos), sm = 0;
    for (int k = 0; k < c->L; ++k) {
        if (c->seed & ((uint64_t)1 << (c->L - 1 - k)))
            sm = (sm << 2) | ((mer >> (62 - 2 * k)) & 3);
    }
    return c->w >= 32 ? sm : sm << (64 - 2 * c->w);
}

/* RevCompMer: SortedMerList.cpp:597-614 (literal restatement) */
static uint64_t revcomp_mer(uint64_t a, int len) {
    uint64_t b = ~a, r = 0;
    for (int i = 0; i < 64; i += 2) {
        r |= b & 3;
        b >>= 2;
        r <<= 2;
    }
    int sh = 64 - 2 * (len + 1);
    r = sh >= 0 ? r << sh : r >> (-sh);
    return r | 1;
}

/* GetDnaSeedMer: SortedMerList.cpp:764-769 */
static uint64_t get_dna_seed_mer(const sml_ctx* c, uint64_t pos) {
    uint64_t s = get_seed_mer(c, pos);
    uint64_t r = revcomp_mer(s, c->w);
    return s < r ? s : r;
}

static int sml_init(sml_ctx* c, const char* seq, uint64_t n, uint64_t seed, uint32_t** words_out) {
    uint32_t* words = (uint32_t*)malloc(packed_words(n) * sizeof(uint32_t) + 16);
    if (!words) return -2;
    if (oracle_pack(seq, n, words) < 0) { free(words); return -1; }
    c->words = words;
    c->n = n;
    c->seed = seed;
    c->L = oracle_seed_length((int64_t)seed);
    c->w = oracle_seed_weight((int64_t)seed);
    c->mer_mask = top_mask(c->L);
    c->seed_mask = top_mask(c->w);
    *words_out = words;
    return 0;
}

/* SMLLength: SortedMerList.cpp:288-295 (linear sequences only) */
static uint64_t sml_length(uint64_t n, int L) { return n < (uint64_t)L ? 0 : n - L + 1; }

int oracle_seed_keys(const char* seq, uint64_t n, uint64_t seed, uint64_t* out) {
    sml_ctx c; uint32_t* w;
    int rc = sml_init(&c, seq, n, seed, &w);
    if (rc) return rc;
    uint64_t m = sml_length(n, c.L);
    for (uint64_t p = 0; p < m; ++p) out[p] = get_dna_seed_mer(&c, p);
    free(w);
    return 0;
}

/* MemorySML::Create: MemorySML.cpp:45-60 -- std::sort(bmer, bmer_lessthan) of the      */
/* {position, mer} array FillDnaSeedSML / FillSML fill in position order                 */
/* (SortedMerList.cpp:771-783).  bmer_lessthan compares the mer only (SortedMerList.h:   */
/* 311-314), so equal mers stay in the order libstdc++'s introsort leaves them: restated */
/* in std_sort.h (the comparisons and moves depend on the keys alone, so sorting the     */
/* position ids by key[id] gives the same permutation as sorting the bmer structs).      */
/* Rule 1 (default) = that order; rule 0 = ties by position (the order of a stable sort, */
/* kept only so tests can count the inputs on which the two differ).                      */
typedef struct { uint64_t key; uint32_t pos; } bmer_t;

static int g_sml_tie_rule = 1;

void oracle_set_sml_tie_rule(int rule) { g_sml_tie_rule = rule; }
int oracle_get_sml_tie_rule(void) { return g_sml_tie_rule; }

static int bmer_cmp(const void* a, const void* b) {
    const bmer_t* x = (const bmer_t*)a; const bmer_t* y = (const bmer_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

static bmer_t* build_sml(const sml_ctx* c, const uint64_t* keys, uint64_t m) {
    bmer_t* v = (bmer_t*)malloc((m ? m : 1) * sizeof(bmer_t));
    (void)c;
    if (g_sml_tie_rule == 0) {
        for (uint64_t p = 0; p < m; ++p) { v[p].key = keys[p]; v[p].pos = (uint32_t)p; }
        qsort(v, m, sizeof(bmer_t), bmer_cmp);
        return v;
    }
    uint32_t* ids = (uint32_t*)malloc((m ? m : 1) * sizeof(uint32_t));
    for (uint64_t p = 0; p < m; ++p) ids[p] = (uint32_t)p;
    ss_std_sort(keys, ids, m, -1);
    for (uint64_t i = 0; i < m; ++i) { v[i].key = keys[ids[i]]; v[i].pos = ids[i]; }
    free(ids);
    return v;
}

int oracle_build_sml(const char* seq, uint64_t n, uint64_t seed, uint32_t* out_pos) {
    sml_ctx c; uint32_t* w;
    int rc = sml_init(&c, seq, n, seed, &w);
    if (rc) return rc;
    uint64_t m = sml_length(n, c.L);
    uint64_t* keys = (uint64_t*)malloc((m ? m : 1) * sizeof(uint64_t));
    for (uint64_t p = 0; p < m; ++p) keys[p] = get_dna_seed_mer(&c, p);
    bmer_t* v = build_sml(&c, keys, m);
    for (uint64_t i = 0; i < m; ++i) out_pos[i] = v[i].pos;
    free(v); free(keys); free(w);
    return 0;
}

/* SeedOccurrenceList::construct (SeedOccurrenceList.h:22-61) and          */
/* smoothFrequencies (:71-87), literally: float32 counts, double running sum. */
int oracle_seed_occurrence(const char* seq, uint64_t n, uint64_t seed, float* count) {
    sml_ctx c; uint32_t* w;
    int rc = sml_init(&c, seq, n, seed, &w);
    if (rc) return rc;
    uint64_t m = sml_length(n, c.L);
    uint64_t* keys = (uint64_t*)malloc((m ? m : 1) * sizeof(uint64_t));
    for (uint64_t p = 0; p < m; ++p) keys[p] = get_dna_seed_mer(&c, p);
    bmer_t* sml = build_sml(&c, keys, m);
    const uint64_t total_len = n, mask = c.seed_mask;
    for (uint64_t i = 0; i < total_len; ++i) count[i] = 0.0f;
    uint64_t seed_start = 0, cur_seed_count = 1, seedI = 1;
    for (seedI = 1; seedI < m; seedI++) {
        if ((sml[seedI].key & mask) == (sml[seedI - 1].key & mask)) { ++cur_seed_count; continue; }
        for (uint64_t i = seed_start; i < seedI; ++i) count[sml[i].pos] = (float)cur_seed_count;
        seed_start = seedI;
        cur_seed_count = 1;
    }
    for (uint64_t i = seed_start; i < seedI && i < m; ++i) count[sml[i].pos] = (float)cur_seed_count;
    for (; seedI < total_len; ++seedI) count[seedI] = 1;
    /* smoothFrequencies */
    {
        const uint64_t L = (uint64_t)c.L;
        float* buf = (float*)malloc(L * sizeof(float));
        for (uint64_t k = 0; k < L; ++k) buf[k] = 1.0f;
        if (total_len > 0) {
            double sum = (double)(L - 1) + count[0];
            buf[0] = count[0];
            for (uint64_t i = 1; i < total_len; i++) {
                count[i - 1] = (float)(sum / (double)L);
                sum += count[i];
                uint64_t bufI = i % L;
                sum -= buf[bufI];
                buf[bufI] = count[i];
            }
        }
        free(buf);
    }
    for (uint64_t i = 0; i < total_len; ++i) if (count[i] == 0) count[i] = 1;
    free(sml); free(keys); free(w);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* MatchHashEntry (MatchHashEntry.h:30-103, MatchHashEntry.cpp).              */
/* A match = one length + G signed 1-based starts (0 = NO_MATCH,             */
/* AbstractMatch.h:27); m_mersize is L for probes (HashMatch, MemHash.cpp:172)*/
/* and 0 for stored copies (operator=, MatchHashEntry.cpp:122).              */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t len;
    int64_t offset;
    int64_t mersize;
    int64_t* s;   /* G starts */
} mhe_t;

typedef struct {
    int G, L;
    uint64_t seed_mask;
    const uint64_t** keys;   /* keys[g][p] = GetDnaSeedMer(p) of genome g */
    const uint64_t* n;       /* genome lengths                            */
    int64_t gnseqi_end;      /* value of (int64)GNSEQI_END                */
} ext_ctx;

/* FirstStart: HybridAbstractMatch.h:121-129 (lowest genome with a start) */
static int first_start(const mhe_t* m, int G) {
    for (int i = 0; i < G; ++i) if (m->s[i] != 0) return i;
    return INT_MAX;
}

/* CalculateOffset: MatchHashEntry.cpp:141-160 */
static void calc_offset(mhe_t* m, int G) {
    int r = first_start(m, G);
    int64_t off = 0;
    for (int i = r + 1; i < G; ++i) {
        if (m->s[i] != 0) {
            int64_t t = m->s[i] - m->s[r];
            if (m->s[i] < 0) t -= m->len;
            off += t;
        }
    }
    m->offset = off;
}

/* Contains: MatchHashEntry.cpp:164-200  (does a contain b) */
static int contains(const mhe_t* a, const mhe_t* b, int G) {
    if (a->offset != b->offset) return 0;
    int i = first_start(b, G);
    int64_t diff = b->s[i] - a->s[i];
    if (a->s[i] == 0) return 0;
    if (diff < 0 || a->len < b->len + diff) return 0;
    int64_t diff_rc = b->len - a->len + diff;
    for (++i; i < G; ++i) {
        int64_t di = b->s[i] - a->s[i];
        if (b->s[i] == 0 && a->s[i] == 0) continue;
        else if (b->s[i] < 0 && diff_rc == di) continue;
        else if (diff != di) return 0;
    }
    return 1;
}

/* strict_start_lessthan_ptr: MatchHashEntry.cpp:48-69 */
static int strict_start_lt(const mhe_t* a, const mhe_t* b, int G) {
    int start_diff = first_start(a, G) - first_start(b, G);
    if (start_diff == 0) {
        for (int i = 0; i < G; ++i) {
            int64_t as = a->s[i], bs = b->s[i];
            if (as < 0) as = -as + a->len - a->mersize;
            if (bs < 0) bs = -bs + b->len - b->mersize;
            int64_t d = as - bs;
            if (d == 0) continue;
            return d < 0;
        }
    }
    return start_diff < 0;
}

/* MheCompare: MatchHashEntry.h:121-143 */
static int mhe_less(const mhe_t* a, const mhe_t* b, int G) {
    int fa = first_start(a, G), fb = first_start(b, G);
    if (fa > fb) return 1;
    if (fa == fb) {
        for (int i = fa; i < G; ++i) {
            if (a->s[i] == 0 && b->s[i] != 0) return 1;
            if (a->s[i] != 0 && b->s[i] == 0) return 0;
        }
        if (contains(a, b, G) || contains(b, a, G)) return 0;
        return strict_start_lt(a, b, G);
    }
    return 0;
}

/* oriented seed test used by ExtendMatch: MatchFinder.h:265-293 */
static void seed_at(const ext_ctx* x, int g, const mhe_t* m, uint64_t* key, int* parity) {
    int64_t mt = m->s[g];
    if (mt < 0) mt = -mt + m->len - x->L;
    uint64_t k = x->keys[g][mt - 1];
    *parity = m->s[g] < 0 ? (int)(k & 1) : !(k & 1);
    *key = k & x->seed_mask;
}

/* ExtendMatch: MatchFinder.h:218-374 (literal restatement of the control   */
/* flow; circular sequences are out of scope).                               */
static void extend_match(const ext_ctx* x, mhe_t* m) {
    int G = x->G, L = x->L;
    int cur[64]; int used = 0;
    for (int g = 0; g < G; ++g) if (m->s[g] != 0) cur[used++] = g;
    int jump = L;
    int extend_again = 0;
    for (int dir = 0; dir < 4; ++dir) {
        int64_t maxlen;
        if (dir == 0 || dir == 1) maxlen = x->gnseqi_end;   /* max_backward / max_forward defaults */
        else maxlen = L;
        for (int q = 0; q < used; ++q) {
            int g = cur[q];
            if (m->s[g] < 0) {
                int64_t rc_len = (int64_t)x->n[g] - m->len + m->s[g] + 1;
                if (rc_len < maxlen) maxlen = rc_len;
            } else if (m->s[g] - 1 < maxlen) {
                maxlen = m->s[g] - 1;
            }
        }
        int j = 0, i = used;
        uint64_t extend_limit = 0, extend_attempts = 0;
        while (maxlen - jump >= 0) {
            m->len += jump;
            maxlen -= jump;
            for (j = 0; j < used; ++j) {
                int g = cur[j];
                if (m->s[g] > 0) {
                    m->s[g] -= jump;
                    if (m->s[g] <= 0) m->s[g] += (int64_t)x->n[g];
                }
            }
            uint64_t k0; int p0;
            seed_at(x, cur[0], m, &k0, &p0);
            for (i = 1; i < used; ++i) {
                uint64_t ki; int pi;
                seed_at(x, cur[i], m, &ki, &pi);
                if (k0 != ki || p0 != pi) {
                    if (dir < 2) maxlen = 0;
                    break;
                }
            }
            extend_attempts += (uint64_t)jump;
            if (i == used) extend_limit = extend_attempts;
            if (dir > 1 && extend_attempts == (uint64_t)L) break;
        }
        if (i < used) {
            m->len -= jump;
            for (; j > 0; j--)
                if (m->s[cur[j - 1]] >= 0) m->s[cur[j - 1]] += jump;
        }
        if (dir > 1 && extend_attempts > 0) {
            if (extend_limit > 0) extend_again = 1;
            int64_t unmatched = (int64_t)(extend_attempts - extend_limit);
            if (i < used) unmatched -= jump;
            m->len -= unmatched;
            for (j = 0; j < used; ++j) {
                int g = cur[j];
                if (m->s[g] > 0) {
                    m->s[g] += unmatched;
                    if (m->s[g] > (int64_t)x->n[g]) m->s[g] -= (int64_t)x->n[g];
                }
            }
        }
        for (int g = 0; g < G; ++g) m->s[g] = -m->s[g];   /* Invert: HybridAbstractMatch.h:206-213 */
        if (dir >= 1) jump = 1;
        if (dir == 3 && extend_again) { dir = -1; jump = L; extend_again = 0; }
    }
}

/* ------------------------------------------------------------------------- */
/* MemHash table (MemHash.cpp:209-251) and driver                             */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t* v; uint32_t n, cap; } bucket_t;
typedef struct { uint32_t g; uint32_t pos; uint64_t key; } idmer_t;

#define MER_REPEAT_LIMIT 1000   /* MatchFinder.cpp:166 */

struct oracle_result {
    int G;
    uint64_t count;
    uint64_t* lengths;
    int64_t* starts;
    uint64_t mem_count, collision_count, max_group, probes, seedmers, chunks, restarts;
    uint64_t* offlog;         /* start points after every restart (SetOffsetLog, MatchFinder.cpp:152-162) */
    int offlog_g;
    uint64_t* mlog_len;       /* SetMatchLog (MemHash.cpp:238-241): inserted entries in insertion order */
    int64_t* mlog_s;
    uint64_t mlog_n, mlog_cap;
    uint32_t* plog_bucket;    /* seeds_only: per AddHashEntry call, its bucket ... */
    uint64_t* plog_ref;       /* ... and the global seed-mer index of the probe's first start */
    /* LogProgress (MatchFinder.cpp:55-56, 137-164, 296-309): the text a log stream receives */
    int prog_on;
    double m_progress;
    uint64_t mers_processed, total_mers;
    char* prog;
    size_t prog_n, prog_cap;
};

static void prog_append(oracle_result* res, const char* t) {
    const size_t k = strlen(t);
    if (res->prog_n + k + 1 > res->prog_cap) {
        res->prog_cap = (res->prog_n + k + 1) * 2 + 64;
        res->prog = (char*)realloc(res->prog, res->prog_cap);
    }
    memcpy(res->prog + res->prog_n, t, k + 1);
    res->prog_n += k;
}

/* a buffer of `size` mers exhausted (MatchFinder.cpp:297-309, PROGRESS_GRANULARITY 100) */
static void prog_event(oracle_result* res, uint64_t size) {
    if (!res->prog_on) return;
    res->mers_processed += size;
    const double old = res->m_progress;
    res->m_progress = ((double)res->mers_processed / (double)res->total_mers) * 100.0;
    if ((int)old != (int)res->m_progress) {
        char b[32];
        snprintf(b, sizeof b, "%d%%..", (int)((res->m_progress / 100.0) * 100));
        prog_append(res, b);
    }
    if (((int)old / 10) != ((int)res->m_progress / 10)) prog_append(res, "\n");
}

/* one SetMatchLog line (MemHash.cpp:238-241): the inserted entry */
static void mlog_push(oracle_result* res, uint64_t len, const int64_t* st, int G) {
    if (res->mlog_n == res->mlog_cap) {
        res->mlog_cap = res->mlog_cap ? res->mlog_cap * 2 : 256;
        res->mlog_len = (uint64_t*)realloc(res->mlog_len, res->mlog_cap * sizeof(uint64_t));
        res->mlog_s = (int64_t*)realloc(res->mlog_s, res->mlog_cap * (size_t)G * sizeof(int64_t));
    }
    res->mlog_len[res->mlog_n] = len;
    memcpy(res->mlog_s + res->mlog_n * (uint64_t)G, st, (size_t)G * sizeof(int64_t));
    ++res->mlog_n;
}

typedef struct {
    ext_ctx x;
    int seeds_only;
    uint64_t bucket_sum;
    uint32_t table_size;
    bucket_t* buckets;
    mhe_t* pool; uint64_t pool_n, pool_cap;
    int64_t* spool; uint64_t spool_n, spool_cap;
    uint64_t mem_count, collisions, probes;
    const uint64_t* gbase;    /* global seed-mer index of each genome's position 0 */
    uint32_t* plog_bucket; uint64_t* plog_ref; uint64_t plog_cap;
    int64_t* scratch;         /* G starts of the probe under construction */
    idmer_t* cm; idmer_t* hl; uint64_t cm_cap;   /* SearchRange's cur_match + hash list */
    int64_t* rec; uint64_t rec_n, rec_cap;       /* OpenMP driver: AddHashEntry calls recorded as rows */
} memhash_t;

static uint32_t pool_add(memhash_t* h, const mhe_t* src) {
    int G = h->x.G;
    if (h->pool_n == h->pool_cap) {
        h->pool_cap = h->pool_cap ? h->pool_cap * 2 : 1024;
        h->pool = (mhe_t*)realloc(h->pool, h->pool_cap * sizeof(mhe_t));
    }
    if (h->spool_n + (uint64_t)G > h->spool_cap) {
        /* starts live in a separate pool; re-point entries after growth */
        uint64_t ncap = h->spool_cap ? h->spool_cap * 2 : 1024 * (uint64_t)G;
        while (ncap < h->spool_n + (uint64_t)G) ncap *= 2;
        int64_t* ns = (int64_t*)realloc(h->spool, ncap * sizeof(int64_t));
        for (uint64_t e = 0; e < h->pool_n; ++e) h->pool[e].s = ns + (h->pool[e].s - h->spool);
        h->spool = ns; h->spool_cap = ncap;
    }
    mhe_t* e = &h->pool[h->pool_n];
    e->len = src->len; e->offset = src->offset;
    e->mersize = 0;   /* operator=: MatchHashEntry.cpp:118-126 */
    e->s = h->spool + h->spool_n;
    memcpy(e->s, src->s, (size_t)G * sizeof(int64_t));
    h->spool_n += (uint64_t)G;
    return (uint32_t)h->pool_n++;
}

/* std::lower_bound (libstdc++ __lower_bound: halve len, middle = first+half) */
static uint32_t lower_bound_mhe(memhash_t* h, const bucket_t* b, const mhe_t* val) {
    uint32_t first = 0, len = b->n;
    while (len > 0) {
        uint32_t half = len >> 1, mid = first + half;
        if (mhe_less(&h->pool[b->v[mid]], val, h->x.G)) { first = mid + 1; len = len - half - 1; }
        else len = half;
    }
    return first;
}

/* MemHash::AddHashEntry: MemHash.cpp:209-251 */
static void add_hash_entry(memhash_t* h, mhe_t* p) {
    int64_t T = (int64_t)h->table_size;
    uint32_t bi = (uint32_t)(((p->offset % T) + T) % T);
    bucket_t* b = &h->buckets[bi];
    ++h->probes;
    if (h->rec_cap) {   /* record mode (oracle_find_matches_omp): the call as a row {starts, offset} */
        const uint64_t W = (uint64_t)h->x.G + 1;
        if (h->rec_n == h->rec_cap) {
            h->rec_cap *= 2;
            h->rec = (int64_t*)realloc(h->rec, h->rec_cap * W * sizeof(int64_t));
        }
        memcpy(h->rec + h->rec_n * W, p->s, (size_t)h->x.G * sizeof(int64_t));
        h->rec[h->rec_n * W + (W - 1)] = p->offset;
        ++h->rec_n;
        return;
    }
    if (h->seeds_only) {
        h->bucket_sum += bi;
        /* probe log (checking aid): the probe's identity = global index of its first start */
        if (h->probes > h->plog_cap) {
            h->plog_cap = h->plog_cap ? 2 * h->plog_cap : 4096;
            h->plog_bucket = (uint32_t*)realloc(h->plog_bucket, h->plog_cap * sizeof(uint32_t));
            h->plog_ref = (uint64_t*)realloc(h->plog_ref, h->plog_cap * sizeof(uint64_t));
        }
        int f = first_start(p, h->x.G);
        int64_t s0 = p->s[f] < 0 ? -p->s[f] : p->s[f];
        h->plog_bucket[h->probes - 1] = bi;
        h->plog_ref[h->probes - 1] = h->gbase[f] + (uint64_t)(s0 - 1);
        return;
    }
    uint32_t it = lower_bound_mhe(h, b, p);
    if (it != b->n) {
        const mhe_t* e = &h->pool[b->v[it]];
        if (!mhe_less(e, p, h->x.G) && !mhe_less(p, e, h->x.G)) { ++h->collisions; return; }
    }
    extend_match(&h->x, p);
    uint32_t id = pool_add(h, p);
    uint32_t ins = lower_bound_mhe(h, b, &h->pool[id]);
    if (b->n == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 4;
        b->v = (uint32_t*)realloc(b->v, b->cap * sizeof(uint32_t));
    }
    memmove(b->v + ins + 1, b->v + ins, (size_t)(b->n - ins) * sizeof(uint32_t));
    b->v[ins] = id;
    ++b->n;
    ++h->mem_count;
}


/* MemHash::HashMatch MemHash.cpp:167-187 / MaskedMemHash::HashMatch          */
/* MaskedMemHash.cpp:38-63, SetDirection MemHash.cpp:189-203.                 */
static void hash_match(memhash_t* h, const oracle_params* prm, const idmer_t* lst, int cnt,
                       int64_t* scratch) {
    int G = h->x.G;
    mhe_t m;
    m.s = scratch;
    memset(m.s, 0, (size_t)G * sizeof(int64_t));
    m.len = h->x.L;
    m.mersize = h->x.L;
    int par[64] = {0};
    for (int k = 0; k < cnt; ++k) { m.s[lst[k].g] = (int64_t)lst[k].pos + 1; par[lst[k].g] = (int)(lst[k].key & 1); }
    int ref = first_start(&m, G);
    int ref_forward = !par[ref];
    for (int g = ref + 1; g < G; ++g)
        if (m.s[g] != 0 && ref_forward == par[g]) m.s[g] = -m.s[g];
    calc_offset(&m, G);
    int mult = 0;
    uint64_t match_number = 0;
    for (int g = 0; g < G; ++g) {
        match_number <<= 1;
        if (m.s[g] != 0) { match_number |= 1; ++mult; }
    }
    if (prm->masked) {
        if (prm->seq_mask == 0 || match_number == prm->seq_mask) add_hash_entry(h, &m);
    } else if (mult >= 2) {
        add_hash_entry(h, &m);
    }
}

/* MatchFinder::EnumerateMatches (odometer): MatchFinder.cpp:342-393 */
static void enumerate_odometer(memhash_t* h, const oracle_params* prm, idmer_t* lst, int cnt,
                               int64_t* scratch) {
    if (cnt == 2) { hash_match(h, prm, lst, cnt, scratch); return; }
    /* stable sort by genome id (std::list::sort is stable) */
    for (int a = 1; a < cnt; ++a) {
        idmer_t t = lst[a]; int b = a - 1;
        while (b >= 0 && lst[b].g > t.g) { lst[b + 1] = lst[b]; --b; }
        lst[b + 1] = t;
    }
    int id_pos[64], id_end[65], nid = 0;
    for (int a = 0; a < cnt; ++a) if (a == 0 || lst[a].g != lst[a - 1].g) id_pos[nid++] = a;
    for (int k = 0; k < nid; ++k) id_end[k] = id_pos[k];
    id_end[nid] = cnt;
    idmer_t cm[64];
    for (;;) {
        for (int k = 0; k < nid; ++k) cm[k] = lst[id_pos[k]];
        hash_match(h, prm, cm, nid, scratch);
        int mm = nid - 1;
        for (;;) {
            ++id_pos[mm];
            if (id_pos[mm] == id_end[mm + 1]) {
                if (mm == 0) return;
                id_pos[mm] = id_end[mm];
                mm--;
            } else break;
        }
    }
}

/* MemHash::EnumerateMatches: MemHash.cpp:139-162 */
static void enumerate_matches(memhash_t* h, const oracle_params* prm, const idmer_t* grp, int cnt,
                              idmer_t* hl, int64_t* scratch) {
    uint32_t tally[64] = {0};
    int nh = 0;
    for (int k = 0; k < cnt; ++k) {
        uint32_t g = grp[k].g;
        if (tally[g] < prm->enum_tol) hl[nh++] = grp[k];
        if (tally[g] > prm->repeat_tol) return;
        ++tally[g];
    }
    if (nh > 1) {
        if (prm->enum_tol == 1) hash_match(h, prm, hl, nh, scratch);
        else enumerate_odometer(h, prm, hl, nh, scratch);
    }
}

/* PairwiseMatchFinder::EnumerateMatches (PairwiseMatchFinder.cpp:37-73): the group   */
/* sorted by genome id (std::list::sort, stable; grp is genome-major already), the     */
/* genomes occurring exactly once kept in order, then MemHash::HashMatch of every pair  */
/* (a before b).  HashMatch always returns true, so the && chain never short-circuits.  */
static void enumerate_pairwise(memhash_t* h, const oracle_params* prm, const idmer_t* grp, int cnt, idmer_t* uniq,
                               int64_t* scratch) {
    int nu = 0;
    for (int a = 0; a < cnt;) {
        int b = a + 1;
        while (b < cnt && grp[b].g == grp[a].g) ++b;
        if (b - a == 1) uniq[nu++] = grp[a];
        a = b;
    }
    for (int a = 0; a < nu; ++a)
        for (int b = a + 1; b < nu; ++b) {
            idmer_t pr[2] = {uniq[a], uniq[b]};
            hash_match(h, prm, pr, 2, scratch);
        }
}

/* One group handed to EnumerateMatches (MatchFinder.cpp:242-246, :335-336). */
static void enumerate_group(memhash_t* h, const oracle_params* prm, idmer_t* grp, uint64_t cnt, idmer_t* hl,
                            oracle_result* res) {
    if (cnt > res->max_group) res->max_group = cnt;
    if (cnt < 2) return;
    if (prm->pairwise) enumerate_pairwise(h, prm, grp, (int)cnt, hl, h->scratch);
    else enumerate_matches(h, prm, grp, (int)cnt, hl, h->scratch);
}

static int sml_find_mer_lit(const bmer_t* v, uint64_t n, int L, uint64_t q, uint64_t* result);
static int get_breakpoint(int sarI, uint64_t startI, int G, bmer_t* const* sml, const uint64_t* m,
                          const uint64_t* lens, int L, uint64_t mask, uint64_t* bp);

#define MER_BUFFER_SIZE 10000u   /* MatchFinder.cpp:175 */

/* MatchFinder::SearchRange (MatchFinder.cpp:172-340), literally: per SML a buffer   */
/* of MER_BUFFER_SIZE entries read from start_points + mer_baseindex                 */
/* (MemorySML::Read, MemorySML.cpp:62-82); cur_mers = the list of buffer heads by    */
/* masked key (initial std::list::sort is stable; a new head goes before the first   */
/* head whose key is >= its own, :320-332); cur_match = the records of the current   */
/* key collected head by head (:281-291).  The MER_REPEAT_LIMIT check runs at the    */
/* top of every iteration (:253-277): with more than 1000 records collected for the  */
/* current key the group is dropped, start_points are moved to the GetBreakpoint     */
/* positions of the next key (never backwards, genomes before seqI exhausted) and 0  */
/* is returned (FindMatchSeeds calls again).  Returns 1 when the merge completes.    */
static int search_range_lit(memhash_t* h, const oracle_params* prm, int G, bmer_t* const* sml, const uint64_t* m,
                            const uint64_t* lens, uint64_t* start_points, const uint64_t* search_len,
                            oracle_result* res) {
    if (G < 1) return 1;
    const uint64_t mask = h->x.seed_mask;
    uint64_t vlo[64], vn[64];              /* buffer = sml[g][vlo .. vlo + vn) */
    uint32_t mer_index[64], mer_baseindex[64];
    idmer_t lst[64];                       /* cur_mers (key field = masked key) */
    int nl = 0;
    #define BUF_READ(g, size, off)                                                    \
        do {                                                                          \
            uint64_t o_ = (off), e_ = o_ + (uint64_t)(size);                          \
            if (o_ > m[g]) { vlo[g] = 0; vn[g] = 0; }                                 \
            else { if (e_ > m[g]) e_ = m[g]; vlo[g] = o_; vn[g] = e_ - o_; }          \
        } while (0)
    for (int g = 0; g < G; ++g) {
        uint64_t rs = MER_BUFFER_SIZE < search_len[g] ? MER_BUFFER_SIZE : search_len[g];
        BUF_READ(g, (uint32_t)rs, start_points[g]);
        mer_index[g] = 0;
        mer_baseindex[g] = 0;
        if (vn[g] > 0) {
            const bmer_t* b = &sml[g][vlo[g]];
            lst[nl].g = (uint32_t)g; lst[nl].pos = b->pos; lst[nl].key = b->key & mask;
            ++nl;
        }
    }
    for (int a = 1; a < nl; ++a) {   /* stable sort of the initial heads by masked key */
        idmer_t t = lst[a]; int b = a - 1;
        while (b >= 0 && lst[b].key > t.key) { lst[b + 1] = lst[b]; --b; }
        lst[b + 1] = t;
    }
    uint64_t cap = h->cm_cap, cn = 0;
    idmer_t* cm = h->cm;
    while (nl > 0) {
        const uint32_t cur = lst[0].g;
        const uint64_t hk = lst[0].key;
        if (cn > 0) {
            if (hk > (cm[0].key & mask)) {
                enumerate_group(h, prm, cm, cn, h->hl, res);
                cn = 0;
            }
        }
        if (cn > MER_REPEAT_LIMIT) {
            /* scan past the repetitive mers: the lexicographically next masked key */
            const uint64_t next_mer = (cm[0].key & mask) + (~mask + 1);
            if (cn > res->max_group) res->max_group = cn;
            uint64_t next_pos = 0;
            int seqI = 0;
            for (; seqI < G; ++seqI) {
                if (!sml_find_mer_lit(sml[seqI], lens[seqI], h->x.L, next_mer, &next_pos)) ++next_pos;
                if (next_pos < m[seqI]) break;
            }
            uint64_t old[64];
            for (int g = 0; g < G; ++g) old[g] = start_points[g];
            if (seqI < G) get_breakpoint(seqI, next_pos, G, sml, m, lens, h->x.L, mask, start_points);
            for (int g = 0; g < G; ++g) {
                const uint64_t done = old[g] + (uint64_t)(uint32_t)(mer_index[g] + mer_baseindex[g]);
                if (start_points[g] < done) start_points[g] = done;   /* don't move backwards */
                if (g < seqI) start_points[g] = m[g];
            }
            ++res->restarts;
            return 0;
        }
        uint64_t merI = mer_index[cur];
        int exhausted = merI < vn[cur] ? 0 : 1;
        while (!exhausted && hk == (sml[cur][vlo[cur] + merI].key & mask)) {
            if (cn == cap) {
                cap = cap ? 2 * cap : 4096;
                cm = (idmer_t*)realloc(cm, cap * sizeof(idmer_t));
                h->hl = (idmer_t*)realloc(h->hl, cap * sizeof(idmer_t));
            }
            const bmer_t* b = &sml[cur][vlo[cur] + merI];
            cm[cn].g = cur; cm[cn].pos = b->pos; cm[cn].key = b->key;
            ++cn;
            ++merI;
            ++mer_index[cur];
            if (merI == vn[cur]) exhausted = 1;
        }
        if (exhausted) {
            prog_event(res, vn[cur]);   /* mers_processed += mer_vector[cur_id].size() */
            mer_baseindex[cur] += (uint32_t)vn[cur];
            uint32_t rs = MER_BUFFER_SIZE;
            if ((uint64_t)MER_BUFFER_SIZE + mer_baseindex[cur] > search_len[cur])
                rs = (uint32_t)(search_len[cur] - mer_baseindex[cur]);
            BUF_READ(cur, rs, start_points[cur] + mer_baseindex[cur]);
            mer_index[cur] = 0;
            if (vn[cur] == 0) {   /* this SML is finished: forget its head */
                memmove(lst, lst + 1, (size_t)(nl - 1) * sizeof(idmer_t));
                --nl;
            }
        } else {
            memmove(lst, lst + 1, (size_t)(nl - 1) * sizeof(idmer_t));
            --nl;
            const bmer_t* b = &sml[cur][vlo[cur] + merI];
            idmer_t nm;
            nm.g = cur; nm.pos = b->pos; nm.key = b->key & mask;
            int at = 0;
            while (at < nl && lst[at].key < nm.key) ++at;
            memmove(lst + at + 1, lst + at, (size_t)(nl - at) * sizeof(idmer_t));
            lst[at] = nm;
            ++nl;
        }
    }
    #undef BUF_READ
    if (cn > 1) enumerate_group(h, prm, cm, cn, h->hl, res);   /* :335-336 */
    else if (cn > res->max_group) res->max_group = cn;
    h->cm = cm; h->cm_cap = cap;
    return 1;
}

/* MatchFinder::FindMatchSeeds(start_offsets) (MatchFinder.cpp:137-164): SearchRange    */
/* over the whole SMLs (search_len = GNSEQI_END) until it completes.                     */
static void find_match_seeds(memhash_t* h, const oracle_params* prm, int G, bmer_t* const* sml, const uint64_t* m,
                             const uint64_t* lens, const uint64_t* start_offsets, oracle_result* res) {
    uint64_t sp[64], sl[64];
    for (int g = 0; g < G; ++g) { sp[g] = start_offsets ? start_offsets[g] : 0; sl[g] = UINT64_MAX; }
    /* progress counters (MatchFinder.cpp:141-148): total = sar_table[i]->Length(), the sequence lengths
       (header.length = seq_len, SortedMerList.cpp:814 -- not SMLLength), processed = the start offsets */
    res->prog_on = 1;
    res->mers_processed = 0;
    res->total_mers = 0;
    res->m_progress = -1;
    for (int g = 0; g < G; ++g) {
        res->total_mers += lens[g];
        res->mers_processed += sp[g];
    }
    while (!search_range_lit(h, prm, G, sml, m, lens, sp, sl, res)) {
        res->mers_processed = 0;   /* :150-158 */
        for (int g = 0; g < G; ++g) res->mers_processed += sp[g];
        /* the offset stream line of this restart (MatchFinder.cpp:152-162) */
        res->offlog = (uint64_t*)realloc(res->offlog, (size_t)res->restarts * (size_t)G * sizeof(uint64_t));
        memcpy(res->offlog + (res->restarts - 1) * (uint64_t)G, sp, (size_t)G * sizeof(uint64_t));
        res->offlog_g = G;
    }
}

/* SortedMerList::bsearch (SortedMerList.cpp:380-394), recursion unrolled; unsigned */
static uint64_t sml_bsearch(const bmer_t* v, uint64_t q, uint64_t start, uint64_t end) {
    for (;;) {
        uint64_t middle = (start + end) / 2;
        uint64_t k = v[middle].key;
        if (k == q) return middle;
        if (k < q && middle < end) start = middle + 1;
        else if (k > q && start < middle) end = middle - 1;
        else return middle;
    }
}

/* SortedMerList::FindMer (SortedMerList.cpp:170-179); Length() = sequence length. */
/* On the early-return path the reference leaves `result` untouched (the caller's */
/* uninitialised cur_start); here it is 0.                                          */
static int sml_find_mer(const bmer_t* v, uint64_t n, int L, uint64_t q, uint64_t* result) {
    if (n == 0 || n < (uint64_t)L) { *result = 0; return 0; }
    uint64_t last_pos = n - (uint64_t)L;
    *result = sml_bsearch(v, q, 0, last_pos);
    return v[*result].key == q;
}

/* FindMer exactly as SortedMerList.cpp:170-179: on the early return (empty SML) the */
/* caller's result is left untouched (SearchRange's next_pos then counts on, :260). */
static int sml_find_mer_lit(const bmer_t* v, uint64_t n, int L, uint64_t q, uint64_t* result) {
    if (n == 0 || n < (uint64_t)L) return 0;
    *result = sml_bsearch(v, q, 0, n - (uint64_t)L);
    return v[*result].key == q;
}

/* MatchFinder::GetBreakpoint (MatchFinder.cpp:89-126).  The backward loop for the */
/* other SMLs compares against (break_mer.mer && mer_mask) (a bool) and re-reads   */
/* cur_start: it never runs unless break_mer.mer == 0, where it runs down to -1.   */
/* Returns -1 when startI is past the SML (operator[] out of range in the ref).    */
static int get_breakpoint(int sarI, uint64_t startI, int G, bmer_t* const* sml, const uint64_t* m,
                          const uint64_t* lens, int L, uint64_t mask, uint64_t* bp) {
    if (startI >= m[sarI]) return -1;
    const uint64_t bm = sml[sarI][startI].key;
    uint64_t prev = bm;
    while ((prev & mask) == (bm & mask)) {
        if (startI == 0) { startI--; break; }
        startI--;
        prev = sml[sarI][startI].key;
    }
    ++startI;
    for (int i = 0; i < G; ++i) {
        if (i == sarI) { bp[i] = startI; continue; }
        uint64_t cur = 0;
        if (sml_find_mer(sml[i], lens[i], L, bm, &cur)) {
            int64_t cur_matchI = (int64_t)cur;
            const uint64_t lhs = sml[i][cur].key & mask, rhs = (bm && mask) ? 1u : 0u;
            while (cur_matchI >= 0 && lhs == rhs) cur_matchI--;
            cur = (uint64_t)(cur_matchI + 1);
        }
        bp[i] = cur;
    }
    return 0;
}

/* Re-add of an already extended entry into another table (the patched 2-argument */
/* AddHashEntry of SURVEY.md Appendix B.3 as MergeTable calls it,                  */
/* ParallelMemHash.cpp:105-121): lower_bound, collision if equivalent, else insert;*/
/* Extended() is set, so no extension (MemHash.cpp:223-224).                        */
static void merge_entry(memhash_t* h, bucket_t* b, uint32_t id, oracle_result* res) {
    const mhe_t* e = &h->pool[id];
    uint32_t it = lower_bound_mhe(h, b, e);
    if (it != b->n) {
        const mhe_t* x = &h->pool[b->v[it]];
        if (!mhe_less(x, e, h->x.G) && !mhe_less(e, x, h->x.G)) { ++h->collisions; return; }
    }
    mlog_push(res, (uint64_t)e->len, e->s, h->x.G);   /* the patched AddHashEntry logs this insert too */
    if (b->n == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 4;
        b->v = (uint32_t*)realloc(b->v, b->cap * sizeof(uint32_t));
    }
    memmove(b->v + it + 1, b->v + it, (size_t)(b->n - it) * sizeof(uint32_t));
    b->v[it] = id;
    ++b->n;
}

/* ParallelMemHash::FindMatches (ParallelMemHash.cpp:42-103) with the thread     */
/* schedule of one OpenMP thread (the reference's output is the same for 1/4/8   */
/* threads): chunk starts from GetBreakpoint on the longest */
/* SML every chunk_size (200000, :51) mers; per chunk, SearchRange into the      */
/* thread table T (= the global table G after the previous merge) and MergeTable */
/* (:105-121): every entry of T re-added into G in bucket/vector order, then     */
/* T = G.  On return h->buckets holds G.  Returns -1 for inputs the reference    */
/* handles through undefined behaviour (a breakpoint past the SML end).          */
static int parallel_compat_search(memhash_t* h, const oracle_params* prm, int G, const uint64_t* lens,
                                  bmer_t* const* sml, const uint64_t* m, oracle_result* res) {
    const uint64_t chunk = prm->chunk_size ? prm->chunk_size : 200000;
    int mx = -1;
    uint64_t maxlen = 0;
    for (int g = 0; g < G; ++g) if (lens[g] > maxlen) { maxlen = lens[g]; mx = g; }
    if (mx < 0) return 0;
    uint64_t ncap = 16, nch = 1;
    uint64_t* cs = (uint64_t*)calloc(ncap * (size_t)G, sizeof(uint64_t));
    while (cs[(nch - 1) * G + mx] + chunk < lens[mx]) {
        if (nch == ncap) {
            ncap *= 2;
            cs = (uint64_t*)realloc(cs, ncap * (size_t)G * sizeof(uint64_t));
        }
        if (get_breakpoint(mx, cs[(nch - 1) * G + mx] + chunk, G, sml, m, lens, h->x.L, h->x.seed_mask,
                           cs + nch * G)) { free(cs); return -1; }
        /* a masked-key group at least a chunk long: GetBreakpoint returns the same start   */
        /* again and the reference's loop (:75-83) never ends -- reported, not replayed     */
        if (cs[nch * G + mx] <= cs[(nch - 1) * G + mx]) { free(cs); return -1; }
        ++nch;
    }
    /* progress counters, set once for the whole loop (:56-61); SearchRange never resets them, so
       with one thread the text is every chunk's buffer refills in chunk order */
    res->prog_on = 1;
    res->mers_processed = 0;
    res->total_mers = 0;
    res->m_progress = -1;
    for (int g = 0; g < G; ++g) res->total_mers += lens[g];
    const uint32_t T = h->table_size;
    bucket_t* gb = (bucket_t*)calloc(T, sizeof(bucket_t));   /* global table G */
    uint64_t* lo = (uint64_t*)malloc((size_t)G * sizeof(uint64_t));
    uint64_t* hi = (uint64_t*)malloc((size_t)G * sizeof(uint64_t));
    /* parallel_compat >= 16: R = parallel_compat - 16 ranks, each searching a contiguous chunk
       range into tables of its own (thread table and G start empty, never synced), their G
       tables re-added rank after rank into one at the end (a model of chunk-parallel GPUs) */
    /* parallel_compat >= 4096: one rank's table alone, R = (pc - 4096) >> 8 ranks, rank       */
    /* (pc - 4096) & 255 (its chunk range from empty tables; oracle_merge_tables re-adds them) */
    const int rank_only = prm->parallel_compat >= 4096;
    const uint64_t R = rank_only ? (uint64_t)((prm->parallel_compat - 4096) >> 8)
                                 : prm->parallel_compat >= 16 ? (uint64_t)(prm->parallel_compat - 16) : 1;
    const uint64_t ronly = rank_only ? (uint64_t)((prm->parallel_compat - 4096) & 255) : 0;
    bucket_t* gf = R > 1 && !rank_only ? (bucket_t*)calloc(T, sizeof(bucket_t)) : NULL;
    uint64_t rank = 0;
    for (uint64_t i = 0; i < nch; ++i) {
        if (rank_only && (i < nch * ronly / R || i >= nch * (ronly + 1) / R)) continue;
        if (gf && i == nch * rank / R) {   /* a new rank's range: fresh tables */
            for (uint32_t bI = 0; bI < T; ++bI) { h->buckets[bI].n = 0; gb[bI].n = 0; }
            ++rank;
        }
        for (int g = 0; g < G; ++g) {
            lo[g] = cs[i * G + g];
            /* chunk_lens = next start - start (gnSeqI, wraps) or GNSEQI_END (:91-96) */
            hi[g] = (i + 1 < nch) ? cs[(i + 1) * G + g] - cs[i * G + g] : UINT64_MAX;
        }
        const uint64_t p0 = h->pool_n;
        (void)search_range_lit(h, prm, G, sml, m, lens, lo, hi, res);   /* return value ignored (:97) */
        /* match log: the thread-table inserts of this chunk (pool order = AddHashEntry order) ... */
        for (uint64_t k = p0; k < h->pool_n; ++k) mlog_push(res, (uint64_t)h->pool[k].len, h->pool[k].s, G);
        if (prm->parallel_compat == 2 && i + 1 < nch) continue;   /* checking aid: one deferred merge */
        for (uint32_t bI = 0; bI < T; ++bI)
            for (uint32_t k = 0; k < h->buckets[bI].n; ++k) merge_entry(h, &gb[bI], h->buckets[bI].v[k], res);   /* ... then MergeTable's */
        for (uint32_t bI = 0; bI < T; ++bI) {   /* thread table = global table */
            bucket_t* tb = &h->buckets[bI];
            if (tb->cap < gb[bI].n) {
                tb->cap = gb[bI].n;
                tb->v = (uint32_t*)realloc(tb->v, tb->cap * sizeof(uint32_t));
            }
            if (gb[bI].n) memcpy(tb->v, gb[bI].v, gb[bI].n * sizeof(uint32_t));
            tb->n = gb[bI].n;
        }
        if (gf && (i + 1 == nch || i + 1 == nch * rank / R))   /* the rank's G into the final table */
            for (uint32_t bI = 0; bI < T; ++bI)
                for (uint32_t k = 0; k < gb[bI].n; ++k) merge_entry(h, &gf[bI], gb[bI].v[k], res);
    }
    if (gf) {
        for (uint32_t bI = 0; bI < T; ++bI) {
            free(gb[bI].v);
            bucket_t* tb = &h->buckets[bI];
            if (tb->cap < gf[bI].n) {
                tb->cap = gf[bI].n;
                tb->v = (uint32_t*)realloc(tb->v, tb->cap * sizeof(uint32_t));
            }
            if (gf[bI].n) memcpy(tb->v, gf[bI].v, gf[bI].n * sizeof(uint32_t));
            tb->n = gf[bI].n;
        }
        free(gb);
        gb = gf;
    }
    uint64_t entries = 0;
    for (uint32_t bI = 0; bI < T; ++bI) { entries += gb[bI].n; free(gb[bI].v); }
    h->mem_count = entries;   /* MemCount of the merged table */
    free(gb); free(lo); free(hi); free(cs);
    res->chunks = nch;
    return 0;
}

/* MergeTable (ParallelMemHash.cpp:105-121) of ntables tables into one empty table, table   */
/* after table: every row through merge_entry (AddHashEntry's lower_bound insert or         */
/* collision).  rows (lens, starts: G per row) hold every table in bucket / vector order,    */
/* tables concatenated, nrows[t] rows in table t.  The bucket owners' step of the chunk-range */
/* ranks.  Result: the merged MatchList in bucket order (TEST INFRASTRUCTURE). */
oracle_result* oracle_merge_tables(int G, uint32_t table_size, const uint64_t* lens, const int64_t* starts,
                                   const uint64_t* nrows, uint32_t ntables) {
    if (G < 1 || G > 64 || table_size == 0) return NULL;
    uint64_t n = 0;
    for (uint32_t t = 0; t < ntables; ++t) n += nrows[t];
    memhash_t h;
    memset(&h, 0, sizeof(h));
    h.x.G = G;
    h.table_size = table_size;
    h.pool = (mhe_t*)calloc(n ? n : 1, sizeof(mhe_t));
    int64_t* sc = (int64_t*)malloc((n ? n : 1) * (size_t)G * sizeof(int64_t));
    if (n) memcpy(sc, starts, n * (size_t)G * sizeof(int64_t));
    bucket_t* b = (bucket_t*)calloc(table_size, sizeof(bucket_t));
    oracle_result tmp;
    memset(&tmp, 0, sizeof(tmp));
    for (uint64_t k = 0; k < n; ++k) {
        mhe_t* e = &h.pool[k];
        e->len = (int64_t)lens[k];
        e->mersize = 0;
        e->s = sc + k * (uint64_t)G;
        calc_offset(e, G);
        const int64_t T = (int64_t)table_size;
        merge_entry(&h, &b[(uint32_t)(((e->offset % T) + T) % T)], (uint32_t)k, &tmp);
    }
    free(tmp.mlog_len);
    free(tmp.mlog_s);
    oracle_result* res = (oracle_result*)calloc(1, sizeof(oracle_result));
    res->G = G;
    uint64_t M = 0;
    for (uint32_t bI = 0; bI < table_size; ++bI) M += b[bI].n;
    res->count = M;
    res->mem_count = M;
    res->collision_count = h.collisions;
    res->lengths = (uint64_t*)malloc((M ? M : 1) * sizeof(uint64_t));
    res->starts = (int64_t*)malloc((M ? M : 1) * (size_t)G * sizeof(int64_t));
    uint64_t o = 0;
    for (uint32_t bI = 0; bI < table_size; ++bI) {
        for (uint32_t k = 0; k < b[bI].n; ++k, ++o) {
            const mhe_t* e = &h.pool[b[bI].v[k]];
            res->lengths[o] = (uint64_t)e->len;
            memcpy(res->starts + o * (uint64_t)G, e->s, (size_t)G * sizeof(int64_t));
        }
        free(b[bI].v);
    }
    free(b);
    free(sc);
    free(h.pool);
    return res;
}

oracle_result* oracle_find_matches(int G, const char* const* seqs, const uint64_t* lens,
                                   const oracle_params* prm) {
    if (G < 1 || G > 64) return NULL;
    oracle_result* res = (oracle_result*)calloc(1, sizeof(oracle_result));
    res->G = G;
    int bad = 0;
    sml_ctx* ctx = (sml_ctx*)calloc((size_t)G, sizeof(sml_ctx));
    uint32_t** words = (uint32_t**)calloc((size_t)G, sizeof(uint32_t*));
    uint64_t** keys = (uint64_t**)calloc((size_t)G, sizeof(uint64_t*));
    bmer_t** sml = (bmer_t**)calloc((size_t)G, sizeof(bmer_t*));
    uint64_t* m = (uint64_t*)calloc((size_t)G, sizeof(uint64_t));
    for (int g = 0; g < G; ++g) {
        if (sml_init(&ctx[g], seqs[g], lens[g], prm->seed, &words[g])) { res->count = 0; goto done; }
        m[g] = sml_length(lens[g], ctx[g].L);
        keys[g] = (uint64_t*)malloc((m[g] ? m[g] : 1) * sizeof(uint64_t));
        for (uint64_t p = 0; p < m[g]; ++p) keys[g][p] = get_dna_seed_mer(&ctx[g], p);
        sml[g] = build_sml(&ctx[g], keys[g], m[g]);
        res->seedmers += m[g];
    }
    {
        memhash_t h;
        memset(&h, 0, sizeof(h));
        h.x.G = G;
        h.x.L = ctx[0].L;
        h.x.seed_mask = ctx[0].seed_mask;
        h.x.keys = (const uint64_t**)keys;
        h.x.n = lens;
        h.x.gnseqi_end = prm->gnseqi_end_neg1 ? (int64_t)-1 : INT64_MAX;
        h.table_size = prm->table_size ? prm->table_size : 40000;
        h.seeds_only = prm->seeds_only;
        uint64_t* gbase = (uint64_t*)calloc((size_t)G + 1, sizeof(uint64_t));
        for (int g = 0; g < G; ++g) gbase[g + 1] = gbase[g] + m[g];
        h.gbase = gbase;
        h.buckets = (bucket_t*)calloc(h.table_size, sizeof(bucket_t));
        int64_t* scratch = (int64_t*)malloc((size_t)G * sizeof(int64_t));
        h.scratch = scratch;

        if (prm->parallel_compat) {
            bad = parallel_compat_search(&h, prm, G, lens, sml, m, res);
        } else {
            find_match_seeds(&h, prm, G, sml, m, lens, prm->start_points, res);
        }
        free(scratch);

        /* MemHash::GetMatchList: MemHash.h:182-203 (bucket-major) */
        res->count = h.mem_count;
        res->lengths = (uint64_t*)malloc((h.mem_count ? h.mem_count : 1) * sizeof(uint64_t));
        res->starts = (int64_t*)malloc((h.mem_count ? h.mem_count : 1) * (size_t)G * sizeof(int64_t));
        uint64_t o = 0;
        for (uint32_t bi = 0; bi < h.table_size; ++bi) {
            for (uint32_t k = 0; k < h.buckets[bi].n; ++k) {
                const mhe_t* e = &h.pool[h.buckets[bi].v[k]];
                res->lengths[o] = (uint64_t)e->len;
                memcpy(res->starts + o * (uint64_t)G, e->s, (size_t)G * sizeof(int64_t));
                ++o;
            }
            free(h.buckets[bi].v);
        }
        res->mem_count = h.mem_count;
        res->collision_count = h.collisions;
        res->probes = h.probes;
        if (!prm->parallel_compat && h.pool_n == h.mem_count) {   /* pool ids = insertion order */
            for (uint64_t k = 0; k < h.pool_n; ++k) mlog_push(res, (uint64_t)h.pool[k].len, h.pool[k].s, G);
        } else if (!prm->parallel_compat) {
            free(res->mlog_len); free(res->mlog_s);
            res->mlog_len = NULL; res->mlog_s = NULL; res->mlog_n = 0;
        }
        if ((prm->parallel_compat || h.pool_n == h.mem_count) && !res->mlog_len) {   /* an empty log */
            res->mlog_len = (uint64_t*)malloc(sizeof(uint64_t));
            res->mlog_s = (int64_t*)malloc((size_t)G * sizeof(int64_t));
        }
        free(h.buckets); free(h.pool); free(h.spool); free(gbase); free(h.cm); free(h.hl);
        res->plog_bucket = h.plog_bucket;
        res->plog_ref = h.plog_ref;
    }
done:
    for (int g = 0; g < G; ++g) { free(words[g]); free(keys[g]); free(sml[g]); }
    free(ctx); free(words); free(keys); free(sml); free(m);
    if (bad) { oracle_result_free(res); return NULL; }
    return res;
}

/* AddHashEntry replay of given probes (test aid for the sharded FindMatches): rows of
 * G+1 int64 {signed starts after SetDirection, offset} in AddHashEntry order; each is
 * looked up, extended and inserted exactly as in oracle_find_matches. */
/* ------------------------------------------------------------------------- */
/* OpenMP CPU path (the bench's CPU baseline on the host cores; TEST/BASELINE   */
/* INFRASTRUCTURE).  Same result as oracle_find_matches, bit for bit:           */
/*   1. per-genome keys + SortedMerList in parallel (MemorySML::Create per      */
/*      genome, MemorySML.cpp:45-60; the reference builds them one by one,      */
/*      MatchList.h:421);                                                        */
/*   2. the G-way merge (SearchRange, MatchFinder.cpp:172-340) split into key   */
/*      ranges cut at masked-key boundaries, one range per task; every          */
/*      AddHashEntry call is recorded as a row, in key order per range;         */
/*   3. rows grouped by hash bucket (stable), then the buckets replayed in      */
/*      parallel: AddHashEntry (MemHash.cpp:209-251) only ever touches its own  */
/*      bucket, and each bucket sees its calls in key order, so the bucket-     */
/*      major MatchList (MemHash.h:182-203) equals the serial one.              */
/* An input whose merge restarts (a group above MER_REPEAT_LIMIT), start points,*/
/* or the ParallelMemHash compat mode run the serial path instead.              */
/* ------------------------------------------------------------------------- */
#ifdef _OPENMP
#include <omp.h>
#endif

static uint64_t lower_bound_masked(const bmer_t* v, uint64_t n, uint64_t mask, uint64_t q) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if ((v[mid].key & mask) < q) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

oracle_result* oracle_find_matches_omp(int G, const char* const* seqs, const uint64_t* lens,
                                       const oracle_params* prm, int threads) {
    if (G < 1 || G > 64) return NULL;
    int serial_only = prm->parallel_compat || prm->start_points;
    if (serial_only) return oracle_find_matches(G, seqs, lens, prm);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    oracle_result* res = (oracle_result*)calloc(1, sizeof(oracle_result));
    res->G = G;
    sml_ctx* ctx = (sml_ctx*)calloc((size_t)G, sizeof(sml_ctx));
    uint32_t** words = (uint32_t**)calloc((size_t)G, sizeof(uint32_t*));
    uint64_t** keys = (uint64_t**)calloc((size_t)G, sizeof(uint64_t*));
    bmer_t** sml = (bmer_t**)calloc((size_t)G, sizeof(bmer_t*));
    uint64_t* m = (uint64_t*)calloc((size_t)G, sizeof(uint64_t));
    int bad = 0, fallback = 0;
    #pragma omp parallel for schedule(dynamic, 1) reduction(|:bad)
    for (int g = 0; g < G; ++g) {
        if (sml_init(&ctx[g], seqs[g], lens[g], prm->seed, &words[g])) { bad = 1; continue; }
        m[g] = sml_length(lens[g], ctx[g].L);
        keys[g] = (uint64_t*)malloc((m[g] ? m[g] : 1) * sizeof(uint64_t));
        for (uint64_t q = 0; q < m[g]; ++q) keys[g][q] = get_dna_seed_mer(&ctx[g], q);
        sml[g] = build_sml(&ctx[g], keys[g], m[g]);
    }
    if (bad) { res->count = 0; goto done; }
    for (int g = 0; g < G; ++g) res->seedmers += m[g];
    {
        const int L = ctx[0].L;
        const uint64_t mask = ctx[0].seed_mask;
        const uint32_t T = prm->table_size ? prm->table_size : 40000;
        uint64_t* gbase = (uint64_t*)calloc((size_t)G + 1, sizeof(uint64_t));
        for (int g = 0; g < G; ++g) gbase[g + 1] = gbase[g] + m[g];
        memhash_t base;
        memset(&base, 0, sizeof(base));
        base.x.G = G;
        base.x.L = L;
        base.x.seed_mask = mask;
        base.x.keys = (const uint64_t**)keys;
        base.x.n = lens;
        base.x.gnseqi_end = prm->gnseqi_end_neg1 ? (int64_t)-1 : INT64_MAX;
        base.table_size = T;
        base.gbase = gbase;
        /* key ranges: splitters = masked keys at quantiles of the longest SML */
        int big = 0;
        for (int g = 1; g < G; ++g) if (m[g] > m[big]) big = g;
        const int R = (int)(m[big] / 65536 + 1 < 4096 ? m[big] / 65536 + 1 : 4096);
        uint64_t* split = (uint64_t*)malloc((size_t)(R + 1) * sizeof(uint64_t));
        split[0] = 0;
        for (int r = 1; r < R; ++r) split[r] = sml[big][(uint64_t)r * m[big] / (uint64_t)R].key & mask;
        uint64_t* rlo = (uint64_t*)malloc((size_t)(R + 1) * (size_t)G * sizeof(uint64_t));
        #pragma omp parallel for schedule(static)
        for (int r = 0; r <= R; ++r)
            for (int g = 0; g < G; ++g)
                rlo[(uint64_t)r * G + g] = (r == R) ? m[g] : (r == 0 ? 0 : lower_bound_masked(sml[g], m[g], mask, split[r]));
        int64_t** rrows = (int64_t**)calloc((size_t)R, sizeof(int64_t*));
        uint64_t* rn = (uint64_t*)calloc((size_t)R, sizeof(uint64_t));
        uint64_t maxg = 0, restarts = 0;
        #pragma omp parallel for schedule(dynamic, 1) reduction(max:maxg) reduction(+:restarts)
        for (int r = 0; r < R; ++r) {
            memhash_t h = base;
            h.rec_cap = 1024;
            h.rec = (int64_t*)malloc(h.rec_cap * (size_t)(G + 1) * sizeof(int64_t));
            h.scratch = (int64_t*)malloc((size_t)G * sizeof(int64_t));
            oracle_result lr;
            memset(&lr, 0, sizeof(lr));
            uint64_t sp[64], sl[64];
            for (int g = 0; g < G; ++g) {
                sp[g] = rlo[(uint64_t)r * G + g];
                sl[g] = rlo[(uint64_t)(r + 1) * G + g] - sp[g];
            }
            if (!search_range_lit(&h, prm, G, sml, m, lens, sp, sl, &lr)) restarts += 1;
            if (lr.max_group > maxg) maxg = lr.max_group;
            rrows[r] = h.rec;
            rn[r] = h.rec_n;
            free(h.scratch); free(h.cm); free(h.hl);
        }
        if (restarts || maxg > MER_REPEAT_LIMIT) fallback = 1;   /* the merge would restart: serial */
        uint64_t P = 0;
        for (int r = 0; r < R; ++r) P += rn[r];
        const uint64_t W = (uint64_t)G + 1;
        /* stable grouping of the rows (key order) by hash bucket */
        uint32_t* rb = NULL;
        uint64_t* boff = NULL;
        uint64_t* order = NULL;
        if (!fallback) {
            int64_t** rowp = (int64_t**)malloc((P ? P : 1) * sizeof(int64_t*));
            rb = (uint32_t*)malloc((P ? P : 1) * sizeof(uint32_t));
            uint64_t k = 0;
            for (int r = 0; r < R; ++r)
                for (uint64_t i = 0; i < rn[r]; ++i, ++k) {
                    rowp[k] = rrows[r] + i * W;
                    const int64_t off = rowp[k][G];
                    rb[k] = (uint32_t)(((off % (int64_t)T) + (int64_t)T) % (int64_t)T);
                }
            res->probes = P;
            res->max_group = maxg;
            if (prm->seeds_only) {   /* the AddHashEntry call log, key order */
                res->plog_bucket = (uint32_t*)malloc((P ? P : 1) * sizeof(uint32_t));
                res->plog_ref = (uint64_t*)malloc((P ? P : 1) * sizeof(uint64_t));
                #pragma omp parallel for schedule(static)
                for (uint64_t i = 0; i < P; ++i) {
                    int f = 0;
                    while (rowp[i][f] == 0) ++f;
                    const int64_t s0 = rowp[i][f] < 0 ? -rowp[i][f] : rowp[i][f];
                    res->plog_bucket[i] = rb[i];
                    res->plog_ref[i] = gbase[f] + (uint64_t)(s0 - 1);
                }
            } else {
                boff = (uint64_t*)calloc((size_t)T + 1, sizeof(uint64_t));
                for (uint64_t i = 0; i < P; ++i) boff[rb[i] + 1]++;
                for (uint32_t b = 0; b < T; ++b) boff[b + 1] += boff[b];
                order = (uint64_t*)malloc((P ? P : 1) * sizeof(uint64_t));
                uint64_t* fill = (uint64_t*)malloc(((size_t)T + 1) * sizeof(uint64_t));
                memcpy(fill, boff, ((size_t)T + 1) * sizeof(uint64_t));
                for (uint64_t i = 0; i < P; ++i) order[fill[rb[i]]++] = i;
                free(fill);
                bucket_t* buckets = (bucket_t*)calloc(T, sizeof(bucket_t));
                int nth = 1;
#ifdef _OPENMP
                nth = omp_get_max_threads();
#endif
                memhash_t* th = (memhash_t*)calloc((size_t)nth, sizeof(memhash_t));
                int* owner = (int*)calloc(T, sizeof(int));
                #pragma omp parallel
                {
                    int tid = 0;
#ifdef _OPENMP
                    tid = omp_get_thread_num();
#endif
                    memhash_t* h = &th[tid];
                    *h = base;
                    h->buckets = buckets;
                    int64_t* sv = (int64_t*)malloc((size_t)G * sizeof(int64_t));
                    #pragma omp for schedule(dynamic, 16)
                    for (uint32_t b = 0; b < T; ++b) {
                        owner[b] = tid;
                        for (uint64_t j = boff[b]; j < boff[b + 1]; ++j) {
                            const int64_t* row = rowp[order[j]];
                            mhe_t pr;
                            memcpy(sv, row, (size_t)G * sizeof(int64_t));
                            pr.s = sv;
                            pr.len = L;
                            pr.mersize = L;
                            calc_offset(&pr, G);
                            add_hash_entry(h, &pr);
                        }
                    }
                    free(sv);
                }
                uint64_t M = 0, coll = 0;
                for (int t = 0; t < nth; ++t) { M += th[t].mem_count; coll += th[t].collisions; }
                res->count = M;
                res->mem_count = M;
                res->collision_count = coll;
                res->lengths = (uint64_t*)malloc((M ? M : 1) * sizeof(uint64_t));
                res->starts = (int64_t*)malloc((M ? M : 1) * (size_t)G * sizeof(int64_t));
                uint64_t o = 0;
                for (uint32_t b = 0; b < T; ++b) {
                    const memhash_t* h = &th[owner[b]];
                    for (uint32_t k2 = 0; k2 < buckets[b].n; ++k2) {
                        const mhe_t* e = &h->pool[buckets[b].v[k2]];
                        res->lengths[o] = (uint64_t)e->len;
                        memcpy(res->starts + o * (uint64_t)G, e->s, (size_t)G * sizeof(int64_t));
                        ++o;
                    }
                    free(buckets[b].v);
                }
                for (int t = 0; t < nth; ++t) { free(th[t].pool); free(th[t].spool); }
                free(th); free(owner); free(buckets);
            }
            free(rowp);
        }
        for (int r = 0; r < R; ++r) free(rrows[r]);
        free(rrows); free(rn); free(rlo); free(split); free(rb); free(boff); free(order); free(gbase);
    }
done:
    for (int g = 0; g < G; ++g) { free(words[g]); free(keys[g]); free(sml[g]); }
    free(ctx); free(words); free(keys); free(sml); free(m);
    if (bad) { oracle_result_free(res); return NULL; }
    if (fallback) { oracle_result_free(res); return oracle_find_matches(G, seqs, lens, prm); }
    return res;
}

int oracle_omp_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

oracle_result* oracle_replay_rows(int G, const char* const* seqs, const uint64_t* lens, const oracle_params* prm,
                                  const int64_t* rows, uint64_t nrows) {
    if (G < 1 || G > 64) return NULL;
    oracle_result* res = (oracle_result*)calloc(1, sizeof(oracle_result));
    res->G = G;
    sml_ctx* ctx = (sml_ctx*)calloc((size_t)G, sizeof(sml_ctx));
    uint32_t** words = (uint32_t**)calloc((size_t)G, sizeof(uint32_t*));
    uint64_t** keys = (uint64_t**)calloc((size_t)G, sizeof(uint64_t*));
    for (int g = 0; g < G; ++g) {
        if (sml_init(&ctx[g], seqs[g], lens[g], prm->seed, &words[g])) goto done;
        uint64_t m = sml_length(lens[g], ctx[g].L);
        keys[g] = (uint64_t*)malloc((m ? m : 1) * sizeof(uint64_t));
        for (uint64_t q = 0; q < m; ++q) keys[g][q] = get_dna_seed_mer(&ctx[g], q);
    }
    {
        memhash_t h;
        memset(&h, 0, sizeof(h));
        h.x.G = G;
        h.x.L = ctx[0].L;
        h.x.seed_mask = ctx[0].seed_mask;
        h.x.keys = (const uint64_t**)keys;
        h.x.n = lens;
        h.x.gnseqi_end = prm->gnseqi_end_neg1 ? (int64_t)-1 : INT64_MAX;
        h.table_size = prm->table_size ? prm->table_size : 40000;
        h.buckets = (bucket_t*)calloc(h.table_size, sizeof(bucket_t));
        int64_t* sv = (int64_t*)malloc((size_t)G * sizeof(int64_t));
        for (uint64_t r = 0; r < nrows; ++r) {
            const int64_t* row = rows + r * (uint64_t)(G + 1);
            mhe_t p;
            memcpy(sv, row, (size_t)G * sizeof(int64_t));
            p.s = sv;
            p.len = h.x.L;
            p.mersize = h.x.L;
            calc_offset(&p, G);
            add_hash_entry(&h, &p);
        }
        free(sv);
        res->count = h.mem_count;
        res->lengths = (uint64_t*)malloc((h.mem_count ? h.mem_count : 1) * sizeof(uint64_t));
        res->starts = (int64_t*)malloc((h.mem_count ? h.mem_count : 1) * (size_t)G * sizeof(int64_t));
        uint64_t o = 0;
        for (uint32_t bi = 0; bi < h.table_size; ++bi) {
            for (uint32_t k = 0; k < h.buckets[bi].n; ++k) {
                const mhe_t* e = &h.pool[h.buckets[bi].v[k]];
                res->lengths[o] = (uint64_t)e->len;
                memcpy(res->starts + o * (uint64_t)G, e->s, (size_t)G * sizeof(int64_t));
                ++o;
            }
            free(h.buckets[bi].v);
        }
        res->mem_count = h.mem_count;
        res->collision_count = h.collisions;
        res->probes = h.probes;
        free(h.buckets); free(h.pool); free(h.spool);
    }
done:
    for (int g = 0; g < G; ++g) { free(words[g]); free(keys[g]); }
    free(ctx); free(words); free(keys);
    return res;
}

uint64_t oracle_result_count(const oracle_result* r) { return r ? r->count : 0; }
int      oracle_result_seqcount(const oracle_result* r) { return r ? r->G : 0; }
void     oracle_result_copy(const oracle_result* r, uint64_t* lengths, int64_t* starts) {
    if (!r) return;
    if (lengths) memcpy(lengths, r->lengths, r->count * sizeof(uint64_t));
    if (starts) memcpy(starts, r->starts, r->count * (size_t)r->G * sizeof(int64_t));
}
uint64_t oracle_result_mem_count(const oracle_result* r) { return r ? r->mem_count : 0; }
uint64_t oracle_result_collision_count(const oracle_result* r) { return r ? r->collision_count : 0; }
uint64_t oracle_result_max_group(const oracle_result* r) { return r ? r->max_group : 0; }
uint64_t oracle_result_probe_count(const oracle_result* r) { return r ? r->probes : 0; }
/* seeds_only runs: the probe log (probe_count entries, AddHashEntry call order) */
int oracle_result_probe_log(const oracle_result* r, uint32_t* buckets, uint64_t* ref) {
    if (!r || !r->plog_bucket) return -1;
    if (buckets) memcpy(buckets, r->plog_bucket, r->probes * sizeof(uint32_t));
    if (ref) memcpy(ref, r->plog_ref, r->probes * sizeof(uint64_t));
    return 0;
}
uint64_t oracle_result_seedmers(const oracle_result* r) { return r ? r->seedmers : 0; }
uint64_t oracle_result_chunks(const oracle_result* r) { return r ? r->chunks : 0; }
uint64_t oracle_result_restarts(const oracle_result* r) { return r ? r->restarts : 0; }
/* rows = restarts, G entries each; returns 0 */
int oracle_result_match_log(const oracle_result* r, uint64_t* lengths, int64_t* starts) {
    if (!r->mlog_len) return -1;
    if (lengths) memcpy(lengths, r->mlog_len, r->mlog_n * sizeof(uint64_t));
    if (starts) memcpy(starts, r->mlog_s, r->mlog_n * (size_t)r->G * sizeof(int64_t));
    return 0;
}
/* lines of the match log (MemCount for MemHash; thread-table + MergeTable inserts in compat) */
uint64_t oracle_result_match_log_count(const oracle_result* r) { return r ? r->mlog_n : 0; }

int oracle_result_offset_log(const oracle_result* r, uint64_t* out) {
    if (!r) return -1;
    if (r->offlog && r->restarts) memcpy(out, r->offlog, (size_t)r->restarts * (size_t)r->offlog_g * sizeof(uint64_t));
    return 0;
}
/* LogProgress text of the last FindMatches ("" unless the serial MemHash path ran) */
const char* oracle_result_progress(const oracle_result* r) { return (r && r->prog) ? r->prog : ""; }

void     oracle_result_free(oracle_result* r) {
    if (!r) return;
    free(r->prog);
    free(r->lengths); free(r->starts); free(r->plog_bucket); free(r->plog_ref); free(r->offlog);
    free(r->mlog_len); free(r->mlog_s); free(r);
}

/* ------------------------------------------------------------------------- */
/* Synthetic genomes: SURVEY.md Appendix C (std::mt19937_64 restated).        */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t mt[312]; int idx; } mt64_t;

static void mt64_seed(mt64_t* r, uint64_t s) {
    r->mt[0] = s;
    for (int i = 1; i < 312; ++i)
        r->mt[i] = 6364136223846793005ULL * (r->mt[i - 1] ^ (r->mt[i - 1] >> 62)) + (uint64_t)i;
    r->idx = 312;
}

static uint64_t mt64_next(mt64_t* r) {
    if (r->idx >= 312) {
        for (int i = 0; i < 312; ++i) {
            uint64_t x = (r->mt[i] & 0xFFFFFFFF80000000ULL) | (r->mt[(i + 1) % 312] & 0x7FFFFFFFULL);
            uint64_t xa = x >> 1;
            if (x & 1) xa ^= 0xB5026F5AA96619E9ULL;
            r->mt[i] = r->mt[(i + 156) % 312] ^ xa;
        }
        r->idx = 0;
    }
    uint64_t y = r->mt[r->idx++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= y >> 43;
    return y;
}

void oracle_generate(int G, uint64_t n, double p, uint64_t rng_seed, char* out) {
    static const char acgt[4] = {'A', 'C', 'G', 'T'};
    mt64_t r;
    mt64_seed(&r, rng_seed);
    for (uint64_t i = 0; i < n; ++i) out[i] = acgt[mt64_next(&r) & 3];
    const double thr = p * 1e6;
    for (int g = 1; g < G; ++g) {
        char* d = out + (uint64_t)g * n;
        memcpy(d, out, n);
        for (uint64_t i = 0; i < n; ++i)
            if ((double)(mt64_next(&r) % 1000000) < thr) d[i] = acgt[mt64_next(&r) & 3];
        if (g == 2) {
            for (uint64_t a = 0, b = n ? n - 1 : 0; a < b; ++a, --b) { char t = d[a]; d[a] = d[b]; d[b] = t; }
            for (uint64_t i = 0; i < n; ++i) {
                char c = d[i];
                d[i] = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'A';
            }
        }
    }
}
