// restart_plan.h -- MatchFinder::SearchRange's MER_REPEAT_LIMIT restart, planned on
// the per-genome sorted mer lists (host/device shared code).
//
// Reference: MatchFinder::SearchRange (MatchFinder.cpp:172-340) merges the G sorted mer
// lists through a std::list of buffer heads.  When more than MER_REPEAT_LIMIT (1000)
// records of one masked key K have been collected and another head still carries K
// (the check at the top of every merge iteration, :253), the group is dropped and the
// merge restarts (FindMatchSeeds, :145) from new start points:
//   next_mer = K + 1; seqI = the first SML whose FindMer(next_mer) position (+1 when
//   absent) lies inside it (:257-263); start_points = GetBreakpoint(seqI, next_pos)
//   (:89-126: the group start of that record's key in seqI; FindMer of its full key
//   in the others, one past the hit because the backward loop compares with a bool,
//   :117-121), never moved backwards past what was consumed (:271-272), SMLs before
//   seqI exhausted (:273-274).
//
// The GPU path merges all genomes with one sort, so this header restates the merge
// order only where it matters: for a key group K of more than 1000 live records it
// derives
//   * the head order of the std::list at K (the order in which the genomes' runs of K
//     are collected): a head is inserted in front of the heads of equal key, when the
//     genome's previous run completes; so two genomes compare by their previous keys
//     (larger first), ties by their order at that previous key, reversed -- a walk back
//     over the distinct keys with alternating direction, done by partition refinement;
//     heads read at the start of a SearchRange call are ordered by genome id;
//   * the collection steps: each genome's run split at its 10000-record buffer
//     boundaries (MER_BUFFER_SIZE, :175; buffers start at the call's start points), plus
//     one empty step when a run ends exactly on a boundary with more records to read;
//   * whether the check fires (more than 1000 collected before some step) and the
//     consumed position of every genome (start + mer_baseindex + mer_index).
// Records live in phase p (keys from the p-th restart key on) iff their SML index is at
// least the phase's start point; restart_plan() returns the restart keys and the start
// points of every phase.  SML arrays hold the compact canonical key
// ckey = (v << 1) | parity (v = the 2w-bit spaced seed), whose order equals the
// reference's full-key order (bmer_lessthan, SortedMerList.h:311-314).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MUMS_HD __host__ __device__
#else
#define MUMS_HD
#endif

namespace mums {
namespace restart {

constexpr int kMaxGenomes = 64;
constexpr uint64_t kRepeatLimit = 1000;   // MER_REPEAT_LIMIT, MatchFinder.cpp:166
constexpr uint64_t kMerBuffer = 10000;    // MER_BUFFER_SIZE, MatchFinder.cpp:175

// per-genome sorted mer lists: genome g's SML = ck[base[g] .. base[g] + m[g]).
// Distributed (off != nullptr, the sharded mode): this rank holds genome g's SML indices
// [off[g], off[g] + n[g]) at ck[base[g] ..], the records of its key range [key_lo, key_hi)
// (full keys; both bounds even: a masked key never straddles two ranks).  Of the other
// indices it knows the keys next to its range: prv[g] at off[g] - 1 (the last key of genome g
// on a lower rank) and nxt[g] at off[g] + n[g] (the first on a higher one).  kc() answers every
// index -- below the range with prv[g] (an upper bound), above it with nxt[g] (a lower bound):
// exact at the two neighbours, and comparing like the real key against any query in
// [key_lo, key_hi] -- what the binary searches need.  kx() needs the real key: outside
// [off[g] - 1, off[g] + n[g]] it flags *bad (the plan is then made on the gathered streams).
struct PlanData {
    int G;
    const uint64_t* m;
    const uint64_t* base;
    const uint64_t* ck;
    const uint64_t* off = nullptr;
    const uint64_t* n = nullptr;
    const uint64_t* prv = nullptr;
    const uint64_t* nxt = nullptr;
    uint64_t key_lo = 0, key_hi = ~0ull;
    unsigned* bad = nullptr;
    MUMS_HD void flag() const {
        if (bad) *bad = 1u;
    }
    MUMS_HD uint64_t kc(int g, uint64_t i) const {
        if (!off) return ck[base[g] + i];
        if (i < off[g]) return prv[g];
        if (i - off[g] >= n[g]) return nxt[g];
        return ck[base[g] + (i - off[g])];
    }
    MUMS_HD uint64_t kx(int g, uint64_t i) const {
        if (off && (i + 1 < off[g] || i > off[g] + n[g])) flag();
        return kc(g, i);
    }
    // a query key the stand-ins cannot answer (beyond this rank's key range)
    MUMS_HD void need(uint64_t q) const {
        if (off && q >= key_hi) flag();
    }
};

// first index i in [lo, hi) of genome g's SML with key >= x (i = hi if none)
MUMS_HD inline uint64_t lower_bound_g(const PlanData& d, int g, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (d.kc(g, mid) < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// first index i in a[0, n) with a[i] >= x
MUMS_HD inline uint64_t lower_bound_u64(const uint64_t* a, uint64_t n, uint64_t x) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// SortedMerList::bsearch (SortedMerList.cpp:380-394), recursion unrolled, unsigned
MUMS_HD inline uint64_t ref_bsearch(const PlanData& d, int g, uint64_t q, uint64_t start, uint64_t end) {
    for (;;) {
        const uint64_t middle = (start + end) / 2;
        const uint64_t k = d.kc(g, middle);
        if (k == q) return middle;
        if (k < q && middle < end) start = middle + 1;
        else if (k > q && start < middle) end = middle - 1;
        else return middle;
    }
}

// SortedMerList::FindMer (SortedMerList.cpp:170-179) on genome g's SML of m records (m = 0
// <=> sequence shorter than the seed: early return, *result untouched).
MUMS_HD inline bool ref_find_mer(const PlanData& d, int g, uint64_t q, uint64_t* result) {
    const uint64_t m = d.m[g];
    if (m == 0) return false;
    d.need(q);
    *result = ref_bsearch(d, g, q, 0, m - 1);
    return d.kc(g, *result) == q;   // (a stand-in never equals a query of this key range)
}

// Per candidate key v (masked, i.e. ckey >> 1): the run [lo, hi) of v in every SML and
// the restart target that depends on the key only: seqI (:257-263; G when none) and the
// GetBreakpoint(seqI, next_pos) start points bp[g] (:89-126).
MUMS_HD inline void cand_precompute(const PlanData& d, uint64_t v, uint64_t* lo, uint64_t* hi, uint64_t* bp,
                                    int* seq_out) {
    const int G = d.G;
    for (int g = 0; g < G; ++g) {
        lo[g] = lower_bound_g(d, g, 0, d.m[g], v << 1);
        hi[g] = lower_bound_g(d, g, 0, d.m[g], (v + 1) << 1);
        bp[g] = 0;
    }
    const uint64_t next = (v + 1) << 1;   // next_mer = K + (~mer_mask + 1), forward parity
    uint64_t next_pos = 0;
    int s = 0;
    for (; s < G; ++s) {
        if (!ref_find_mer(d, s, next, &next_pos)) ++next_pos;
        if (next_pos < d.m[s]) break;
    }
    *seq_out = s;
    if (s >= G) return;
    const uint64_t brk = d.kx(s, next_pos);
    const uint64_t start = lower_bound_g(d, s, 0, next_pos + 1, (brk >> 1) << 1);   // backward loop :104-112
    for (int i = 0; i < G; ++i) {
        if (i == s) { bp[i] = start; continue; }
        uint64_t cur = 0;   // the reference's uninitialised cur_start (only for empty SMLs)
        if (ref_find_mer(d, i, brk, &cur)) {
            // (matchmer.mer & mer_mask) == (break_mer.mer && mer_mask): true only for the
            // all-A key hit by a zero break key; the loop then runs down to -1
            const bool runs = (d.kx(i, cur) >> 1) == 0 && brk == 0;
            cur = runs ? 0 : cur + 1;
        }
        bp[i] = cur;
    }
}

// first index of genome g's masked-key run containing p (key >> 1 == X), galloping backwards
// (a masked-key run of this rank's key range ends at its lower edge: kc's stand-in there is
// smaller; the run of prv[g] at off[g] - 1 lies on a lower rank)
MUMS_HD inline uint64_t run_start_back(const PlanData& d, int g, uint64_t p, uint64_t X) {
    if (d.off && p < d.off[g] && p > 0) d.flag();
    uint64_t good = p, step = 1;
    int64_t bad = -1;
    for (;;) {
        if (good >= step && (d.kc(g, good - step) >> 1) == X) {
            good -= step;
            step <<= 1;
        } else {
            bad = good >= step ? (int64_t)(good - step) : -1;
            break;
        }
    }
    uint64_t lo = (uint64_t)(bad + 1), hi = good;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if ((d.kc(g, mid) >> 1) < X) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

struct OrderClass {
    uint64_t mask;
    uint32_t cnt;   // distinct keys walked at which every member was present
};

// Head order of the genomes in U at key K (run starts a[g]) in the SearchRange call
// with start points S.  ord[] receives the genomes, first head first; returns |U|.
// Partition refinement over the distinct keys before K, walking down: a class splits
// at the first key only some members hold; those holding it were re-inserted later at
// that depth -- first in the list when the number of keys shared so far is even,
// last when odd.  Members that share their whole history since the call's start were
// read as initial heads: ascending ids (even) / descending ids (odd).
MUMS_HD inline int head_order(const PlanData& d, uint64_t U, const uint64_t* a, const uint64_t* S, int* ord,
                              uint64_t* walk_steps) {
    const int G = d.G;
    OrderClass cls[kMaxGenomes];
    int ncls = 1;
    cls[0].mask = U;
    cls[0].cnt = 0;
    uint64_t p[kMaxGenomes];
    uint64_t active = 0;
    for (int g = 0; g < G; ++g) {
        p[g] = 0;
        if (((U >> g) & 1) && a[g] > S[g]) {
            p[g] = a[g] - 1;
            active |= 1ull << g;
        }
    }
    for (;;) {
        bool more = false;
        for (int c = 0; c < ncls; ++c)
            if ((cls[c].mask & (cls[c].mask - 1)) != 0 && (cls[c].mask & active) != 0) more = true;
        if (!more) break;
        uint64_t X = 0;
        bool any = false;
        for (int g = 0; g < G; ++g) {
            if (!((active >> g) & 1)) continue;
            const uint64_t x = d.kx(g, p[g]) >> 1;
            if (!any || x > X) { X = x; any = true; }
        }
        uint64_t pres = 0;
        for (int g = 0; g < G; ++g)
            if (((active >> g) & 1) && (d.kx(g, p[g]) >> 1) == X) pres |= 1ull << g;
        ++*walk_steps;
        // fold the key into the classes (in order)
        OrderClass nc[kMaxGenomes];
        int n2 = 0;
        for (int c = 0; c < ncls; ++c) {
            const uint64_t A = cls[c].mask & pres, B = cls[c].mask & ~pres;
            if (A == 0) { nc[n2++] = cls[c]; continue; }
            if (B == 0) { nc[n2] = cls[c]; nc[n2].cnt++; ++n2; continue; }
            const uint32_t depth = cls[c].cnt + 1;
            OrderClass ca{A, cls[c].cnt + 1}, cb{B, cls[c].cnt};
            if (depth & 1u) { nc[n2++] = ca; nc[n2++] = cb; }
            else { nc[n2++] = cb; nc[n2++] = ca; }
        }
        for (int c = 0; c < n2; ++c) cls[c] = nc[c];
        ncls = n2;
        // step the holders back past their run of X
        for (int g = 0; g < G; ++g) {
            if (!((pres >> g) & 1)) continue;
            const uint64_t st = run_start_back(d, g, p[g], X);
            if (st > S[g]) p[g] = st - 1;
            else active &= ~(1ull << g);
        }
    }
    int n = 0;
    for (int c = 0; c < ncls; ++c) {
        const uint64_t mk = cls[c].mask;
        if ((cls[c].cnt & 1u) == 0) {
            for (int g = 0; g < G; ++g)
                if ((mk >> g) & 1) ord[n++] = g;
        } else {
            for (int g = G - 1; g >= 0; --g)
                if ((mk >> g) & 1) ord[n++] = g;
        }
    }
    return n;
}

enum PlanStatus { kPlanOk = 0, kPlanTableFull = 1 };

struct PlanOut {
    uint64_t nrestarts;      // restarts recorded in rkey / rS
    uint64_t cap;            // capacity of rkey (rS holds cap * G)
    uint64_t* rkey;          // masked key of every dropped group (ascending)
    uint64_t* rS;            // start points after restart r: rS[r * G + g]
    uint64_t walk_steps;     // distinct keys walked for head orders (diagnostic)
    uint64_t checked;        // candidates with more than 1000 live records
    int status;
    uint64_t* rC;            // optional: consumed SML position of every genome at restart r: rC[r * G + g]
};

// Consume the candidates (groups of > 1000 records, ascending masked keys cand[c], with
// cand_precompute results clo / chi / cbp [c * G + g] and cseq[c]) in key order with the
// running start points S (in: the FindMatchSeeds start offsets; out: the last phase's).
// cbad (distributed): cand_precompute needed a key of another rank for candidate c -- its
// restart target is unknown, so firing it flags d.bad.
MUMS_HD inline void restart_plan(const PlanData& d, const uint64_t* cand, uint64_t C, const uint64_t* clo,
                                 const uint64_t* chi, const uint64_t* cbp, const int* cseq, uint64_t* S,
                                 PlanOut* out, const unsigned* cbad = nullptr) {
    const int G = d.G;
    for (uint64_t c = 0; c < C; ++c) {
        const uint64_t* lo = clo + c * (uint64_t)G;
        const uint64_t* hi = chi + c * (uint64_t)G;
        uint64_t a[kMaxGenomes], b[kMaxGenomes];
        uint64_t tot = 0, U = 0;
        for (int g = 0; g < G; ++g) {
            a[g] = lo[g] > S[g] ? lo[g] : S[g];
            b[g] = hi[g] > S[g] ? hi[g] : S[g];
            if (b[g] > a[g]) {
                tot += b[g] - a[g];
                U |= 1ull << g;
            }
        }
        if (tot <= kRepeatLimit) continue;
        ++out->checked;
        int ord[kMaxGenomes];
        const int n = head_order(d, U, a, S, ord, &out->walk_steps);
        // collection steps in head order; the check precedes every step (:253)
        uint64_t consumed[kMaxGenomes];
        for (int g = 0; g < G; ++g) consumed[g] = ((U >> g) & 1) ? a[g] : b[g];   // others: head past K
        uint64_t cum = 0;
        bool fired = false;
        for (int k = 0; k < n && !fired; ++k) {
            const int g = ord[k];
            uint64_t x = a[g];
            while (x < b[g]) {
                if (cum > kRepeatLimit) { fired = true; break; }
                const uint64_t nb = S[g] + ((x - S[g]) / kMerBuffer + 1) * kMerBuffer;
                const uint64_t y = b[g] < nb ? b[g] : nb;
                cum += y - x;
                x = y;
                consumed[g] = x;
            }
            // a run ending on a buffer boundary: the refilled head still carries K for
            // one more iteration (nothing collected), unless the SML is exhausted
            if (!fired && (b[g] - S[g]) % kMerBuffer == 0 && b[g] < d.m[g] && cum > kRepeatLimit) fired = true;
        }
        if (!fired) continue;
        if (cbad && cbad[c]) d.flag();
        if (out->nrestarts >= out->cap) { out->status = kPlanTableFull; return; }
        const int s = cseq[c];
        const uint64_t* bp = cbp + c * (uint64_t)G;
        uint64_t* ns = out->rS + out->nrestarts * (uint64_t)G;
        if (out->rC)   // LogProgress: buffers of that phase ending at or before these positions were exhausted
            for (int g = 0; g < G; ++g) out->rC[out->nrestarts * (uint64_t)G + g] = consumed[g];
        for (int g = 0; g < G; ++g) {
            uint64_t v = s < G ? bp[g] : S[g];
            if (v < consumed[g]) v = consumed[g];   // don't allow it to move backwards (:271-272)
            if (g < s) v = d.m[g];                   // :273-274
            ns[g] = v;
        }
        for (int g = 0; g < G; ++g) S[g] = ns[g];
        out->rkey[out->nrestarts++] = cand[c];
    }
}

}  // namespace restart
}  // namespace mums
