/* TEST INFRASTRUCTURE ONLY -- a literal, reentrant restatement of libstdc++'s std::sort
 * (GCC bits/stl_algo.h / stl_heap.h) over uint32 ids compared by key[id] (the reference's
 * comparators compare one integer: bmer_lessthan, SortedMerList.h:311-314, and
 * SingleStartComparator, AbstractMatch.h:324-351).  Both std::sort call sites of the hot
 * path leave ties in introsort order, which is part of the reference's output:
 *   - MemorySML::Create (MemorySML.cpp:54): the order of equal seed mers in every
 *     SortedMerList (observable through GetBreakpoint's FindMer + 1, MatchFinder.cpp:113-121,
 *     the MER_REPEAT_LIMIT restart, ParallelMemHash's chunk starts, repeat / enumeration
 *     tolerance and the SML itself);
 *   - EliminateOverlaps (Aligner.cpp:62-176).
 * __introsort_loop (_S_threshold 16, depth 2 * __lg(n)), __move_median_to_first,
 * __unguarded_partition, __partial_sort (heap select + sort_heap), __final_insertion_sort.
 * Pinned against the real std::sort of this toolchain by tests/eo_model.cpp and
 * tests/sml_sort_model.cpp.  Only tests/ and bench.py's CPU baseline reach this code. */
#ifndef MUMS_ORACLE_STD_SORT_H
#define MUMS_ORACLE_STD_SORT_H

#include <stdint.h>
#include <string.h>

#define SS_LT(K, a, b) ((K)[(a)] < (K)[(b)])

static inline void ss_swap(uint32_t* a, uint32_t* b) { uint32_t t = *a; *a = *b; *b = t; }

static inline void ss_move_median_to_first(const uint64_t* K, uint32_t* result, uint32_t* a, uint32_t* b,
                                           uint32_t* c) {
    if (SS_LT(K, *a, *b)) {
        if (SS_LT(K, *b, *c)) ss_swap(result, b);
        else if (SS_LT(K, *a, *c)) ss_swap(result, c);
        else ss_swap(result, a);
    } else if (SS_LT(K, *a, *c)) ss_swap(result, a);
    else if (SS_LT(K, *b, *c)) ss_swap(result, c);
    else ss_swap(result, b);
}

static inline uint32_t* ss_unguarded_partition(const uint64_t* K, uint32_t* first, uint32_t* last,
                                               uint32_t* pivot) {
    for (;;) {
        while (SS_LT(K, *first, *pivot)) ++first;
        --last;
        while (SS_LT(K, *pivot, *last)) --last;
        if (!(first < last)) return first;
        ss_swap(first, last);
        ++first;
    }
}

static inline void ss_push_heap(const uint64_t* K, uint32_t* first, int64_t hole, int64_t top, uint32_t value) {
    int64_t parent = (hole - 1) / 2;
    while (hole > top && SS_LT(K, first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

static inline void ss_adjust_heap(const uint64_t* K, uint32_t* first, int64_t hole, int64_t len, uint32_t value) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (SS_LT(K, first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    ss_push_heap(K, first, hole, top, value);
}

/* __partial_sort(first, last, last): __heap_select (make_heap; nothing after middle) then
 * __sort_heap (__pop_heap from the back) */
static inline void ss_heap_sort(const uint64_t* K, uint32_t* first, uint32_t* last) {
    const int64_t len = last - first;
    if (len >= 2) {
        for (int64_t parent = (len - 2) / 2;; --parent) {
            ss_adjust_heap(K, first, parent, len, first[parent]);
            if (parent == 0) break;
        }
    }
    while (last - first > 1) {
        --last;
        const uint32_t value = *last;
        *last = *first;
        ss_adjust_heap(K, first, 0, last - first, value);
    }
}

static inline void ss_introsort_loop(const uint64_t* K, uint32_t* first, uint32_t* last, int64_t depth_limit) {
    while (last - first > 16) {
        if (depth_limit == 0) {
            ss_heap_sort(K, first, last);
            return;
        }
        --depth_limit;
        uint32_t* mid = first + (last - first) / 2;
        ss_move_median_to_first(K, first, first + 1, mid, last - 1);
        uint32_t* cut = ss_unguarded_partition(K, first + 1, last, first);
        ss_introsort_loop(K, cut, last, depth_limit);
        last = cut;
    }
}

static inline void ss_unguarded_linear_insert(const uint64_t* K, uint32_t* last) {
    const uint32_t val = *last;
    uint32_t* next = last - 1;
    while (SS_LT(K, val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

static inline void ss_insertion_sort(const uint64_t* K, uint32_t* first, uint32_t* last) {
    if (first == last) return;
    for (uint32_t* i = first + 1; i != last; ++i) {
        if (SS_LT(K, *i, *first)) {
            const uint32_t val = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(uint32_t));   /* move_backward */
            *first = val;
        } else {
            ss_unguarded_linear_insert(K, i);
        }
    }
}

/* std::sort(ids, ids + n, [K](a, b) { return K[a] < K[b]; }); depth < 0: 2 * __lg(n) */
static inline void ss_std_sort(const uint64_t* K, uint32_t* ids, uint64_t n, int64_t depth) {
    if (n == 0) return;
    if (depth < 0) depth = 2 * (int64_t)(63 - __builtin_clzll(n));
    ss_introsort_loop(K, ids, ids + n, depth);
    if (n > 16) {
        ss_insertion_sort(K, ids, ids + 16);
        for (uint32_t* i = ids + 16; i != ids + n; ++i) ss_unguarded_linear_insert(K, i);
    } else {
        ss_insertion_sort(K, ids, ids + n);
    }
}

#endif
