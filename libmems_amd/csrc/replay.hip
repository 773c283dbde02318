// replay.hip -- per-bucket AddHashEntry replay (rows A10-A12).
//
// Reference: MemHash::AddHashEntry (MemHash.cpp:209-251) keeps every hash
// bucket as a vector sorted by MheCompare (MatchHashEntry.h:121-143); each probe
// is looked up with std::lower_bound, dropped as a collision when the entry
// there is equivalent, otherwise extended (MatchFinder::ExtendMatch,
// MatchFinder.h:218-374) and inserted at lower_bound of the extended copy
// (whose m_mersize is 0, MatchHashEntry.cpp:122).  Because MheCompare treats
// containment as equivalence it is not a strict weak ordering, so the exact
// binary-search probe sequence matters; it is replayed here
// with the libstdc++ __lower_bound recurrence.
//
// MI355X mapping: one workgroup (1024 / 512 / 256 lanes for G <= 4 / 8 / more) per hash bucket.
// Extensions are not computed here: chains.hip has labelled every probe with its
// chain, whose extended entry sits in the chain pool, so an insert is a pool id.
// The bucket's vector lives in LDS as 16-B slots {id, presence mask, first-genome
// start, length} (spilling to a global slice when it outgrows the LDS capacity), so
// the binary search reads LDS and touches an entry in HBM only where a span could
// contain the probe.  A window of up to RB consecutive probes stays in the lanes'
// registers; per round every unconsumed lane runs its lower_bound against the
// current vector, the workgroup takes the first non-colliding probe (ballot),
// inserts its chain entry with a one-barrier LDS shift and goes on after it.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "match_device.h"
#include "seed_device.h"

namespace mums {

namespace {

// MemHash::SetMatchLog (MemHash.h:149, written at MemHash.cpp:238-241): every insert, as
// (AddHashEntry call = probe index in key order, chain), sorted by the call afterwards
__device__ __forceinline__ void log_insert(uint64_t* mlog, DevCounters* ctr, uint32_t probe, uint32_t cid) {
    if (mlog) mlog[atomicAdd(&ctr->log_n, 1ull)] = ((uint64_t)probe << 32) | cid;
}

template <int RB>
__device__ __forceinline__ int block_first_true(bool pred, int* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t b = __ballot(pred);
    if (lane == 0) red[wv] = b ? wv * 64 + (__ffsll((long long)b) - 1) : RB;
    __syncthreads();
    int r = red[0];
    #pragma unroll
    for (int w = 1; w < RB / 64; ++w) r = min(r, red[w]);
    __syncthreads();
    return r;
}

// A vector slot: {pool id, block key, first-genome start, length}.  The block key orders
// presence masks (bit g = genome g) as MheCompare does -- FirstStart index descending,
// then the first genome present in only one: absent first -- i.e. as bitreverse(mask):
// bitreverse32(mask) itself up to 32 genomes, its dense rank among the chains' masks
// beyond (block_keys).  The slot decides MheCompare (MatchHashEntry.h:121-143) without
// the entry unless one first-genome span can contain the other:
//   * X is V's own chain entry (same pool id): X contains V -> equivalent
//   * masks differ: block key order
//   * same mask, V starts before X: only V can contain X (needs X's span inside V's)
//   * same mask, V starts after X : only X can contain V (needs V's span inside X's)
// with no containment possible, strict_start_lessthan_ptr is decided by the first
// genome's (positive) start.  Returns 0 / 1 (X < V false / true), 2 = needs the entries.
__device__ __forceinline__ int slot_cmp(const uint4 X, uint32_t vmask, int64_t vs, int64_t vl, uint32_t vcid) {
    if (X.x == vcid) return 0;
    if (X.y != vmask) return X.y < vmask ? 1 : 0;
    const int64_t xs = (int64_t)X.z, xl = (int64_t)X.w;
    if (vs < xs) return (xs + xl > vs + vl) ? 0 : 2;
    if (vs > xs) return (vs + vl > xs + xl) ? 1 : 2;
    return 2;
}

// can X and V be equivalent (one contains the other)?  0 no, 1 yes, 2 needs the entries
__device__ __forceinline__ int slot_equiv(const uint4 X, uint32_t vmask, int64_t vs, int64_t vl, uint32_t vcid) {
    if (X.x == vcid) return 1;
    if (X.y != vmask) return 0;
    const int64_t xs = (int64_t)X.z, xl = (int64_t)X.w;
    if (vs < xs) return (xs + xl > vs + vl) ? 0 : 2;
    if (vs > xs) return (vs + vl > xs + xl) ? 0 : 2;
    return 2;
}

// std::lower_bound (libstdc++: half = len >> 1, middle = first + half) over slots
// tb[0..t); full(id) = MheCompare(entry id, V) for the rare undecided slots
template <typename Acc, typename Full>
__device__ __forceinline__ uint32_t lower_bound_acc(Acc&& at, uint32_t t, uint32_t vmask, int64_t vs, int64_t vl,
                                                   uint32_t vcid, Full&& full) {
    uint32_t first = 0, len = t;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        const uint4 X = at(mid);
        int r = slot_cmp(X, vmask, vs, vl, vcid);
        if (r == 2) r = full(X.x) ? 1 : 0;
        if (r) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

template <typename Full>
__device__ __forceinline__ uint32_t lower_bound_slots(const uint4* tb, uint32_t t, uint32_t vmask, int64_t vs,
                                                     int64_t vl, uint32_t vcid, Full&& full) {
    uint32_t first = 0, len = t;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        const uint4 X = tb[mid];
        int r = slot_cmp(X, vmask, vs, vl, vcid);
        if (r == 2) r = full(X.x) ? 1 : 0;
        if (r) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

// block key of a probe: bitreverse32(presence mask) up to 32 genomes, else its chain's
// dense rank (bkey, from block_keys)
template <int MG>
__device__ __forceinline__ uint32_t block_key(const Mhe<MG>& m, int G, const uint32_t* __restrict__ bkey,
                                              uint32_t cid) {
    if constexpr (MG > 32) {
        return bkey[cid];
    } else {
        uint32_t k = 0;
        #pragma unroll
        for (int g = 0; g < MG; ++g) k |= (g < G && m.s[g] != 0) ? (1u << g) : 0u;
        return __builtin_bitreverse32(k);
    }
}

// more than 32 genomes: bitreverse64(presence mask) of every chain entry, then each
// chain's dense rank among them (block_keys)
__global__ __launch_bounds__(kBlock) void chain_bmask_kernel(const int64_t* __restrict__ pool, uint32_t nch, int G,
                                                             uint64_t* __restrict__ out) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= nch) return;
    const int64_t* e = pool + (uint64_t)c * (uint64_t)(G + 2);
    uint64_t m = 0;
    for (int g = 0; g < G; ++g) m |= e[2 + g] != 0 ? (1ull << g) : 0ull;
    out[c] = __builtin_bitreverse64(m);
}

__global__ __launch_bounds__(kBlock) void dense_step_kernel(const uint64_t* __restrict__ skey, uint32_t n,
                                                            uint32_t* __restrict__ step) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) step[i] = (i + 1 < n && skey[i + 1] != skey[i]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void dense_scatter_kernel(const uint32_t* __restrict__ ord,
                                                               const uint32_t* __restrict__ rank, uint32_t n,
                                                               uint32_t* __restrict__ bkey) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) bkey[ord[i]] = rank[i];
}

// Sort keys of the chain entries: (hash bucket, block key) and first-genome start (the
// block key orders blocks as MheCompare does, see slot_cmp).
__global__ __launch_bounds__(kBlock) void chain_keys_kernel(const int64_t* __restrict__ pool, uint32_t nch, int G,
                                                            uint32_t table_size, double inv_t,
                                                            const uint32_t* __restrict__ bkey,
                                                            uint64_t* __restrict__ key_s, uint64_t* __restrict__ key_b) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= nch) return;
    const int64_t* e = pool + (uint64_t)c * (uint64_t)(G + 2);
    uint32_t m = 0;
    int64_t s0 = 0;
    for (int g = G - 1; g >= 0; --g) {
        const int64_t sg = e[2 + g];
        if (sg != 0) { m |= g < 32 ? 1u << g : 0u; s0 = sg; }
    }
    key_s[c] = (uint64_t)s0;
    key_b[c] = ((uint64_t)bucket_of_fast(e[1], table_size, inv_t) << 32) | (bkey ? bkey[c] : __builtin_bitreverse32(m));
}

// (bucket, block key) of chain idx[i] packed on kb + bucket bits: the block key's kb
// significant bits (the bit-reversed G-genome mask sits in the top G of its 32 bits; dense
// block ranks are < 2^kb) under the bucket, so the sort that follows needs few passes
__global__ __launch_bounds__(kBlock) void gather_gkey_kernel(const uint64_t* __restrict__ key_b,
                                                             const uint32_t* __restrict__ idx, uint32_t n,
                                                             int low_shift, int kb, uint64_t* __restrict__ dst) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t b = key_b[idx[i]];
    dst[i] = ((b >> 32) << kb) | (uint64_t)((uint32_t)b >> low_shift);
}

// next_s[c] = smallest first-genome start >= c's among the OTHER chains of c's bucket
// and presence mask (c's own start on a tie), ~0 if none.  rank[c] = c's index in
// (bucket, block, start) order = MheCompare order inside a bucket, bit 31 set when
// another chain of the block has the same start (order then decided by later genomes).
__global__ __launch_bounds__(kBlock) void chain_next_kernel(const uint32_t* __restrict__ ord,
                                                            const uint64_t* __restrict__ key_s,
                                                            const uint64_t* __restrict__ key_b, uint32_t nch,
                                                            uint32_t* __restrict__ next_s,
                                                            uint32_t* __restrict__ rank) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nch) return;
    const uint32_t c = ord[i];
    const uint64_t g = key_b[c], sc = key_s[c];
    uint64_t nx = ~0ull;
    bool tie = false;
    if (i + 1 < nch) {
        const uint32_t d = ord[i + 1];
        if (key_b[d] == g) nx = key_s[d];
        tie = nx == sc;
    }
    if (i > 0) {
        const uint32_t d = ord[i - 1];
        if (key_b[d] == g && key_s[d] == sc) { nx = sc; tie = true; }
    }
    next_s[c] = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
    rank[c] = i | (tie ? 0x80000000u : 0u);
}

// Per-probe decision flags (bits 31 / 30 of summ.w):
//   first: the earliest probe of its chain in the bucket -> AddHashEntry inserts it (no
//          entry can contain it: only its own chain's entries do)
//   susp : another chain of the bucket and mask starts inside [chain start, probe start];
//          only then can lower_bound miss the probe's chain entry (the non-transitive
//          MheCompare case), so only these probes run the exact search.
// Every other probe collides with its chain entry: the vector stays sorted by (block,
// first-genome start) and is partitioned with respect to such a probe.
// summ_b[q] = {chain entry's first-genome start, its length, its rank | tie}: the slot
// an insert of this probe's chain writes, and its order among the bucket's chains.
// per chain {entry's first-genome start, its length, its rank, next_s}: one 16-B record
// the probe pass gathers (instead of the G + 2 int64 pool entry per probe)
__global__ __launch_bounds__(kBlock) void chain_sb_kernel(const int64_t* __restrict__ pool, uint32_t nch, int G,
                                                          const uint32_t* __restrict__ rank,
                                                          const uint32_t* __restrict__ next_s,
                                                          uint4* __restrict__ chain_sb) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= nch) return;
    const int64_t* e = pool + (uint64_t)c * (uint64_t)(G + 2);
    int64_t es = 0;
    for (int g = G - 1; g >= 0; --g) es = e[2 + g] != 0 ? e[2 + g] : es;
    chain_sb[c] = make_uint4((uint32_t)es, (uint32_t)e[0], rank[c], next_s[c]);
}

// the probe of stream group k (AddHashEntry's argument), built on the rare slow path
template <int MG, typename View>
__device__ __noinline__ void probe_full(const View& v, const GenomeTable& gt, const MatchParams& /*mp*/, int L,
                                        const uint64_t* __restrict__ /*probe_info*/, uint32_t k, Mhe<MG>& P) {
    load_probe<MG>(v, k, gt.G, L, P);
}

// one round: every unconsumed lane of the window runs its lower_bound against the
// current vector (AddHashEntry's lookup, MemHash.cpp:215-218); returns the first lane
// whose probe is not a collision (RB if none).  tb is an LDS or a global slot array.
template <int MG, int RB, typename View>
__device__ __forceinline__ int round_first(const uint4* tb, uint32_t t, uint32_t done, uint32_t c, uint4 me,
                                           uint4 mb, const View& v, const GenomeTable& gt, const MatchParams& mp, int L,
                                           const uint64_t* __restrict__ probe_info,
                                           const int64_t* __restrict__ pool, int* red) {
    const uint32_t tid = threadIdx.x;
    bool isnew = false;
    if (tid >= done && tid < c && (me.w & 0x80000000u)) {
        isnew = true;
    } else if (tid >= done && tid < c && (me.w & 0x40000000u)) {
        const int G = gt.G;
        const uint32_t pmask = me.x, pcid = me.z;
        const int64_t ps = (int64_t)me.y, pl = L;
        Mhe<MG> P;
        bool have = false;
        auto full = [&](uint32_t xid) -> bool {
            if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
            Mhe<MG> E;
            load_entry<MG>(pool, xid, G, E);
            return mhe_less(E, P);
        };
        const uint32_t lb = lower_bound_slots(tb, t, pmask, ps, pl, pcid, full);
        if (lb < t) {
            const uint4 X = tb[lb];
            int q = slot_equiv(X, pmask, ps, pl, pcid);
            if (q == 2) {
                if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
                Mhe<MG> E;
                load_entry<MG>(pool, X.x, G, E);
                q = (mhe_less(E, P) || mhe_less(P, E)) ? 0 : 1;
            }
            isnew = q == 0;
        } else {
            isnew = true;
        }
    }
    return block_first_true<RB>(isnew, red);
}

// insert position of chain entry cid (lower_bound of the extended copy, MemHash.cpp:247);
// the entries are read only for the rare undecided slots
template <int MG>
__device__ __forceinline__ uint32_t insert_pos(const uint4* tb, uint32_t t, uint32_t cid, uint32_t em, int64_t es,
                                              int64_t el, const int64_t* __restrict__ pool, int G) {
    Mhe<MG> E;
    bool have = false;
    auto full = [&](uint32_t xid) -> bool {
        if (!have) { load_entry<MG>(pool, cid, G, E); have = true; }
        Mhe<MG> X;
        load_entry<MG>(pool, xid, G, X);
        return mhe_less(X, E);
    };
    return lower_bound_slots(tb, t, em, es, el, cid, full);
}

// vector insert at ins (MemHash.cpp:247): shift tb[ins, t) up by one.  Each lane owns
// a contiguous run [ra, re); it reads the run's first slot before the barrier and
// moves the run top-down after it (the slot it overwrites was read by its owner).
template <int RB>
__device__ __forceinline__ void shift_insert(uint4* tb, uint32_t t, uint32_t ins, uint4 nv) {
    const uint32_t tid = threadIdx.x;
    const uint32_t n = t - ins;
    const uint32_t per = (n + RB - 1) / RB;
    const uint32_t ra = ins + min(n, tid * per), re = ins + min(n, (tid + 1) * per);
    const uint4 head = ra < re ? tb[ra] : make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (ra < re) {
        for (uint32_t k = re - 1; k > ra; --k) tb[k + 1] = tb[k];
        tb[ra + 1] = head;
    }
    if (tid == 0) tb[ins] = nv;
    __syncthreads();
}

template <int MG>
constexpr int replay_block() { return MG <= 4 ? 1024 : (MG <= 8 ? 512 : 256); }

// RB lanes per bucket; the kernel takes the buckets with kmin < probes <= kmax (small
// buckets run as single waves: their rounds cost no workgroup barriers).
template <int MG, int RB, typename View>
__global__ __launch_bounds__(RB) void replay_kernel(
    View v, GenomeTable gt, MatchParams mp, int L, const uint64_t* __restrict__ probe_info,
    const uint4* __restrict__ summ, const uint4* __restrict__ summ_b, const uint32_t* __restrict__ bstart,
    const uint32_t* __restrict__ bend, const uint32_t* __restrict__ obase,
    uint32_t* __restrict__ tbl, uint4* __restrict__ spill, const int64_t* __restrict__ pool, uint32_t lds_cap,
    uint32_t* __restrict__ tsize, DevCounters* ctr, uint64_t* __restrict__ dbg, uint32_t kmin, uint32_t kmax,
    uint64_t* __restrict__ mlog) {
    extern __shared__ uint4 s_tab[];
    __shared__ int red[RB / 64];
    __shared__ uint32_t s_ins, s_rank;
    __shared__ uint4 s_new;
    uint64_t c_win = 0, c_round = 0, c_ins = 0, n_win = 0, n_round = 0, t0 = 0;
    const uint64_t t_all = dbg ? wall_clock64() : 0;

    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t beg = bstart[b];       // this bucket's probes in the (compacted) summaries
    const uint32_t K_b = bend[b] - beg;
    if (K_b <= kmin || K_b > kmax) return;
    const uint32_t ob = obase[b];         // its slice of tbl / spill (>= the entries it ends with)
    const int G = gt.G;
    bool in_lds = true;
    uint32_t t = 0;
    unsigned long long coll = 0;

    // Fast path: every (compacted) probe is its chain's first, none is suspicious and no
    // two chains tie on their first-genome start.  Then every probe inserts, every
    // lower_bound lands on the sorted position, and the vector ends as the bucket's chains
    // in (block, first-genome start) order = their rank order (chain_next_kernel).
    {
        __shared__ uint32_t s_ok, s_rmin, s_rmax;
        if (tid == 0) { s_ok = 1u; s_rmin = 0xFFFFFFFFu; s_rmax = 0u; }
        __syncthreads();
        uint32_t ok = 1u, rmin = 0xFFFFFFFFu, rmax = 0u;
        for (uint32_t k = tid; k < K_b; k += RB) {
            const uint4 a = summ[beg + k], c = summ_b[beg + k];
            ok &= ((a.w & 0xC0000000u) == 0x80000000u && !(c.z & 0x80000000u)) ? 1u : 0u;
            rmin = min(rmin, c.z & 0x7FFFFFFFu);
            rmax = max(rmax, c.z & 0x7FFFFFFFu);
        }
        if (!ok) atomicAnd(&s_ok, 0u);
        atomicMin(&s_rmin, rmin);
        atomicMax(&s_rmax, rmax);
        __syncthreads();
        if (s_ok && s_rmax - s_rmin + 1u == K_b) {
            const uint32_t r0 = s_rmin;
            for (uint32_t k = tid; k < K_b; k += RB) {
                tbl[ob + ((summ_b[beg + k].z & 0x7FFFFFFFu) - r0)] = summ[beg + k].z;
                log_insert(mlog, ctr, summ_b[beg + k].w, summ[beg + k].z);
            }
            if (tid == 0) {
                tsize[b] = K_b;
                atomicAdd(&ctr->entries, (unsigned long long)K_b);
            }
            return;
        }
    }

    // the window of probes [w0, w0 + c) stays in the lanes' registers until every
    // one of them is consumed (collided or inserted); `done` = consumed prefix
    // A chain-first lane keeps the insert position of its chain entry up to date: an
    // insert at ins moves it up iff ins < pos, or ins == pos and the inserted chain
    // precedes it (rank); chains tied on their first-genome start re-search instead.
    uint4 nxt = (uint32_t)tid < K_b ? summ[beg + tid] : make_uint4(0, 0, 0, 0);
    uint4 nxt_b = (uint32_t)tid < K_b ? summ_b[beg + tid] : make_uint4(0, 0, 0, 0);
    for (uint32_t w0 = 0; w0 < K_b; w0 += RB) {
        const uint32_t c = min((uint32_t)RB, K_b - w0);
        if (dbg) { t0 = wall_clock64(); ++n_win; }
        const uint4 me = nxt, mb = nxt_b;
        if (w0 + RB + tid < K_b) {   // prefetch the next window
            nxt = summ[beg + w0 + RB + tid];
            nxt_b = summ_b[beg + w0 + RB + tid];
        }
        const bool is_first = (uint32_t)tid < c && (me.w & 0x80000000u) && !(mb.z & 0x80000000u);
        uint32_t mypos = 0;
        if (is_first)
            mypos = in_lds ? insert_pos<MG>(s_tab, t, me.z, me.x, (int64_t)mb.x, (int64_t)mb.y, pool, G)
                           : insert_pos<MG>(spill + ob, t, me.z, me.x, (int64_t)mb.x, (int64_t)mb.y, pool, G);
        if (dbg) { __syncthreads(); c_win += wall_clock64() - t0; }
        uint32_t done = 0;
        while (done < c) {
            if (dbg) { t0 = wall_clock64(); ++n_round; }
            const int first = in_lds
                ? round_first<MG, RB, View>(s_tab, t, done, c, me, mb, v, gt, mp, L, probe_info, pool, red)
                : round_first<MG, RB, View>(spill + ob, t, done, c, me, mb, v, gt, mp, L, probe_info, pool, red);
            if (dbg) { const uint64_t t1 = wall_clock64(); c_round += t1 - t0; t0 = t1; }
            if (first == RB) {
                coll += c - done;
                break;
            }
            coll += (unsigned long long)(first - (int)done);
            if (tid == first) {
                if (is_first)
                    s_ins = mypos;
                else
                    s_ins = in_lds ? insert_pos<MG>(s_tab, t, me.z, me.x, (int64_t)mb.x, (int64_t)mb.y, pool, G)
                                   : insert_pos<MG>(spill + ob, t, me.z, me.x, (int64_t)mb.x, (int64_t)mb.y, pool, G);
                s_rank = mb.z & 0x7FFFFFFFu;
                s_new = make_uint4(me.z, me.x, mb.x, mb.y);
                log_insert(mlog, ctr, mb.w, me.z);
            }
            if (in_lds && t + 1 > lds_cap) {   // spill the vector to the bucket's global slice
                for (uint32_t k = tid; k < t; k += RB) spill[ob + k] = s_tab[k];
                in_lds = false;
            }
            __syncthreads();
            if (in_lds) shift_insert<RB>(s_tab, t, s_ins, s_new);
            else shift_insert<RB>(spill + ob, t, s_ins, s_new);
            if (is_first && tid > first)
                mypos += (s_ins < mypos || (s_ins == mypos && s_rank < (mb.z & 0x7FFFFFFFu))) ? 1u : 0u;
            if (dbg) c_ins += wall_clock64() - t0;
            t += 1;
            done = (uint32_t)first + 1;
        }
    }
    if (in_lds)
        for (uint32_t k = tid; k < t; k += RB) tbl[ob + k] = s_tab[k].x;
    else
        for (uint32_t k = tid; k < t; k += RB) tbl[ob + k] = spill[ob + k].x;
    if (tid == 0) {
        tsize[b] = t;
        atomicAdd(&ctr->collisions, coll);
        atomicAdd(&ctr->entries, (unsigned long long)t);
        if (dbg) {
            uint64_t* d = dbg + (uint64_t)b * 8;
            d[0] = K_b; d[1] = t; d[2] = n_win; d[3] = n_round;
            d[4] = c_win; d[5] = c_round; d[6] = c_ins; d[7] = wall_clock64() - t_all;
        }
    }
}

// Big buckets with few exact-search probes (the main diagonal of related genomes: 10^6
// chain-first inserts and a handful of suspicious probes).  The vector is always sorted by
// chain rank, duplicates adjacent, so it is held as a copy count per rank
// of the bucket, cnt[r]: a run of chain-first probes only sets its ranks' counts, and
// before each suspicious probe an exclusive scan E of the counts gives the virtual vector
// V[i] = slot of the rank r with E[r] <= i < E[r + 1], on which that probe runs the exact
// libstdc++ lower_bound of AddHashEntry (MemHash.cpp:215-247).  An insert must land
// between its rank's neighbours (else the bucket is flagged: DevCounters.err bit 2).
// Buckets with tied chains or more than kBigSlow suspicious probes stay on replay_kernel;
// handled buckets get cend = cbeg so that replay_kernel skips them.
constexpr uint32_t kBigBucket = 4096;   // compacted probes above which a bucket may come here
                                        // (MUMS_DEV_BIG_BUCKET overrides it: tests)
constexpr int kBigSlow = 2048;          // suspicious probes per bucket (LDS list)
constexpr int kBigRB = 1024;

__device__ __forceinline__ uint32_t blk_scan_excl(uint32_t v, uint32_t* red, uint32_t* total) {
    // exclusive block scan over kBigRB lanes (wave scans + wave totals in LDS)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) red[wv] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int w = 0; w < kBigRB / 64; ++w) {
        const uint32_t r = red[w];
        base += w < wv ? r : 0u;
        tot += r;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// E[0..R] = exclusive scan of cnt[0..R); returns E[R].  Tiles of kBigIPT * kBigRB counts
// are loaded coalesced into LDS (tile), scanned as kBigIPT consecutive counts per lane and
// written back coalesced.
constexpr int kBigIPT = 8;
__device__ uint32_t scan_counts(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ E, uint32_t R, uint32_t* red,
                                uint32_t* tile) {
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t T = kBigIPT * kBigRB;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < R; base += T) {
        #pragma unroll
        for (int k = 0; k < kBigIPT; ++k) {
            const uint32_t i = base + k * kBigRB + tid;
            tile[k * kBigRB + tid] = i < R ? cnt[i] : 0u;
        }
        __syncthreads();
        uint32_t v[kBigIPT], sum = 0;
        #pragma unroll
        for (int k = 0; k < kBigIPT; ++k) {
            v[k] = tile[tid * kBigIPT + k];
            sum += v[k];
        }
        uint32_t tot;
        uint32_t run = carry + blk_scan_excl(sum, red, &tot);   // barriers inside: tile reads are done
        #pragma unroll
        for (int k = 0; k < kBigIPT; ++k) {
            tile[tid * kBigIPT + k] = run;
            run += v[k];
        }
        __syncthreads();
        #pragma unroll
        for (int k = 0; k < kBigIPT; ++k) {
            const uint32_t i = base + k * kBigRB + tid;
            if (i < R) E[i] = tile[k * kBigRB + tid];
        }
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) E[R] = carry;
    __syncthreads();
    return carry;
}

template <int MG, typename View>
__global__ __launch_bounds__(kBigRB) void replay_big_kernel(
    View v, GenomeTable gt, MatchParams mp, int L, const uint64_t* __restrict__ probe_info,
    const uint4* __restrict__ summ, const uint4* __restrict__ summ_b, const uint32_t* __restrict__ cbeg,
    uint32_t* __restrict__ cend, const uint32_t* __restrict__ obase, uint32_t* __restrict__ tbl,
    const int64_t* __restrict__ pool, const uint4* __restrict__ chain_sb, uint32_t* __restrict__ scr_cnt,
    uint32_t* __restrict__ scr_e, uint4* __restrict__ scr_slot, uint32_t* __restrict__ tsize, DevCounters* ctr, uint32_t big_min,
    uint64_t* __restrict__ mlog) {
    __shared__ uint32_t slow[kBigSlow], slow_sorted[kBigSlow];
    __shared__ uint32_t red[kBigRB / 64];
    __shared__ uint32_t s_ns, s_bad, s_rmin, s_rmax;
    __shared__ uint32_t tile[kBigIPT * kBigRB];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t beg = cbeg[b], K = cend[b] - beg;
    if (K <= big_min) return;
    if (tid == 0) { s_ns = 0; s_bad = 0; s_rmin = 0xFFFFFFFFu; s_rmax = 0; }
    __syncthreads();
    uint32_t rmin = 0xFFFFFFFFu, rmax = 0;
    for (uint32_t k = tid; k < K; k += kBigRB) {
        const uint4 a = summ[beg + k], c = summ_b[beg + k];
        if (c.z & 0x80000000u) s_bad = 1;                     // tied chains: exact order unknown
        if (a.w & 0x80000000u) {
            rmin = min(rmin, c.z);
            rmax = max(rmax, c.z);
        } else {
            const uint32_t q = atomicAdd(&s_ns, 1u);
            if (q < (uint32_t)kBigSlow) slow[q] = k;
        }
    }
    atomicMin(&s_rmin, rmin);
    atomicMax(&s_rmax, rmax);
    __syncthreads();
    const uint32_t S = s_ns;
    if (s_bad || S > (uint32_t)kBigSlow || s_rmin > s_rmax) return;
    const uint32_t r0 = s_rmin, R = s_rmax - s_rmin + 1;
    for (uint32_t i = tid; i < S; i += kBigRB) {   // ascending probe order
        const uint32_t x = slow[i];
        uint32_t rk = 0;
        for (uint32_t j = 0; j < S; ++j) rk += slow[j] < x ? 1u : 0u;
        slow_sorted[rk] = x;
    }
    uint32_t* cnt = scr_cnt + beg;
    uint32_t* E = scr_e + beg + b;   // R + 1 entries per bucket
    uint4* sbr = scr_slot + beg;
    for (uint32_t r = tid; r < R; r += kBigRB) cnt[r] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < K; k += kBigRB) {      // slot of every chain, by rank
        const uint4 a = summ[beg + k];
        if (a.w & 0x80000000u) {
            const uint4 c = summ_b[beg + k];
            if (c.z - r0 < R) sbr[c.z - r0] = make_uint4(a.z, a.x, c.x, c.y);
        }
    }
    __syncthreads();
    const int G = gt.G;
    unsigned long long coll = 0;
    uint32_t k0 = 0;
    for (uint32_t si = 0; si <= S; ++si) {
        const uint32_t j = si < S ? slow_sorted[si] : K;
        for (uint32_t k = k0 + tid; k < j; k += kBigRB) {   // chain-first run: one copy each
            const uint4 a = summ[beg + k];
            if (a.w & 0x80000000u) {
                cnt[(summ_b[beg + k].z) - r0] = 1u;
                log_insert(mlog, ctr, summ_b[beg + k].w, a.z);
            }
        }
        __syncthreads();
        if (j == K) break;
        const uint32_t t = scan_counts(cnt, E, R, red, tile);
        if (tid == 0) {
            auto at = [&](uint32_t i) -> uint4 {   // V[i]: rank r with E[r] <= i < E[r + 1]
                uint32_t lo = 0, n = R;
                while (n > 0) {
                    const uint32_t h = n >> 1;
                    if (E[lo + h + 1] <= i) { lo += h + 1; n -= h + 1; } else n = h;
                }
                return sbr[lo];
            };
            const uint4 me = summ[beg + j], mb = summ_b[beg + j];
            const uint32_t pmask = me.x, pcid = me.z;
            const int64_t ps = (int64_t)me.y, pl = L;
            Mhe<MG> P;
            bool have = false;
            auto full = [&](uint32_t xid) -> bool {
                if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
                Mhe<MG> X;
                load_entry<MG>(pool, xid, G, X);
                return mhe_less(X, P);
            };
            const uint32_t lb = lower_bound_acc(at, t, pmask, ps, pl, pcid, full);
            bool isnew = true;
            if (lb < t) {
                const uint4 X = at(lb);
                int q = slot_equiv(X, pmask, ps, pl, pcid);
                if (q == 2) {
                    if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
                    Mhe<MG> X2;
                    load_entry<MG>(pool, X.x, G, X2);
                    q = (mhe_less(X2, P) || mhe_less(P, X2)) ? 0 : 1;
                }
                isnew = q == 0;
            }
            if (!isnew) {
                ++coll;
            } else {   // insert the chain entry at lower_bound of its copy (MemHash.cpp:247)
                Mhe<MG> Ec;
                bool hv = false;
                auto fullc = [&](uint32_t xid) -> bool {
                    if (!hv) { load_entry<MG>(pool, pcid, G, Ec); hv = true; }
                    Mhe<MG> X;
                    load_entry<MG>(pool, xid, G, X);
                    return mhe_less(X, Ec);
                };
                const uint32_t ins = lower_bound_acc(at, t, pmask, (int64_t)mb.x, (int64_t)mb.y, pcid, fullc);
                const uint32_t rr = mb.z - r0;
                const uint32_t rl = ins > 0 ? chain_sb[at(ins - 1).x].z - r0 : 0u;
                const uint32_t rh = ins < t ? chain_sb[at(ins).x].z - r0 : 0xFFFFFFFFu;
                if (rr < R && rl <= rr && rr <= rh) {
                    cnt[rr] += 1u;
                    log_insert(mlog, ctr, mb.w, pcid);
                } else {
                    s_bad = 2;
                }
            }
        }
        __syncthreads();
        if (s_bad) break;
        k0 = j + 1;
    }
    if (s_bad) {
        if (tid == 0) atomicOr(&ctr->err, 4u);
        return;
    }
    const uint32_t t = scan_counts(cnt, E, R, red, tile);
    const uint32_t ob = obase[b];
    for (uint32_t r = tid; r < R; r += kBigRB) {
        const uint32_t e0 = E[r], c = E[r + 1] - e0;
        const uint32_t id = c ? sbr[r].x : 0u;
        for (uint32_t d = 0; d < c; ++d) tbl[ob + e0 + d] = id;
    }
    if (tid == 0) {
        tsize[b] = t;
        atomicAdd(&ctr->collisions, coll);
        atomicAdd(&ctr->entries, (unsigned long long)t);
        cend[b] = beg;   // replay_kernel skips it
    }
}

// Grid path of the big-bucket replay (host-driven, one bucket at a time): the same rank
// counts as replay_big_kernel, but every pass over the bucket's probes or ranks is a grid
// launch, the counts' scan is the device-wide scan, and only the exact lower_bound of each
// suspicious probe runs on one lane.  For buckets with few suspicious probes (<= kGridSlow).
constexpr uint32_t kGridSlow = 512;

// info: [0] min rank, [1] max rank, [2] tied, [3] suspicious count, [4] error, [5] collisions
__global__ __launch_bounds__(kBlock) void bigg_classify_kernel(const uint4* __restrict__ summ,
                                                               const uint4* __restrict__ summ_b, uint32_t beg,
                                                               uint32_t K, uint32_t* __restrict__ info,
                                                               uint32_t* __restrict__ slow, uint32_t cap) {
    __shared__ uint32_t s_min[kBlock / 64], s_max[kBlock / 64], s_tie;
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_tie = 0;
    uint32_t rmin = 0xFFFFFFFFu, rmax = 0;
    if (k < K) {
        const uint4 a = summ[beg + k], c = summ_b[beg + k];
        if (c.z & 0x80000000u) s_tie = 1;
        if (a.w & 0x80000000u) {
            rmin = c.z;
            rmax = c.z;
        } else {
            const uint32_t q = atomicAdd(&info[3], 1u);
            if (q < cap) slow[q] = k;
        }
    }
    #pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        rmin = min(rmin, (uint32_t)__shfl_xor((int)rmin, d));
        rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, d));
    }
    if (lane == 0) { s_min[wv] = rmin; s_max[wv] = rmax; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) { rmin = min(rmin, s_min[w]); rmax = max(rmax, s_max[w]); }
        rmin = min(rmin, s_min[0]);
        rmax = max(rmax, s_max[0]);
        if (rmin != 0xFFFFFFFFu) atomicMin(&info[0], rmin);
        atomicMax(&info[1], rmax);
        if (s_tie) atomicOr(&info[2], 1u);
    }
}

__global__ __launch_bounds__(kBlock) void bigg_slots_kernel(const uint4* __restrict__ summ,
                                                            const uint4* __restrict__ summ_b, uint32_t beg, uint32_t K,
                                                            uint32_t r0, uint32_t R, uint4* __restrict__ sbr) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= K) return;
    const uint4 a = summ[beg + k];
    if (a.w & 0x80000000u) {
        const uint4 c = summ_b[beg + k];
        if (c.z - r0 < R) sbr[c.z - r0] = make_uint4(a.z, a.x, c.x, c.y);
    }
}

// chain-first probes [k0, k1) of the bucket: one copy of their chain each
__global__ __launch_bounds__(kBlock) void bigg_fill_kernel(const uint4* __restrict__ summ,
                                                           const uint4* __restrict__ summ_b, uint32_t beg, uint32_t k0,
                                                           uint32_t k1, uint32_t r0, uint32_t* __restrict__ cnt,
                                                           uint64_t* __restrict__ mlog, DevCounters* ctr) {
    const uint32_t k = k0 + blockIdx.x * kBlock + threadIdx.x;
    if (k >= k1) return;
    const uint4 a = summ[beg + k];
    if (a.w & 0x80000000u) {
        cnt[summ_b[beg + k].z - r0] = 1u;
        log_insert(mlog, ctr, summ_b[beg + k].w, a.z);
    }
}

// suspicious probe j against the virtual vector V[i] = sbr[r], E[r] <= i < E[r + 1]
template <int MG, typename View>
__global__ void bigg_slow_kernel(View v, GenomeTable gt, MatchParams mp, int L, const uint64_t* __restrict__ probe_info,
                                 const uint4* __restrict__ summ, const uint4* __restrict__ summ_b, uint32_t beg,
                                 uint32_t j, uint32_t r0, uint32_t R, const uint32_t* __restrict__ E,
                                 const uint4* __restrict__ sbr, const uint4* __restrict__ chain_sb,
                                 const int64_t* __restrict__ pool, uint32_t* __restrict__ cnt,
                                 uint32_t* __restrict__ info, uint64_t* __restrict__ mlog, DevCounters* ctr) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const int G = gt.G;
    const uint32_t t = E[R];
    auto at = [&](uint32_t i) -> uint4 {
        uint32_t lo = 0, n = R;
        while (n > 0) {
            const uint32_t h = n >> 1;
            if (E[lo + h + 1] <= i) { lo += h + 1; n -= h + 1; } else n = h;
        }
        return sbr[lo];
    };
    const uint4 me = summ[beg + j], mb = summ_b[beg + j];
    const uint32_t pmask = me.x, pcid = me.z;
    const int64_t ps = (int64_t)me.y, pl = L;
    Mhe<MG> P;
    bool have = false;
    auto full = [&](uint32_t xid) -> bool {
        if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
        Mhe<MG> X;
        load_entry<MG>(pool, xid, G, X);
        return mhe_less(X, P);
    };
    const uint32_t lb = lower_bound_acc(at, t, pmask, ps, pl, pcid, full);
    bool isnew = true;
    if (lb < t) {
        const uint4 X = at(lb);
        int q = slot_equiv(X, pmask, ps, pl, pcid);
        if (q == 2) {
            if (!have) { probe_full<MG, View>(v, gt, mp, L, probe_info, mb.w, P); have = true; }
            Mhe<MG> X2;
            load_entry<MG>(pool, X.x, G, X2);
            q = (mhe_less(X2, P) || mhe_less(P, X2)) ? 0 : 1;
        }
        isnew = q == 0;
    }
    if (!isnew) {
        info[5] += 1u;
        return;
    }
    Mhe<MG> Ec;
    bool hv = false;
    auto fullc = [&](uint32_t xid) -> bool {
        if (!hv) { load_entry<MG>(pool, pcid, G, Ec); hv = true; }
        Mhe<MG> X;
        load_entry<MG>(pool, xid, G, X);
        return mhe_less(X, Ec);
    };
    const uint32_t ins = lower_bound_acc(at, t, pmask, (int64_t)mb.x, (int64_t)mb.y, pcid, fullc);
    const uint32_t rr = mb.z - r0;
    const uint32_t rl = ins > 0 ? chain_sb[at(ins - 1).x].z - r0 : 0u;
    const uint32_t rh = ins < t ? chain_sb[at(ins).x].z - r0 : 0xFFFFFFFFu;
    if (rr < R && rl <= rr && rr <= rh) {
        cnt[rr] += 1u;
        log_insert(mlog, ctr, mb.w, pcid);
        info[6] = 1u;   // inserted (the closed-form path counts it as a duplicate)
    } else {
        info[4] = 1u;
    }
}

__global__ __launch_bounds__(kBlock) void bigg_out_kernel(const uint32_t* __restrict__ E, uint32_t R,
                                                          const uint4* __restrict__ sbr,
                                                          const uint32_t* __restrict__ obase, uint32_t b,
                                                          uint32_t* __restrict__ tbl) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= R) return;
    const uint32_t ob = obase[b];
    const uint32_t e0 = E[r], c = E[r + 1] - e0;
    for (uint32_t d = 0; d < c; ++d) tbl[ob + e0 + d] = sbr[r].x;
}

__global__ void bigg_finish_kernel(const uint32_t* __restrict__ E, uint32_t R, const uint32_t* __restrict__ info,
                                   uint32_t b, uint32_t* __restrict__ tsize, uint32_t* __restrict__ cend, uint32_t beg,
                                   DevCounters* ctr) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const uint32_t t = E[R];
    tsize[b] = t;
    atomicAdd(&ctr->entries, (unsigned long long)t);
    atomicAdd(&ctr->collisions, (unsigned long long)info[5]);
    if (info[4]) atomicOr(&ctr->err, 4u);
    cend[b] = beg;   // replay_kernel / replay_big_kernel skip it
}

// ---- closed-form path for big buckets with many suspicious probes -----------------------
// BASELINE config 5's main diagonal: 4.2e4 chain-first inserts and 1.9e6 suspicious probes in
// one bucket.  Between two inserts every suspicious probe V (of chain A, rank a) meets a vector
// whose MheCompare pattern is fixed by counts alone: entries of ranks < a are less than V
// (earlier block, or same block and start < A's), A's copies are equivalent (A contains V),
// ranks in (a, x] (same block, start in (A.start, V.start)) are less (no other chain contains
// V: containment needs the same line, MatchHashEntry.cpp:164-200, and chains of one line are
// disjoint), ranks after x are not less.  So with pA / dA / nC inserted entries of those three
// groups and t in all, lower_bound (MemHash.cpp:215) is the libstdc++ recurrence over
//   T^pA F^dA T^nC F^(t - pA - dA - nC)
// and V collides iff it lands on A's copies; else a copy of A goes in front of A's copies
// (its own lower_bound: T^pA then F).  Ranks with start == V.start (other genomes decide the
// order) make a probe "exact": it runs the rank-count path (bigg_slow_kernel) at its time.
// The counts come from the chain-first insert times (prefix tables over the firsts in time
// order) plus the duplicate inserts found so far; rounds find the earliest probe that is
// not a collision, apply it, and go on from there.
constexpr uint32_t kQW = 11;   // words per query record

// ff[k] = chain-first flag of bucket probe k (ff[K] = 0); ft[rank] = its time; logs the inserts
__global__ __launch_bounds__(kBlock) void bigq_first_kernel(const uint4* __restrict__ summ,
                                                            const uint4* __restrict__ summ_b, uint32_t beg, uint32_t K,
                                                            uint32_t r0, uint32_t* __restrict__ ff,
                                                            uint32_t* __restrict__ sf, uint32_t* __restrict__ ft,
                                                            uint64_t* __restrict__ mlog, DevCounters* ctr) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k > K) return;
    if (k == K) { ff[K] = 0; sf[K] = 0; return; }
    const uint4 a = summ[beg + k];
    const bool first = (a.w & 0x80000000u) != 0u;
    ff[k] = first ? 1u : 0u;
    sf[k] = first ? 0u : 1u;
    if (first) {
        const uint4 c = summ_b[beg + k];
        ft[(c.z & 0x7FFFFFFFu) - r0] = k;
        log_insert(mlog, ctr, c.w, a.z);
    }
}

// after the scans: fr[i] = rank of the i-th chain-first probe (time order), fi[rank] = i
__global__ __launch_bounds__(kBlock) void bigq_fr_kernel(const uint4* __restrict__ summ, const uint4* __restrict__ summ_b,
                                                         uint32_t beg, uint32_t K, uint32_t r0,
                                                         const uint32_t* __restrict__ fpos, uint32_t* __restrict__ fr,
                                                         uint32_t* __restrict__ fi) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= K || !(summ[beg + k].w & 0x80000000u)) return;
    const uint32_t r = (summ_b[beg + k].z & 0x7FFFFFFFu) - r0, i = fpos[k];
    fr[i] = r;
    fi[r] = i;
}

// PT[blk][r] = chain-first probes among the first blk * bs (time order) with rank < r: one
// workgroup per row, exclusive scan of the indicator over r with a carry
__global__ __launch_bounds__(kBigRB) void bigq_table_kernel(const uint32_t* __restrict__ fi, uint32_t R, uint32_t bs,
                                                            uint32_t* __restrict__ PT) {
    __shared__ uint32_t red[kBigRB / 64];
    const uint32_t blk = blockIdx.x, lim = blk * bs;
    uint32_t* row = PT + (uint64_t)blk * (R + 1);
    uint32_t carry = 0;
    for (uint32_t base = 0; base < R; base += kBigRB) {
        const uint32_t r = base + threadIdx.x;
        const uint32_t v = (r < R && fi[r] < lim) ? 1u : 0u;
        uint32_t tot;
        const uint32_t ex = blk_scan_excl(v, red, &tot);
        if (r < R) row[r] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) row[R] = carry;
}

// first rank r in [0, R) with (block key, start) of sbr[r] >= (m, s)
__device__ __forceinline__ uint32_t rank_lb(const uint4* __restrict__ sbr, uint32_t R, uint32_t m, uint64_t s) {
    uint32_t lo = 0, n = R;
    while (n > 0) {
        const uint32_t h = n >> 1;
        const uint4 X = sbr[lo + h];
        const bool less = X.y < m || (X.y == m && (uint64_t)X.z < s);
        if (less) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo;
}

// one query per suspicious probe, in time order (spos = exclusive scan of the flags):
// Q[q] = {time, a, x, xe, pA, dA, nC, eq, t, status, duplicates applied}
__global__ __launch_bounds__(kBlock) void bigq_query_kernel(const uint4* __restrict__ summ,
                                                            const uint4* __restrict__ summ_b, uint32_t beg, uint32_t K,
                                                            uint32_t r0, uint32_t R, const uint4* __restrict__ sbr,
                                                            const uint32_t* __restrict__ fpos,
                                                            const uint32_t* __restrict__ spos,
                                                            const uint32_t* __restrict__ fr,
                                                            const uint32_t* __restrict__ PT, uint32_t bs,
                                                            uint32_t* __restrict__ Q) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= K) return;
    const uint4 me = summ[beg + k];
    if (me.w & 0x80000000u) return;
    const uint4 mb = summ_b[beg + k];
    const uint32_t a = (mb.z & 0x7FFFFFFFu) - r0;
    const uint32_t x = rank_lb(sbr, R, me.x, (uint64_t)me.y) - 1u;          // start < V.start
    const uint32_t xe = rank_lb(sbr, R, me.x, (uint64_t)me.y + 1u) - 1u;    // start <= V.start
    const uint32_t kq = fpos[k];   // chain-first inserts before V
    const uint32_t blk = kq / bs;
    const uint32_t* row = PT + (uint64_t)blk * (R + 1);
    uint32_t c_a = row[a], c_a1 = row[a + 1], c_x1 = row[x + 1], c_xe1 = row[xe + 1];
    for (uint32_t i = blk * bs; i < kq; ++i) {
        const uint32_t r = fr[i];
        c_a += r < a;
        c_a1 += r < a + 1;
        c_x1 += r < x + 1;
        c_xe1 += r < xe + 1;
    }
    uint32_t* q = Q + (uint64_t)spos[k] * kQW;
    q[0] = k;
    q[1] = a;
    q[2] = x;
    q[3] = xe;
    q[4] = c_a;                       // pA
    q[5] = c_a1 - c_a;                // dA (A's first insert precedes V)
    q[6] = c_x1 - c_a1;               // nC
    q[7] = c_xe1 - c_x1;              // eq
    q[8] = kq;                        // t
    q[9] = 0;
    q[10] = 0;
}

// libstdc++ __lower_bound over the pattern T^pA F^dA T^nC F^...
__device__ __forceinline__ uint32_t lb_pattern(uint32_t t, uint32_t pA, uint32_t dA, uint32_t nC) {
    const uint32_t e1 = pA + dA, e2 = e1 + nC;
    uint32_t first = 0, len = t;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = first + half;
        if (mid < pA || (mid >= e1 && mid < e2)) {
            first = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return first;
}

// one round over the window [q0, q1) of the queries: bring each up to date with the
// duplicate inserts so far (all of them precede the window: dups[], their ranks in order),
// classify (0 collision, 1 insert, 2 exact) and find the earliest non-collision
__global__ __launch_bounds__(kBlock) void bigq_round_kernel(uint32_t* __restrict__ Q, uint32_t q0, uint32_t q1,
                                                            const uint32_t* __restrict__ dups, uint32_t nd,
                                                            uint32_t* __restrict__ best) {
    const uint32_t i = q0 + blockIdx.x * kBlock + threadIdx.x;
    if (i >= q1) return;
    uint32_t* q = Q + (uint64_t)i * kQW;
    const uint32_t a = q[1], x = q[2], xe = q[3];
    uint32_t pA = q[4], dA = q[5], nC = q[6], eq = q[7], t = q[8];
    const uint32_t done = q[10];
    if (done < nd) {
        for (uint32_t d = done; d < nd; ++d) {
            const uint32_t da = dups[d];
            pA += da < a;
            dA += da == a;
            nC += (da > a && da <= x);
            eq += (da > x && da <= xe);
        }
        t += nd - done;
        q[4] = pA; q[5] = dA; q[6] = nC; q[7] = eq; q[8] = t; q[10] = nd;
    }
    uint32_t st = 2;
    if (eq == 0) {
        const uint32_t lb = lb_pattern(t, pA, dA, nC);
        st = (lb >= pA && lb < pA + dA) ? 0u : 1u;
    }
    q[9] = st;
    if (st) atomicMin(best, i);
}

// counts of the virtual vector at time tau: chain-first inserts before tau + duplicates
__global__ __launch_bounds__(kBlock) void bigq_cnt_kernel(const uint32_t* __restrict__ ft,
                                                          const uint32_t* __restrict__ dup, uint32_t R, uint32_t tau,
                                                          uint32_t* __restrict__ cnt) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < R) cnt[r] = (ft[r] < tau ? 1u : 0u) + dup[r];
}

// a duplicate insert of rank da (probe at bucket time k): counted, logged unless the exact
// path logged it
__global__ void bigq_dup_kernel(uint32_t* __restrict__ dup, uint32_t* __restrict__ dups, uint32_t nd, uint32_t da,
                                const uint4* __restrict__ summ, const uint4* __restrict__ summ_b, uint32_t beg,
                                uint32_t k, int log, uint64_t* __restrict__ mlog, DevCounters* ctr) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    dup[da] += 1u;
    dups[nd] = da;
    if (log) log_insert(mlog, ctr, summ_b[beg + k].w, summ[beg + k].z);
}

__global__ __launch_bounds__(kBlock) void bigq_final_kernel(const uint32_t* __restrict__ dup, uint32_t R,
                                                            uint32_t* __restrict__ cnt) {
    const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
    if (r < R) cnt[r] = 1u + dup[r];
}

__global__ void bucket_ranges_kernel(const uint32_t* __restrict__ sb, uint64_t P, uint32_t* __restrict__ bstart,
                                     uint32_t* __restrict__ bend, uint32_t* __restrict__ d_max) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P) return;
    const uint32_t b = sb[k];
    if (k == 0 || sb[k - 1] != b) bstart[b] = (uint32_t)k;
    if (k == P - 1 || sb[k + 1] != b) {
        bend[b] = (uint32_t)(k + 1);
        uint64_t lo = k;   // first probe of this bucket: binary search back over sb
        uint64_t a = 0;
        while (a < lo) {
            const uint64_t m = (a + lo) >> 1;
            if (sb[m] < b) a = m + 1; else lo = m;
        }
        atomicMax(d_max, (uint32_t)(k + 1 - a));
    }
}

// MatchList output (GetMatchList, MemHash.h:182-203): output row o belongs to the bucket
// b with obase[b] <= o < obase[b] + tsize[b] (last bucket whose exclusive output base is
// <= o); one row per thread, so a bucket holding most entries (the main diagonal of
// related genomes) is written by the whole grid.
__global__ __launch_bounds__(kBlock) void emit_kernel(const uint32_t* __restrict__ obase,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ tbl,
                                                      const int64_t* __restrict__ pool, int G, uint32_t table_size,
                                                      uint64_t M, uint64_t* __restrict__ out_len,
                                                      int64_t* __restrict__ out_s) {
    const uint64_t o = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (o >= M) return;
    uint32_t lo = 0, n = table_size;   // upper_bound(obase, o) - 1
    while (n > 0) {
        const uint32_t h = n >> 1;
        if ((uint64_t)obase[lo + h] <= o) { lo += h + 1; n -= h + 1; }
        else n = h;
    }
    const uint32_t b = lo - 1;
    const uint32_t id = tbl[bstart[b] + (uint32_t)(o - obase[b])];
    const int64_t* e = pool + (uint64_t)id * (uint64_t)(G + 2);
    out_len[o] = (uint64_t)e[0];
    for (int g = 0; g < G; ++g) out_s[o * (uint64_t)G + g] = e[2 + g];
}

}  // namespace

hipError_t launch_bucket_ranges(const uint32_t* sb, uint64_t P, uint32_t* bstart, uint32_t* bend, uint32_t* d_max,
                                hipStream_t st) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(bucket_ranges_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, sb, P, bstart, bend,
                       d_max);
    return hipGetLastError();
}

// Closed-form replay of one big bucket (probes [beg, beg + K), S suspicious, chain ranks
// r0 .. r0 + R - 1, no tied chains): see bigq_round_kernel.  Scratch is allocated here (the
// path runs for a handful of buckets per FindMatches).
template <int MG, typename View>
hipError_t bigq_bucket(View v, const GenomeTable& gt, const MatchParams& mp, int L, const uint64_t* probe_info,
                       const uint4* summ, const uint4* summ_b, uint32_t beg, uint32_t K, uint32_t S, uint32_t r0,
                       uint32_t R, uint32_t b, uint32_t* cend, const uint32_t* bstart, uint32_t* tbl,
                       const int64_t* pool, const uint4* chain_sb, uint32_t* info, void* stmp, uint32_t* tsize,
                       void* ctr, hipStream_t st, uint64_t* mlog) {
    const uint32_t F = K - S;
    const uint32_t bs = std::max<uint32_t>(256u, (F + 255u) / 256u);
    const uint32_t NB = F / bs + 1;
    const size_t words = 3ull * (K + 1) + 5ull * (R + 1) + (size_t)F + 1 + (size_t)NB * (R + 1) +
                         (size_t)S * (kQW + 1) + 64 + 64 * 8;
    size_t stmp_need = scan_tmp_bytes((uint64_t)std::max(K, R) + 1);
    char* base = nullptr;
    hipError_t e = hipMalloc(&base, words * 4 + 16 * (size_t)(R + 1) + stmp_need + 4096);
    if (e != hipSuccess) return e;
    char* p = base;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    uint32_t* ff = (uint32_t*)carve((K + 1) * 4ull);     // first flags -> fpos
    uint32_t* sf = (uint32_t*)carve((K + 1) * 4ull);     // suspicious flags -> spos
    uint32_t* ft = (uint32_t*)carve((R + 1) * 4ull);     // time of each rank's first insert
    uint32_t* fi = (uint32_t*)carve((R + 1) * 4ull);     // index of each rank's first among the firsts
    uint32_t* dup = (uint32_t*)carve((R + 1) * 4ull);    // duplicate inserts per rank
    uint32_t* dups = (uint32_t*)carve((S + 1) * 4ull);   // their ranks, in insert order
    uint32_t* cnt = (uint32_t*)carve((R + 1) * 4ull);
    uint32_t* E = (uint32_t*)carve((R + 1) * 4ull);
    uint32_t* fr = (uint32_t*)carve((F + 1) * 4ull);
    uint32_t* PT = (uint32_t*)carve((size_t)NB * (R + 1) * 4);
    uint32_t* Q = (uint32_t*)carve((size_t)S * kQW * 4 + 4);
    uint32_t* best = (uint32_t*)carve(64);
    uint4* sbr = (uint4*)carve((R + 1) * 16ull);
    void* tmp = carve(stmp_need);
    (void)stmp;
    auto done = [&](hipError_t x) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(base);
        return x;
    };
    auto grid = [](uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); };
    if ((e = hipMemsetAsync(dup, 0, (R + 1) * 4ull, st)) != hipSuccess) return done(e);
    hipLaunchKernelGGL(bigg_slots_kernel, grid(K), dim3(kBlock), 0, st, summ, summ_b, beg, K, r0, R, sbr);
    hipLaunchKernelGGL(bigq_first_kernel, grid(K + 1), dim3(kBlock), 0, st, summ, summ_b, beg, K, r0, ff, sf, ft, mlog,
                       (DevCounters*)ctr);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    if ((e = exclusive_scan_u32(ff, (uint64_t)K + 1, tmp, nullptr, st)) != hipSuccess) return done(e);
    if ((e = exclusive_scan_u32(sf, (uint64_t)K + 1, tmp, nullptr, st)) != hipSuccess) return done(e);
    hipLaunchKernelGGL(bigq_fr_kernel, grid(K), dim3(kBlock), 0, st, summ, summ_b, beg, K, r0, (const uint32_t*)ff, fr,
                       fi);
    hipLaunchKernelGGL(bigq_table_kernel, dim3(NB), dim3(kBigRB), 0, st, (const uint32_t*)fi, R, bs, PT);
    hipLaunchKernelGGL(bigq_query_kernel, grid(K), dim3(kBlock), 0, st, summ, summ_b, beg, K, r0, R,
                       (const uint4*)sbr, (const uint32_t*)ff, (const uint32_t*)sf, (const uint32_t*)fr,
                       (const uint32_t*)PT, bs, Q);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    // rounds over a window of the queries: it doubles while no event turns up in it
    uint32_t q0 = 0, ndup = 0;
    constexpr uint32_t kWin0 = 32768;
    uint32_t win = kWin0;
    std::vector<uint32_t> hq(kQW);
    const bool stats = getenv("MUMS_DEV_REPLAY_STATS") != nullptr;
    uint32_t nexact = 0, rounds = 0;
    while (q0 < S) {
        const uint32_t inf = 0xFFFFFFFFu;
        const uint32_t q1 = (uint32_t)std::min<uint64_t>(S, (uint64_t)q0 + win);
        if ((e = hipMemcpyAsync(best, &inf, 4, hipMemcpyHostToDevice, st)) != hipSuccess) return done(e);
        hipLaunchKernelGGL(bigq_round_kernel, grid(q1 - q0), dim3(kBlock), 0, st, Q, q0, q1, (const uint32_t*)dups,
                           ndup, best);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        uint32_t m = inf;
        if ((e = hipMemcpyAsync(&m, best, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return done(e);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return done(e);
        ++rounds;
        if (m == inf) {   // every query of the window collides
            q0 = q1;
            win = std::min<uint32_t>(win * 2, 1u << 30);
            continue;
        }
        win = kWin0;
        if ((e = hipMemcpy(hq.data(), Q + (size_t)m * kQW, kQW * 4, hipMemcpyDeviceToHost)) != hipSuccess) return done(e);
        const uint32_t k = hq[0], a = hq[1];
        bool inserted = hq[9] == 1;
        if (hq[9] == 2) {   // exact lower_bound on the rank counts at this probe's time
            ++nexact;
            hipLaunchKernelGGL(bigq_cnt_kernel, grid(R), dim3(kBlock), 0, st, (const uint32_t*)ft,
                               (const uint32_t*)dup, R, k, cnt);
            if ((e = hipMemcpyAsync(E, cnt, (size_t)R * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return done(e);
            if ((e = hipMemsetAsync(E + R, 0, 4, st)) != hipSuccess) return done(e);
            if ((e = exclusive_scan_u32(E, (uint64_t)R + 1, tmp, nullptr, st)) != hipSuccess) return done(e);
            if ((e = hipMemsetAsync(info + 6, 0, 4, st)) != hipSuccess) return done(e);
            hipLaunchKernelGGL((bigg_slow_kernel<MG, View>), dim3(1), dim3(64), 0, st, v, gt, mp, L, probe_info, summ,
                               summ_b, beg, k, r0, R, (const uint32_t*)E, (const uint4*)sbr, chain_sb, pool, cnt, info,
                               mlog, (DevCounters*)ctr);
            uint32_t ins = 0;
            if ((e = hipMemcpyAsync(&ins, info + 6, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return done(e);
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return done(e);
            inserted = ins != 0;
        }
        if (inserted) {
            hipLaunchKernelGGL(bigq_dup_kernel, dim3(1), dim3(64), 0, st, dup, dups, ndup, a, summ, summ_b, beg, k,
                               hq[9] == 1 ? 1 : 0, mlog, (DevCounters*)ctr);
            ++ndup;
        }
        q0 = m + 1;
    }
    if (stats)
        fprintf(stderr, "closed-form bucket %u: K %u suspicious %u ranks %u duplicates %u exact %u rounds %u\n", b, K, S,
                R, ndup, nexact, rounds);
    hipLaunchKernelGGL(bigq_final_kernel, grid(R), dim3(kBlock), 0, st, (const uint32_t*)dup, R, cnt);
    if ((e = hipMemcpyAsync(E, cnt, (size_t)R * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return done(e);
    if ((e = hipMemsetAsync(E + R, 0, 4, st)) != hipSuccess) return done(e);
    if ((e = exclusive_scan_u32(E, (uint64_t)R + 1, tmp, nullptr, st)) != hipSuccess) return done(e);
    const uint32_t coll = S - ndup;   // every other suspicious probe collided
    if ((e = hipMemcpyAsync(info + 5, &coll, 4, hipMemcpyHostToDevice, st)) != hipSuccess) return done(e);
    hipLaunchKernelGGL(bigg_out_kernel, grid(R), dim3(kBlock), 0, st, (const uint32_t*)E, R, (const uint4*)sbr, bstart,
                       b, tbl);
    hipLaunchKernelGGL(bigg_finish_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)E, R, (const uint32_t*)info, b,
                       tsize, cend, beg, (DevCounters*)ctr);
    return done(hipGetLastError());
}

// The replay over the compacted probes (chain-first / suspicious, bucket-major, cbeg /
// cend per bucket): big buckets by rank counts (grid path, then one workgroup), then the
// per-bucket rounds.  scr: scratch of replay_scratch_bytes(scr_n) for scr_n compacted probes.
template <int MG, typename View>
hipError_t replay_tail(View v, const GenomeTable& gt, const MatchParams& mp, int L, const uint64_t* probe_info,
                       const uint4* summ_c, const uint4* summ_bc, uint32_t* cbeg, uint32_t* cend,
                       const uint32_t* bstart, uint32_t* tbl, void* spill, const int64_t* pool,
                       const uint4* chain_sb, uint64_t scr_n, void* scr, void* stmp, uint32_t lds_cap,
                       uint32_t* tsize, void* ctr, uint64_t* dbg, hipStream_t st, uint64_t* mlog) {
    hipError_t e = hipSuccess;
    char* p = (char*)scr;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    // big buckets with few suspicious probes: rank counts (replay_big_kernel), first
    {
        const char* bm_env = getenv("MUMS_DEV_BIG_BUCKET");
        const uint32_t big_min = bm_env ? (uint32_t)atoi(bm_env) : kBigBucket;
        const char* gs_env = getenv("MUMS_DEV_GRID_SLOW");   // tests: force the closed-form path
        const uint32_t grid_slow = gs_env ? (uint32_t)atoi(gs_env) : kGridSlow;
        uint32_t* scr_cnt = (uint32_t*)carve((scr_n + 1) * 4);
        uint32_t* scr_e = (uint32_t*)carve((scr_n + 1 + mp.table_size + 1) * 4);
        uint4* scr_slot = (uint4*)carve((scr_n + 1) * 16);
        uint32_t* ginfo = (uint32_t*)carve(64);
        uint32_t* gslow = (uint32_t*)carve((kGridSlow + 1) * 4);
        // grid path first, for the big buckets with few suspicious probes (host-driven)
        std::vector<uint32_t> hb(mp.table_size), he(mp.table_size);
        if ((e = hipMemcpyAsync(hb.data(), cbeg, mp.table_size * 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(he.data(), cend, mp.table_size * 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        // the LDS vector of the big-bucket kernel: at most the fullest bucket's kept probes (a
        // bucket's vector holds <= its kept probes; a larger one would spill, correctly)
        uint32_t kmax = 0;
        for (uint32_t b = 0; b < mp.table_size; ++b) kmax = std::max(kmax, he[b] - hb[b]);
        lds_cap = std::min(lds_cap, kmax);
        for (uint32_t b = 0; b < mp.table_size; ++b) {
            const uint32_t beg = hb[b], K = he[b] - hb[b];
            if (K <= big_min) continue;
            uint32_t hinfo[8] = {0xFFFFFFFFu, 0, 0, 0, 0, 0, 0, 0};
            if ((e = hipMemcpyAsync(ginfo, hinfo, 32, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
            hipLaunchKernelGGL(bigg_classify_kernel, dim3((K + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                               (const uint4*)summ_c, (const uint4*)summ_bc, beg, K, ginfo, gslow, kGridSlow);
            if ((e = hipMemcpyAsync(hinfo, ginfo, 32, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            const uint32_t S = hinfo[3];
            if (getenv("MUMS_DEV_REPLAY_STATS"))
                fprintf(stderr, "grid path bucket %u: K %u flags %u slow %u ranks %u..%u\n", b, K, hinfo[2], S, hinfo[0],
                        hinfo[1]);
            if (hinfo[2] || hinfo[0] > hinfo[1]) continue;   // tied chains: left to the kernels below
            if (S > grid_slow) {   // many suspicious probes: closed form (bigq_*)
                if ((e = bigq_bucket<MG, View>(v, gt, mp, L, probe_info, summ_c, summ_bc, beg, K, S, hinfo[0],
                                               hinfo[1] - hinfo[0] + 1, b, cend, bstart, tbl, pool, chain_sb, ginfo,
                                               stmp, tsize, ctr, st, mlog)) != hipSuccess)
                    return e;
                continue;
            }
            const uint32_t r0 = hinfo[0], R = hinfo[1] - hinfo[0] + 1;
            std::vector<uint32_t> hs(S);
            if (S) {
                if ((e = hipMemcpy(hs.data(), gslow, S * 4, hipMemcpyDeviceToHost)) != hipSuccess) return e;
                std::sort(hs.begin(), hs.end());
            }
            uint32_t* cnt = scr_cnt;
            uint32_t* E = scr_e;
            uint4* sbr = scr_slot;
            if ((e = hipMemsetAsync(cnt, 0, (size_t)R * 4, st)) != hipSuccess) return e;
            hipLaunchKernelGGL(bigg_slots_kernel, dim3((K + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                               (const uint4*)summ_c, (const uint4*)summ_bc, beg, K, r0, R, sbr);
            auto scan = [&]() -> hipError_t {
                hipError_t x = hipMemcpyAsync(E, cnt, (size_t)R * 4, hipMemcpyDeviceToDevice, st);
                if (x == hipSuccess) x = hipMemsetAsync(E + R, 0, 4, st);
                if (x == hipSuccess) x = exclusive_scan_u32(E, (uint64_t)R + 1, stmp, nullptr, st);
                return x;
            };
            uint32_t k0 = 0;
            for (uint32_t si = 0; si <= S; ++si) {
                const uint32_t j = si < S ? hs[si] : K;
                if (j > k0)
                    hipLaunchKernelGGL(bigg_fill_kernel, dim3((j - k0 + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                                       (const uint4*)summ_c, (const uint4*)summ_bc, beg, k0, j, r0, cnt, mlog,
                                       (DevCounters*)ctr);
                if (j == K) break;
                if ((e = scan()) != hipSuccess) return e;
                hipLaunchKernelGGL((bigg_slow_kernel<MG, View>), dim3(1), dim3(64), 0, st, v, gt, mp, L, probe_info,
                                   (const uint4*)summ_c, (const uint4*)summ_bc, beg, j, r0, R, (const uint32_t*)E,
                                   (const uint4*)sbr, (const uint4*)chain_sb, pool, cnt, ginfo, mlog,
                                   (DevCounters*)ctr);
                k0 = j + 1;
            }
            if ((e = scan()) != hipSuccess) return e;
            hipLaunchKernelGGL(bigg_out_kernel, dim3((R + kBlock - 1) / kBlock), dim3(kBlock), 0, st, (const uint32_t*)E,
                               R, (const uint4*)sbr, bstart, b, tbl);
            hipLaunchKernelGGL(bigg_finish_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)E, R, ginfo, b, tsize,
                               cend, beg, (DevCounters*)ctr);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        hipLaunchKernelGGL((replay_big_kernel<MG, View>), dim3(mp.table_size), dim3(kBigRB), 0, st, v, gt, mp, L,
                           probe_info, (const uint4*)summ_c, (const uint4*)summ_bc, cbeg, cend, bstart, tbl, pool,
                           (const uint4*)chain_sb, scr_cnt, scr_e, scr_slot, tsize, (DevCounters*)ctr, big_min, mlog);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // buckets of <= 64 probes: one wave each; the rest: one big workgroup each
    constexpr uint32_t kSmall = 64;
    hipLaunchKernelGGL((replay_kernel<MG, 64, View>), dim3(mp.table_size), dim3(64), kSmall * sizeof(uint4), st, v, gt,
                       mp, L, probe_info, (const uint4*)summ_c, (const uint4*)summ_bc, cbeg, cend, bstart, tbl,
                       (uint4*)spill, pool, kSmall, tsize, (DevCounters*)ctr, dbg, 0u, kSmall, mlog);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (lds_cap <= kSmall) return hipSuccess;   // lds_cap = min(fullest bucket, LDS slots)
    constexpr int RB = replay_block<MG>();
    const size_t lds = (size_t)lds_cap * sizeof(uint4);
    e = hipFuncSetAttribute((const void*)replay_kernel<MG, RB, View>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((replay_kernel<MG, RB, View>), dim3(mp.table_size), dim3(RB), lds, st, v, gt, mp, L, probe_info,
                       (const uint4*)summ_c, (const uint4*)summ_bc, cbeg, cend, bstart, tbl, (uint4*)spill, pool,
                       lds_cap, tsize, (DevCounters*)ctr, dbg, kSmall, 0xFFFFFFFFu, mlog);
    return hipGetLastError();
}

// G > 32: bkey[c] = dense rank of bitreverse64(mask of chain c) (kA..vB: sort buffers
// of nch, step: nch words, stmp: scan scratch); nullptr for G <= 32
uint32_t* block_keys(const int64_t* pool, uint32_t nch, int G, uint64_t* bm, uint64_t* kA, uint32_t* vA, uint64_t* kB,
                     uint32_t* vB, uint32_t* step, uint32_t* bkey, void* d_radix_tmp, void* stmp, hipStream_t st,
                     hipError_t* err) {
    *err = hipSuccess;
    if (G <= 32 || nch == 0) return nullptr;
    const unsigned cgrid = (nch + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(chain_bmask_kernel, dim3(cgrid), dim3(kBlock), 0, st, pool, nch, G, bm);
    int buf = 0;
    if ((*err = radix_sort<uint64_t>(bm, nullptr, nch, 64, kA, vA, kB, vB, d_radix_tmp, &buf, st)) != hipSuccess)
        return nullptr;
    const uint64_t* sk = buf ? kB : kA;
    const uint32_t* ord = buf ? vB : vA;
    hipLaunchKernelGGL(dense_step_kernel, dim3(cgrid), dim3(kBlock), 0, st, sk, nch, step);
    if ((*err = exclusive_scan_u32(step, nch, stmp, nullptr, st)) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(dense_scatter_kernel, dim3(cgrid), dim3(kBlock), 0, st, ord, (const uint32_t*)step, nch, bkey);
    *err = hipGetLastError();
    return bkey;
}

size_t replay_scratch_bytes(uint64_t n, uint32_t table_size) {
    return (n + 1) * 4 + (n + 2 + (uint64_t)table_size) * 4 + (n + 1) * 16 + 64 + (kGridSlow + 1) * 4 + 5 * 256;
}

// ---- the replay from the probes in key order ------------------------------------------
// Only two kinds of AddHashEntry call can touch a bucket vector: the chain's first probe in
// key order (= in its bucket's order: the bucket partition is stable)
// inserts the chain, and a suspicious probe (another chain of the bucket and block starts in
// [chain start, probe start]) runs the exact search; every other probe collides with its
// chain's entry.  Both tests need only the probe's chain and first-genome start, so one pass
// over the probes in key order keeps those (first: fk[chain] == k, from chains.hip; suspicious:
// start >= next_s of the chain), and the bucket order, the summaries and the replay work on
// the kept probes alone -- no per-probe pass in bucket order.
constexpr int kKeepIPT = 8;
constexpr int kKeepStageW = 17;   // rows of up to 16 genomes are staged through LDS in keep_fill_kernel

__device__ __forceinline__ uint32_t row_first_start(const int64_t* __restrict__ rows, uint64_t k, int G) {
    const int64_t* r = rows + k * (uint64_t)(G + 1);
    for (int g = 0; g < G; ++g) {
        const int64_t x = r[g];
        if (x != 0) return (uint32_t)x;   // forward by SetDirection: the first present genome's start > 0
    }
    return 0u;
}

// per chain, what the keep test reads: {first probe (key order), next_s, hash bucket, 0}
__global__ __launch_bounds__(kBlock) void chain_keep_kernel(const uint32_t* __restrict__ fk,
                                                            const uint32_t* __restrict__ next_s,
                                                            const uint64_t* __restrict__ key_b, uint32_t nch,
                                                            uint4* __restrict__ ck) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c < nch) ck[c] = make_uint4(fk[c], next_s[c], (uint32_t)(key_b[c] >> 32), 0u);
}

// kept probe k (chain-first or suspicious) -> *key = bucket << 32 | k
__device__ __forceinline__ bool keep_probe(const int64_t* __restrict__ rows, uint64_t k, int G,
                                           const uint32_t* __restrict__ chain_of, const uint4* __restrict__ ck,
                                           uint64_t* key) {
    const uint4 c = ck[chain_of[k]];
    const bool first = c.x == (uint32_t)k;
    bool keep = first;
    if (!first) keep = row_first_start(rows, k, G) >= c.y;
    *key = ((uint64_t)c.z << 32) | k;
    return keep;
}

// the kept keys, one pass: per block an offset from one atomic (the order is restored by
// the sort that follows: the key holds the probe index)
__global__ __launch_bounds__(kBlock) void keep_fill_kernel(const int64_t* __restrict__ rows, uint64_t P, int G,
                                                           const uint32_t* __restrict__ chain_of,
                                                           const uint4* __restrict__ ck,
                                                           unsigned int* __restrict__ nkept, uint64_t cap,
                                                           uint64_t* __restrict__ kept,
                                                           const uint32_t* __restrict__ fsk,
                                                           uint32_t* __restrict__ kcid) {
    __shared__ uint32_t s_w[kBlock / 64 + 1];
    __shared__ int64_t srow[kBlock * kKeepStageW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t keys[kKeepIPT];
    uint32_t cids[kKeepIPT];
    uint32_t want = 0;
    const int W = G + 1;
    const bool staged = W <= kKeepStageW;   // uniform
    #pragma unroll
    for (int i = 0; i < kKeepIPT; ++i) {
        const uint64_t k0 = (uint64_t)blockIdx.x * (kBlock * kKeepIPT) + (uint64_t)i * kBlock;
        const uint64_t k = k0 + threadIdx.x;
        keys[i] = 0;
        cids[i] = k < P ? chain_of[k] : 0u;
        if (fsk) {   // first-genome starts in key order (rows stored in line order)
            if (k < P) {
                const uint4 c = ck[cids[i]];
                const bool keep = c.x == (uint32_t)k || fsk[k] >= c.y;
                keys[i] = ((uint64_t)c.z << 32) | k;
                if (keep) want |= 1u << i;
            }
        } else if (staged) {
            // the round's rows are one contiguous range: read it with consecutive lanes on
            // consecutive words (one lane per row touches a 128-B line per lane)
            if (k0 < P) {
                const uint64_t nk = P - k0 < (uint64_t)kBlock ? P - k0 : (uint64_t)kBlock;
                const int64_t* src = rows + k0 * (uint64_t)W;
                for (uint32_t j = threadIdx.x; j < nk * (uint64_t)W; j += kBlock) srow[j] = src[j];
            }
            __syncthreads();
            if (k < P) {
                const uint4 c = ck[cids[i]];
                bool keep = c.x == (uint32_t)k;
                if (!keep) {
                    uint32_t fs = 0;
                    for (int g = 0; g < G && fs == 0; ++g) fs = (uint32_t)srow[threadIdx.x * W + g];
                    keep = fs >= c.y;
                }
                keys[i] = ((uint64_t)c.z << 32) | k;
                if (keep) want |= 1u << i;
            }
            __syncthreads();
        } else if (k < P && keep_probe(rows, k, G, chain_of, ck, &keys[i])) {
            want |= 1u << i;
        }
    }
    const uint32_t n = (uint32_t)__builtin_popcount(want);
    uint32_t x = n;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const uint32_t c = s_w[w];
            s_w[w] = tot;
            tot += c;
        }
        s_w[kBlock / 64] = tot ? atomicAdd(nkept, tot) : 0u;
    }
    __syncthreads();
    uint64_t o = (uint64_t)s_w[kBlock / 64] + s_w[wv] + x - n;
    #pragma unroll
    for (int i = 0; i < kKeepIPT; ++i)
        if ((want >> i) & 1u) {
            if (o < cap) {
                kept[o] = keys[i];
                kcid[o] = cids[i];
            }
            ++o;
        }
}

// the same from the chains' line-order arrays (launch_chains jl): chain, probe and first
// start of line position j, read in line order -- the chain summaries ck[s] are read in chain
// order and no per-probe chain id is gathered
__global__ __launch_bounds__(kBlock) void keep_fill_line_kernel(const uint32_t* __restrict__ jl, uint64_t P,
                                                                const uint4* __restrict__ ck,
                                                                unsigned int* __restrict__ nkept, uint64_t cap,
                                                                uint64_t* __restrict__ kept,
                                                                uint32_t* __restrict__ kcid) {
    __shared__ uint32_t s_w[kBlock / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t keys[kKeepIPT];
    uint32_t cids[kKeepIPT];
    uint32_t want = 0;
    #pragma unroll
    for (int i = 0; i < kKeepIPT; ++i) {
        const uint64_t j = (uint64_t)blockIdx.x * (kBlock * kKeepIPT) + (uint64_t)i * kBlock + threadIdx.x;
        keys[i] = 0;
        cids[i] = 0;
        if (j < P) {
            const uint32_t s = jl[j], k = jl[P + j];
            const uint4 c = ck[s];
            if (c.x == k || jl[2 * P + j] >= c.y) want |= 1u << i;
            keys[i] = ((uint64_t)c.z << 32) | k;
            cids[i] = s;
        }
    }
    const uint32_t n = (uint32_t)__builtin_popcount(want);
    uint32_t x = n;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const uint32_t c = s_w[w];
            s_w[w] = tot;
            tot += c;
        }
        s_w[kBlock / 64] = tot ? atomicAdd(nkept, tot) : 0u;
    }
    __syncthreads();
    uint64_t o = (uint64_t)s_w[kBlock / 64] + s_w[wv] + x - n;
    #pragma unroll
    for (int i = 0; i < kKeepIPT; ++i)
        if ((want >> i) & 1u) {
            if (o < cap) {
                kept[o] = keys[i];
                kcid[o] = cids[i];
            }
            ++o;
        }
}

// summaries of the kept probes in bucket order (sorted keys): {block key, first-genome start,
// chain id, flags (bit 31 chain-first, bit 30 suspicious)}, {chain entry's start, its length,
// its rank | tie, probe index}
template <int MG, typename View>
__global__ __launch_bounds__(kBlock) void kept_summary_kernel(View v, GenomeTable gt, int L,
                                                              const uint64_t* __restrict__ skey, uint32_t Kc,
                                                              const uint32_t* __restrict__ scid,
                                                              const uint32_t* __restrict__ fk,
                                                              const uint4* __restrict__ chain_sb,
                                                              const uint32_t* __restrict__ bkey,
                                                              uint4* __restrict__ summ, uint4* __restrict__ summ_b) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= Kc) return;
    const uint32_t k = (uint32_t)skey[i];
    Mhe<MG> Q;
    load_probe<MG>(v, k, gt.G, L, Q);
    const uint32_t cid = scid[i];
    const uint4 cs = chain_sb[cid];
    const bool first = fk[cid] == k;
    summ[i] = make_uint4(block_key<MG>(Q, gt.G, bkey, cid), (uint32_t)start_at(Q, first_start(Q)), cid,
                         first ? 0x80000000u : 0x40000000u);
    summ_b[i] = make_uint4(cs.x, cs.y, cs.z, k);
}

// bucket ranges of the sorted kept keys (cbeg / cend zeroed before)
__global__ __launch_bounds__(kBlock) void kept_ranges_kernel(const uint64_t* __restrict__ skey, uint32_t Kc,
                                                             uint32_t* __restrict__ cbeg, uint32_t* __restrict__ cend,
                                                             uint64_t P, DevCounters* __restrict__ ctr) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) atomicAdd(&ctr->collisions, (unsigned long long)(P - Kc));   // the dropped probes collide
    if (i >= Kc) return;
    const uint32_t b = (uint32_t)(skey[i] >> 32);
    if (i == 0 || (uint32_t)(skey[i - 1] >> 32) != b) cbeg[b] = i;
    if (i + 1 == Kc || (uint32_t)(skey[i + 1] >> 32) != b) cend[b] = i + 1;
}

// The nch chains of a merged pool in (hash bucket, block, first-genome start) order =
// MheCompare's order inside a bucket: rank[c] and next_s[c] (chain_next_kernel); key_b[c] =
// bucket << 32 | block key.  Buffers of nch entries: key_s, key_b, key_g, kA, kB (8 B), vA, vB,
// step, bkey_buf (4 B; step may alias next_s).  *bkey_out: the dense block keys (G > 32) or null.
static hipError_t chain_order(const int64_t* pool, uint32_t nch, const GenomeTable& gt, const MatchParams& mp,
                              uint64_t* key_s, uint64_t* key_b, uint64_t* key_g, uint64_t* kA, uint64_t* kB,
                              uint32_t* vA, uint32_t* vB, uint32_t* step, uint32_t* bkey_buf, void* d_radix_tmp,
                              void* d_scan_tmp, uint32_t* next_s, uint32_t* rank, const uint32_t** bkey_out,
                              hipStream_t st) {
    const unsigned cgrid = (nch + kBlock - 1) / kBlock;
    hipError_t e = hipSuccess;
    const uint32_t* bkey = block_keys(pool, nch, gt.G, key_g, kA, vA, kB, vB, step, bkey_buf, d_radix_tmp,
                                      d_scan_tmp, st, &e);
    if (e != hipSuccess) return e;
    *bkey_out = bkey;
    hipLaunchKernelGGL(chain_keys_kernel, dim3(cgrid), dim3(kBlock), 0, st, pool, nch, gt.G, mp.table_size,
                       1.0 / (double)mp.table_size, bkey, key_s, key_b);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    int buf = 0;
    if ((e = radix_sort<uint64_t>(key_s, nullptr, nch, 32, kA, vA, kB, vB, d_radix_tmp, &buf, st)) != hipSuccess)
        return e;
    const uint32_t* ord1 = buf ? vB : vA;
    int tb = 1;   // bucket bits
    while (tb < 32 && ((uint64_t)1 << tb) < (uint64_t)mp.table_size) ++tb;
    int kb = 32, low_shift = 0;   // block key bits
    if (!bkey) {
        kb = gt.G;
        low_shift = 32 - gt.G;
    } else {
        kb = 1;
        while (kb < 32 && ((uint64_t)1 << kb) < (uint64_t)nch) ++kb;
    }
    hipLaunchKernelGGL(gather_gkey_kernel, dim3(cgrid), dim3(kBlock), 0, st, key_b, ord1, nch, low_shift, kb, key_g);
    uint32_t* vin = buf ? vB : vA;
    uint32_t* vout = buf ? vA : vB;
    int buf2 = 0;
    if ((e = radix_sort<uint64_t>(key_g, vin, nch, kb + tb, kA, vout, kB, vin, d_radix_tmp, &buf2, st)) != hipSuccess)
        return e;
    const uint32_t* ord = buf2 ? vin : vout;
    hipLaunchKernelGGL(chain_next_kernel, dim3(cgrid), dim3(kBlock), 0, st, ord, key_s, key_b, nch, next_s, rank);
    return hipGetLastError();
}

template <int MG, typename View>
hipError_t launch_replay_kept(View v, const GenomeTable& gt, const MatchParams& mp, int L, uint64_t P,
                              const int64_t* pool, const uint32_t* chain_of, const uint32_t* fk, uint32_t nch,
                              void* d_tmp, void* d_radix_tmp, void* d_scan_tmp, uint32_t lds_cap, uint32_t* tsize,
                              void* ctr, uint64_t* dbg, hipStream_t st, uint64_t* mlog, uint32_t** tbl_out,
                              const uint32_t** base_out, void* (*alloc)(void*, size_t), void* alloc_ctx,
                              const uint32_t* jl) {
    char* p = (char*)d_tmp;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    uint64_t* key_s = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* key_b = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* key_g = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* kA = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* kB = (uint64_t*)carve((size_t)nch * 8);
    uint32_t* vA = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* vB = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* next_s = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* rank = (uint32_t*)carve((size_t)nch * 4);
    uint4* chain_sb = (uint4*)carve((size_t)nch * 16);
    uint32_t* bkey_buf = (uint32_t*)carve((size_t)nch * 4);
    const uint64_t nblk = (P + kBlock * kKeepIPT - 1) / (kBlock * kKeepIPT);
    unsigned int* nkept = (unsigned int*)carve(64);
    uint4* ckeep = (uint4*)carve((size_t)nch * 16);
    const unsigned cgrid = (nch + kBlock - 1) / kBlock;
    hipError_t e = hipSuccess;
    const uint32_t* bkey = nullptr;
    if ((e = chain_order(pool, nch, gt, mp, key_s, key_b, key_g, kA, kB, vA, vB, next_s, bkey_buf, d_radix_tmp,
                         d_scan_tmp, next_s, rank, &bkey, st)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(chain_sb_kernel, dim3(cgrid), dim3(kBlock), 0, st, pool, nch, gt.G, rank, next_s, chain_sb);
    hipLaunchKernelGGL(chain_keep_kernel, dim3(cgrid), dim3(kBlock), 0, st, fk, (const uint32_t*)next_s,
                       (const uint64_t*)key_b, nch, ckeep);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the kept probes, one pass into a buffer of a guessed capacity (again, exactly sized,
    // when the guess was short)
    const int G = gt.G;
    const uint32_t Tb = mp.table_size;
    int tbits = 1;
    while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)Tb) ++tbits;
    uint64_t cap = std::min<uint64_t>(P, (uint64_t)nch * 2 + (P >> 6) + 4096);
    uint32_t Kc = 0;
    char* cb = nullptr;
    uint64_t* kept = nullptr;
    for (int attempt = 0; attempt < 2; ++attempt) {
        const uint64_t K1 = cap + 1;
        const size_t rtmp = radix_tmp_bytes(K1);
        cb = (char*)alloc(alloc_ctx, K1 * (8 * 3 + 4 * 3 + 16 * 3 + 4) + ((uint64_t)Tb + 64) * 8 + rtmp +
                                         replay_scratch_bytes(cap, Tb) + 16 * 256);
        if (!cb) return hipErrorOutOfMemory;
        kept = (uint64_t*)cb;
        uint32_t* kcid = (uint32_t*)(cb + ((K1 * 8 + 255) & ~(uint64_t)255));
        if ((e = hipMemsetAsync(nkept, 0, 4, st)) != hipSuccess) return e;
        if (jl)
            hipLaunchKernelGGL(keep_fill_line_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, jl, P,
                               (const uint4*)ckeep, nkept, cap, kept, kcid);
        else
            hipLaunchKernelGGL(keep_fill_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, st, v.rows, P, G, chain_of,
                               (const uint4*)ckeep, nkept, cap, kept, v.fs, kcid);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(&Kc, nkept, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        if (Kc <= cap) break;
        cap = Kc;
    }
    const uint64_t K1 = (uint64_t)cap + 1;
    const size_t rtmp = radix_tmp_bytes(K1);
    p = cb;
    carve(K1 * 8);   // kept
    uint32_t* kcid = (uint32_t*)carve(K1 * 4);   // their chains
    uint64_t* sA = (uint64_t*)carve(K1 * 8);
    uint64_t* sB = (uint64_t*)carve(K1 * 8);
    uint32_t* iA = (uint32_t*)carve(K1 * 4);
    uint32_t* iB = (uint32_t*)carve(K1 * 4);
    uint4* summ_c = (uint4*)carve(K1 * 16);
    uint4* summ_bc = (uint4*)carve(K1 * 16);
    uint4* spill = (uint4*)carve(K1 * 16);
    uint32_t* tbl = (uint32_t*)carve(K1 * 4);
    uint32_t* cbeg = (uint32_t*)carve(((uint64_t)Tb + 32) * 4);
    uint32_t* cend = (uint32_t*)carve(((uint64_t)Tb + 32) * 4);
    void* rt = carve(rtmp);
    void* scr = carve(replay_scratch_bytes(cap, Tb));
    *tbl_out = tbl;
    *base_out = cbeg;
    const uint64_t* skey = kept;
    const uint32_t* scid = kcid;
    if (Kc > 1) {
        int b3 = 0;
        if ((e = radix_sort<uint64_t>(kept, kcid, Kc, 32 + tbits, sA, iA, sB, iB, rt, &b3, st)) != hipSuccess)
            return e;
        skey = b3 ? sB : sA;
        scid = b3 ? iB : iA;
    }
    if ((e = hipMemsetAsync(cbeg, 0, ((uint64_t)Tb + 32) * 4, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(cend, 0, ((uint64_t)Tb + 32) * 4, st)) != hipSuccess) return e;
    const unsigned kgrid = (unsigned)((Kc + 1 + kBlock - 1) / kBlock);
    hipLaunchKernelGGL((kept_summary_kernel<MG, View>), dim3(kgrid), dim3(kBlock), 0, st, v, gt, L, skey, Kc, scid,
                       fk, (const uint4*)chain_sb, bkey, summ_c, summ_bc);
    hipLaunchKernelGGL(kept_ranges_kernel, dim3(kgrid), dim3(kBlock), 0, st, skey, Kc, cbeg, cend, P,
                       (DevCounters*)ctr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return replay_tail<MG, View>(v, gt, mp, L, nullptr, summ_c, summ_bc, cbeg, cend, cbeg, tbl, spill, pool, chain_sb,
                                 Kc, scr, d_scan_tmp, lds_cap, tsize, ctr, dbg, st, mlog);
}

// ---- the sharded kept-probe export -------------------------------
// The bucket owner receives every rank's chain entries (source-rank order; a chain whose probes
// sit on several ranks arrives once per rank), merges equal ones (launch_chain_merge) and
// answers per received entry what the source needs to pick the probes the replay keeps: the
// chain's next_s and whether this entry is the chain's first in source order (its rank holds
// the chain's first AddHashEntry call).
size_t chain_thr_tmp_bytes(uint64_t n) {
    return chain_merge_tmp_bytes(n) + (n + 64) * (8 * 5 + 4 * 9) + 32 * 256;
}

namespace {

__global__ __launch_bounds__(kBlock) void iota_kernel(uint32_t* __restrict__ a, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] = (uint32_t)i;
}

__global__ __launch_bounds__(kBlock) void entry_thr_kernel(const uint32_t* __restrict__ gmap,
                                                           const uint32_t* __restrict__ first,
                                                           const uint32_t* __restrict__ next_s, uint64_t n,
                                                           uint2* __restrict__ thr) {
    const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const uint32_t m = gmap[e];
    thr[e] = make_uint2(next_s[m], first[m] == (uint32_t)e ? 1u : 0u);
}

}  // namespace

hipError_t launch_chain_thresholds(const int64_t* entries, uint64_t n, const GenomeTable& gt, const MatchParams& mp,
                                   int64_t* pool_out, void* d_tmp, void* d_radix_tmp, void* d_scan_tmp,
                                   uint32_t* d_nchains, uint32_t* h_nchains, uint2* thr, hipStream_t st) {
    *h_nchains = 0;
    if (n == 0) return hipSuccess;
    char* p = (char*)d_tmp;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    void* mtmp = carve(chain_merge_tmp_bytes(n));
    uint32_t* gmap = (uint32_t*)carve(n * 4);    // received entry -> merged chain (chain_remap of an iota)
    uint32_t* ident = (uint32_t*)carve(n * 4);   // first-probe stand-ins: the received entry's own index
    uint32_t* first = (uint32_t*)carve(n * 4);   // per merged chain: its first received entry
    const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(iota_kernel, dim3(grid), dim3(kBlock), 0, st, gmap, n);
    hipLaunchKernelGGL(iota_kernel, dim3(grid), dim3(kBlock), 0, st, ident, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_chain_merge(entries, n, gt.G, gmap, n, pool_out, mtmp, d_radix_tmp, d_scan_tmp, d_nchains, st,
                                ident, first)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(h_nchains, d_nchains, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    const uint32_t nch = *h_nchains;
    uint64_t* key_s = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* key_b = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* key_g = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* kA = (uint64_t*)carve((size_t)nch * 8);
    uint64_t* kB = (uint64_t*)carve((size_t)nch * 8);
    uint32_t* vA = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* vB = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* next_s = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* rank = (uint32_t*)carve((size_t)nch * 4);
    uint32_t* bkey_buf = (uint32_t*)carve((size_t)nch * 4);
    const uint32_t* bkey = nullptr;
    if ((e = chain_order(pool_out, nch, gt, mp, key_s, key_b, key_g, kA, kB, vA, vB, next_s, bkey_buf, d_radix_tmp,
                         d_scan_tmp, next_s, rank, &bkey, st)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(entry_thr_kernel, dim3(grid), dim3(kBlock), 0, st, (const uint32_t*)gmap,
                       (const uint32_t*)first, (const uint32_t*)next_s, n, thr);
    return hipGetLastError();
}

hipError_t launch_emit(const uint32_t* obase, const uint32_t* bstart, const uint32_t* tbl, const int64_t* pool, int G,
                       uint32_t table_size, uint64_t M, uint64_t* out_len, int64_t* out_s, hipStream_t st) {
    if (M == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_kernel, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, obase, bstart,
                       tbl, pool, G, table_size, M, out_len, out_s);
    return hipGetLastError();
}

#define MUMS_INST_REPLAY_KEPT(MG, V)                                                                              \
    template hipError_t launch_replay_kept<MG, V>(V, const GenomeTable&, const MatchParams&, int, uint64_t,           \
                                                  const int64_t*, const uint32_t*, const uint32_t*, uint32_t, void*,  \
                                                  void*, void*, uint32_t, uint32_t*, void*, uint64_t*, hipStream_t,   \
                                                  uint64_t*, uint32_t**, const uint32_t**, void* (*)(void*, size_t),  \
                                                  void*, const uint32_t*);
MUMS_INST_REPLAY_KEPT(4, MatProbes)
MUMS_INST_REPLAY_KEPT(8, MatProbes)
MUMS_INST_REPLAY_KEPT(16, MatProbes)
MUMS_INST_REPLAY_KEPT(32, MatProbes)
MUMS_INST_REPLAY_KEPT(64, MatProbes)

}  // namespace mums
