// mums_capi.hip -- C ABI (include/mums.h) over the gfx950 multi-MUM pipeline.
//
// One context = one MemHash instance (MemHash.h:38).  mums_find runs, on the
// context's HIP stream:
//   keys     seed_keys_kernel            ASCII -> ckey[N]             (A2-A4)
//   sort     radix_sort<K>               (ckey, idx) stable, 2w+1 bits  (A5-A7)
//   groups   probe_pass x2 + scan        accepted probes in key order (A8-A9)
//   buckets  radix_sort<u32> on bucket   probes grouped per bucket    (A10)
//   replay   replay_kernel               AddHashEntry + ExtendMatch   (A10-A11)
//   output   scan + emit_kernel          bucket-major MatchList       (A12)
// There is no CPU fallback: without a HIP device every call that would compute
// returns MUMS_E_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <functional>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mums.h"
#include "match_device.h"
#include "mums_internal.h"
#include "seed_device.h"

using namespace mums;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool borrowed = false;   // a view into another DevBuf's dead contents (not ours to free)
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        release();
        size_t want = bytes + (bytes >> 4) + 4096;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        else p = nullptr;
        return e;
    }
    void release() {
        if (p && !borrowed) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        borrowed = false;
    }
    // borrow [off, off + bytes) of `host` when it has room (host's contents are dead):
    // hipMalloc / hipFree of tens of GB cost about a second each at BASELINE config 5
    bool borrow(const DevBuf& host, size_t off, size_t bytes) {
        off = (off + 255) & ~(size_t)255;
        if (!host.p || off + bytes > host.cap) return false;
        release();
        p = (char*)host.p + off;
        cap = bytes;   // a larger ensure() reallocates instead of growing into the host
        borrowed = true;
        return true;
    }
    void drop_view() {
        if (borrowed) release();
    }
    template <typename T> T* as() const { return (T*)p; }
};

// host -> device on the context's stream, waited for: the context's kernels run on a
// non-blocking stream, which a null-stream hipMemcpy does not order itself against
static hipError_t h2d_sync(void* d, const void* h, size_t bytes, hipStream_t st) {
    const hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
    return e != hipSuccess ? e : hipStreamSynchronize(st);
}

struct GenomeIn {
    const char* d_ptr;
    uint64_t n;
    bool owned;
};

enum { EV_START, EV_KEYS, EV_SORT, EV_GROUPS, EV_BUCKETS, EV_CHAINS, EV_REPLAY, EV_OUTPUT, EV_COUNT };

constexpr uint32_t kReplayLdsIds = 8192;    // 16-B slots: 128 KiB of LDS per replay workgroup

}  // namespace

struct mums_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint64_t seed = 0;
    uint32_t repeat_tol = 0, enum_tol = 1, table_size = 40000;
    int masked = 0;
    uint64_t seq_mask = 0;
    std::vector<GenomeIn> genomes;
    std::string err;

    DevBuf packed, recA, recB, hist, tiles, ckey, kA, kB, vA, vB, tmp, partials, counters;
    DevBuf bstart, bend, tsize, obase, pool, tbl, out_len, out_s, pbuf, keybuf, mstart;
    DevBuf cmerge;   // compat MergeTable: first entry of every bucket that does not append
    DevBuf chain_tmp, chain_of, radix_tmp, spill, summ, dbgbuf, mprobe, rowtmp;
    DevBuf fk, fkloc;        // each chain's first probe in key order (merged / per slice)
    DevBuf side, bst8;       // keys wider than 32 + 8 bits: side bytes, 8-bit bucket starts (msdsplit.hip)
    DevBuf cbst;             // chunked mode, w20-21: every chunk's bucket starts after the split
    bool use_onesweep = true;
    // ParallelMemHash chunk-compat mode (compat.hip): chunk = CHUNK_SIZE, ParallelMemHash.cpp:51
    bool pcompat = false;
    bool compat_rec = false;   // compat: the chunk-major stream as packed records (run_pipeline_compat)
    // compat over ranks (compat_ranks.hip): this context searches chunks [nch * compat_rank /
    // compat_ranks, nch * (compat_rank + 1) / compat_ranks) with tables of its own
    uint32_t compat_rank = 0, compat_ranks = 1;
    mums_ctx* compat_sub = nullptr;   // sharded compat: the rank's search over all genomes
    DevBuf rkpool0, rkpool1, rku32, ascii_all;   // sharded compat: the owner's merge (ctx_compat_rank_merge)
    bool prelabelled = false;   // find_tail: chain_of / pool_loc / fkloc hold the ranks' chain labels
    uint64_t prelab_n = 0;      // entries in pool_loc
    const int64_t* lab_rows = nullptr;   // sharded: the rank's own probe rows the labels refer to
    uint64_t lab_nch = 0;                // sharded: chains labelled among them
    uint64_t lab_p = 0;                  // sharded: probes labelled (the rank's own)
    double lab_ms = 0;                   // sharded: device time of the labelling
    // sharded kept-probe export (mums_shard_chain_entries -> mums_shard_kept_export): the
    // destinations computed for the entries, kept in labx; rows received as bucket owner
    uint32_t kx_nranks = 0;              // 0: no entry export pending
    std::vector<uint32_t> kx_estart;     // per destination: its first entry in the export order
    uint64_t own_rows = 0;               // rows the last sharded FindMatches replayed on this rank
    uint64_t own_dropped = 0;            // AddHashEntry calls of the owned buckets not sent (collisions)
    bool kept_rows = false;              // mums_shard_find_kept: entries may outnumber the rows
    bool pairwise = false;   // PairwiseMatchFinder (pairwise.hip)
    uint64_t chunk_size = 200000;
    uint32_t nchunks = 0;
    DevBuf cval, ctab;
    DevBuf fsk;              // FindMatches: first-genome start of each probe (key order)
    DevBuf bst2;             // {0, P}: the one bucket of the probes' onesweep bucket sort
    bool fused_keys = false; // materialize_seeds also writes the line keys and fsk (find_tail)
    bool rows_narrow = false; // ctx->mprobe holds int32 rows (MatProbes::rows32; materialize_dispatch)
    // one genome's SML / seed frequencies (sml_tools.hip) and filtered MatchLists
    DevBuf smlk0, smlkA, smlkB, smlvA, smlvB, smltmp, flen, fs;
    DevBuf rowsall;          // chunked mode: probe rows of all chunks
    DevBuf pool_loc, cbuf;   // chunked FindMatches: per-slice chain entries, compacted probes
    DevBuf sids;             // chunked FindMatches: the bucket order (its sort scratch released)
    DevBuf labx;             // sharded chain export scratch (mums_shard_chain_export)
    uint32_t* emit_tbl = nullptr;          // bucket vectors / slice bases of the last replay
    const uint32_t* emit_base = nullptr;   // (chunked: compacted, in cbuf; else tbl / bstart)
    EoWork eo;               // EliminateOverlaps work arrays (overlaps.hip)
    bool match_log = false;  // MemHash::SetMatchLog: record the inserts (replay.hip)
    uint64_t log_n = 0;
    DevBuf logA, logB, logvA, logvB;
    // MER_REPEAT_LIMIT restart / FindMatchesFromPosition (restart.hip)
    std::vector<uint64_t> start_points;   // per genome SML start index (empty = all 0)
    DevBuf rsbuf, rsplan, rsbst;
    DevBuf tiebuf;                        // SML tie order (smlsort.hip)
    DevBuf crbuf, crcnt, crlive, crruns;  // chunked-mode restarts (chunked.hip)
    uint64_t cr_cands = 0;                // groups above MER_REPEAT_LIMIT (chunked restart)
    DevBuf crall;                         // sharded restart planner: the whole stream's SMLs
    bool shard_restart_pending = false;
    uint64_t live_n = 0;                   // sharded: the live stream's records (after a restart)
    std::vector<uint32_t> live_bst;        // and its local bucket starts   // mums_shard_merge saw a group above the limit / start points
    int shard_mb = 0;                     // local bucket bits of the last mums_shard_merge
    int shard_side = 0;                   // 33-bit records at w20-21: side bits split below the 8-bit scatter
    uint64_t shard_n = 0;                 // its records
    uint32_t shard_kfirst = 0, shard_kcount = 0;   // its key range (first MSD bucket, buckets)
    std::vector<uint32_t> shard_bst;      // its local bucket starts (2^shard_mb + 1)
    // the restart planned where the records are (mums_shard_restart_counts .. _finish)
    DevBuf dsarr;                         // PlanData arrays (m, lbase, off, n, prv, nxt), S0, flags
    bool ds_ready = false;
    uint64_t ds_C = 0;                    // this rank's candidates (groups above MER_REPEAT_LIMIT)
    std::vector<uint64_t> ds_n, ds_off;   // SML indices [off, off + n) of every genome held here
    std::vector<uint64_t> ds_rkey, ds_rS; // this rank's restarts (last step)
    bool ds_ties = false;                 // repeat tolerance: every run's ids rewritten (mums_shard_tie_apply)
    uint64_t rs_info[4] = {0, 0, 0, 0};   // mums_shard_restart_info
    bool ties_fixed = false;              // the stream holds every run of equal keys in std::sort order
    uint64_t tie_slots = 0;               // slots of the runs replayed by the last run (stats)
    // seed-stage-only chunked runs keep the tie workspace between calls when memory allows:
    // its hipMalloc is 3-4 s at 2 x 3 Gbp (135 GB), the replay itself 0.15 s
    int keep_tiebuf = 0;                  // 1: keep when memory stays free beside it, 2: keep (the tail lives inside)
    bool tiebuf_kept = false;             // the last chunked seed-stage-only call kept tiebuf
    uint64_t restarts = 0;
    std::vector<uint64_t> offset_log;     // start points after every restart (R x G)
    std::vector<uint64_t> consumed_log;   // consumed SML positions at every restart (R x G, restart plan)
    std::vector<uint32_t> compat_pfirst;  // compat + match log: first probe of every chunk (nch + 1)
    std::vector<uint32_t> log_ids;        // compat + match log: the logged entries (pool ids) in log order
    // compat ranks: the one-thread log made on rank 0 (ctx_compat_rank_find); mums_match_log_copy
    // reads these when log_host is set
    bool log_host = false;
    std::vector<uint64_t> log_hlen;
    std::vector<int64_t> log_hs;
    std::vector<uint64_t> compat_cons;    // compat: consumed SML positions of every chunk cut by MER_REPEAT_LIMIT
    const uint64_t* compat_ck_src = nullptr;   // compat: crall not built yet, derive it from these SML keys
    uint64_t compat_ck_mask = 0;
                                          // (nch x G, ~0 = not cut), compat_truncate
    bool progress_on = false;             // MatchFinder::LogProgress: restate the progress text
    std::string progress;                 // its text for the last seed stage
    hipEvent_t ev[EV_COUNT] = {};
    bool profiling = false;
    bool walk_events = false;    // ev_walk recorded by the last FindMatches
    hipEvent_t ev_ds[16] = {};   // 2 per radix pass (<= 8 passes)
    hipEvent_t ev_walk[6] = {};  // per walk pass: before the short walks, after them, after the long walks (chains.hip)

    // sharded seed stage: this context owns genomes [shard_first,
    // shard_first + genomes.size()) of a problem whose genome lengths are shard_len
    bool shard = false;
    uint32_t shard_first = 0;
    std::vector<uint64_t> shard_len;
    GenomeTable lgt{};        // the owned genomes, global seed-mer bases
    double shard_keys_ms = 0;
    // position-sharded layout (BASELINE config 5 on 8 GPUs): this context's one genome is
    // the ASCII of genome slice_genome's bases [slice_begin, slice_end + L - 1), it owns
    // the SML positions [slice_begin, slice_end)
    bool slice = false;
    uint32_t slice_genome = 0;
    uint64_t slice_begin = 0, slice_end = 0;
    int rec_ib = 32;          // index bits of the packed records (33: > 2^32 seed-mers)
    bool merge_chunked = false;   // the last shard merge ran in key chunks of < 2^30 records
    bool shard_rows_built = false;   // chunked merge: every chunk's probe rows in rowsall (shard_chunk_rows)

    // state of the last run
    int stage_done = 0;
    bool key64 = false;
    bool packed_path = false;
    int msd_bits = 0;
    int L = 0, w = 0;
    uint64_t pattern = 0, N = 0, P = 0, M = 0;
    int sorted_buf = 0;
    int sort_passes = 0;
    bool parity_masked = false;   // sorted_rec ordered by the masked key only (seg_parity_fix restores)
    const uint64_t* sorted_rec = nullptr;   // packed path
    const void* sorted_key = nullptr;       // pair path
    const uint32_t* sorted_idx = nullptr;
    GenomeTable gt{};
    SeedSpec ss{};
    DevCounters hc{};
    mums_stats st{};
    const uint32_t* sorted_ids = nullptr;
    const uint32_t* sorted_buckets = nullptr;
    const uint64_t* probe_info = nullptr;
};

namespace {

void release_tiebuf(mums_ctx* ctx);
hipError_t tiebuf_ensure(mums_ctx* ctx, size_t bytes);
void release_find_buffers(mums_ctx* ctx);
void note_rs_bytes(mums_ctx* ctx);

int fail(mums_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hipfail(mums_ctx* c, hipError_t e, const char* where) {
    return fail(c, e == hipErrorOutOfMemory ? MUMS_E_NOMEM : MUMS_E_HIP,
                std::string(where) + ": " + hipGetErrorString(e));
}

#define HIPCHK(expr)                                               \
    do {                                                           \
        hipError_t e_ = (expr);                                    \
        if (e_ != hipSuccess) return hipfail(ctx, e_, #expr);      \
    } while (0)

bool have_device() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

SeedSpec make_seed_spec(uint64_t pattern, int L, int w) {
    SeedSpec ss{};
    ss.pattern = pattern;
    ss.L = L;
    ss.w = w;
    int cum = 0, r = -1;
    bool prev = false;
    for (int k = 0; k < L; ++k) {
        const bool care = (pattern >> (L - 1 - k)) & 1;
        if (care) {
            if (!prev) {
                ++r;
                ss.run_start[r] = k;
                ss.run_len[r] = 0;
            }
            ss.run_len[r]++;
        }
        prev = care;
    }
    ss.nruns = r + 1;
    for (int i = 0; i < ss.nruns; ++i) {
        cum += ss.run_len[i];
        ss.run_dst[i] = 2 * (w - cum);
        ss.run_sh[i] = 64 - 2 * (ss.run_start[i] + ss.run_len[i]) - ss.run_dst[i];
        ss.run_mask[i] = ((ss.run_len[i] >= 32) ? ~0ull : ((1ull << (2 * ss.run_len[i])) - 1)) << ss.run_dst[i];
    }
    return ss;
}

int seed_len(uint64_t s) {
    if (!s) return 0;
    int lo = __builtin_ctzll(s), hi = 63 - __builtin_clzll(s);
    return hi - lo + 1;
}

// probes of the merged stream -> probe_info/probe_bucket (ascending key order)
template <int MG, typename View>
int run_groups(mums_ctx* ctx, View v, const SegTile* tiles, uint64_t ntiles, const MatchParams& mp,
               uint64_t* probe_info, uint32_t* probe_bucket, uint64_t* slot_info, uint32_t* slot_bucket,
               hipStream_t st) {
    // one count per probe-stage workgroup: [nb] probes, then [nb] groups, then offsets
    const bool packed = RecIB<View>::value > 0;
    const uint64_t nb = group_blocks(ntiles, packed);
    uint32_t* counts = ctx->partials.as<uint32_t>();
    uint32_t* gcounts = counts + nb + 32;
    uint32_t* offs = gcounts + nb + 32;
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK((launch_probe_tiles<MG, View>(v, tiles, ntiles, ctx->N, ctx->gt, mp, ctx->L, counts, slot_info, slot_bucket,
                                         dc, st)));
    HIPCHK(exclusive_scan_u32(gcounts, nb, ctx->tmp.p, &dc->ngroups, st));
    HIPCHK(hipMemcpyAsync(offs, counts, nb * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(exclusive_scan_u32(offs, nb, ctx->tmp.p, &dc->nprobes, st));
    HIPCHK(launch_probe_compact(nb, counts, offs, slot_info, slot_bucket, probe_info, probe_bucket, st, packed));
    return MUMS_OK;
}

template <typename View>
int groups_dispatch(mums_ctx* ctx, View v, const SegTile* tiles, uint64_t ntiles, const MatchParams& mp,
                    uint64_t* pi, uint32_t* pb, uint64_t* si, uint32_t* sb, hipStream_t st) {
    const int G = ctx->gt.G;   // genomes of the whole problem (sharded contexts own a subset)
    if (G <= 4) return run_groups<4, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    if (G <= 8) return run_groups<8, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    if (G <= 16) return run_groups<16, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    if (G <= 32) return run_groups<32, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    return run_groups<64, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
}

void* devbuf_alloc(void* b, size_t bytes) {
    DevBuf* d = (DevBuf*)b;
    return d->ensure(bytes) == hipSuccess ? d->p : nullptr;
}

// chain labelling (chains.hip) then the per-bucket replay (replay.hip) of the P probe
// rows v (key order), bucket-sorted as ctx->sorted_ids; packed = all genomes (gt layout)
template <int MG>
int find_replay(mums_ctx* ctx, MatProbes v, const MatchParams& mp, hipStream_t st);

// v.fs set: the materialize pass also wrote the line keys (chain_lkey_slot) and first starts
template <int MG>
int find_rows(mums_ctx* ctx, MatProbes v, const uint32_t* packed, const MatchParams& mp, hipStream_t st) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t P = ctx->P;
    HIPCHK(ctx->fk.ensure((P + 1) * 4));
    // chain / probe / first start per line position in ctx->chain_of (3 P words, find_tail):
    // the replay's keep pass reads them in line order, no per-probe chain id is scattered
    HIPCHK((launch_chains<MG, MatProbes>(v, nullptr, P, ctx->gt, mp, ctx->ss, packed,
                                    ctx->chain_tmp.p, ctx->tmp.p, ctx->radix_tmp.p, nullptr,
                                    ctx->pool.as<int64_t>(), &dc->nchains, st, dc,
                                    ctx->profiling ? ctx->ev_walk : nullptr, ctx->fk.as<uint32_t>(), 0u,
                                    v.fs != nullptr, ctx->chain_of.as<uint32_t>())));
    return find_replay<MG>(ctx, v, mp, st);
}

template <int MG>
int find_replay(mums_ctx* ctx, MatProbes v, const MatchParams& mp, hipStream_t st) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t P = ctx->P;
    ctx->walk_events = ctx->profiling;
    HIPCHK(hipEventRecord(ctx->ev[EV_CHAINS], st));
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint64_t* dbg = nullptr;
    if (getenv("MUMS_DEV_REPLAY_DEBUG")) {
        HIPCHK(ctx->dbgbuf.ensure((size_t)ctx->table_size * 64));
        HIPCHK(hipMemsetAsync(ctx->dbgbuf.p, 0, (size_t)ctx->table_size * 64, st));
        dbg = ctx->dbgbuf.as<uint64_t>();
    }
    uint64_t* mlog = nullptr;
    ctx->log_n = 0;
    if (ctx->match_log) {
        HIPCHK(ctx->logA.ensure((P + 1) * 8));
        HIPCHK(ctx->logB.ensure((P + 1) * 8));
        mlog = ctx->logB.as<uint64_t>();   // unsorted events; sorted into logA
    }
    // the fullest bucket's vector in LDS when it fits (it holds <= its probes)
    const uint32_t lds_cap = std::max<uint32_t>(64, std::min<uint32_t>(ctx->hc.max_bucket, kReplayLdsIds));
    HIPCHK((launch_replay_kept<MG, MatProbes>(v, ctx->gt, mp, ctx->L, P, ctx->pool.as<int64_t>(), nullptr,
                                         ctx->fk.as<uint32_t>(), ctx->hc.nchains,
                                         ctx->chain_tmp.p, ctx->radix_tmp.p, ctx->tmp.p, lds_cap,
                                         ctx->tsize.as<uint32_t>(), ctx->counters.p, dbg, st, mlog, &ctx->emit_tbl,
                                         &ctx->emit_base, devbuf_alloc, &ctx->cbuf, ctx->chain_of.as<uint32_t>())));
    if (mlog) {   // the inserts in AddHashEntry call order (probe index << 32 | chain)
        HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const uint64_t n = ctx->hc.log_n;
        HIPCHK(ctx->logB.ensure((n + 1) * 8));
        HIPCHK(ctx->logvA.ensure((n + 1) * 4));
        HIPCHK(ctx->logvB.ensure((n + 1) * 4));
        int buf = 0;
        if (n) HIPCHK(radix_sort<uint64_t>(mlog, nullptr, n, 64, ctx->logA.as<uint64_t>(), ctx->logvA.as<uint32_t>(),
                                           ctx->logB.as<uint64_t>(), ctx->logvB.as<uint32_t>(), ctx->radix_tmp.p, &buf,
                                           st));
        if (buf) std::swap(ctx->logA, ctx->logB);   // sorted events in logA
        ctx->log_n = n;
    }
    if (dbg) {   // development instrumentation: the slowest buckets of the replay
        std::vector<uint64_t> h((size_t)ctx->table_size * 8);
        HIPCHK(hipMemcpyAsync(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::vector<uint32_t> idx(ctx->table_size);
        for (uint32_t i = 0; i < ctx->table_size; ++i) idx[i] = i;
        std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return h[a * 8 + 7] > h[b * 8 + 7]; });
        for (int k = 0; k < 5; ++k) {
            const uint64_t* d = &h[(size_t)idx[k] * 8];
            fprintf(stderr, "replay bucket %u: probes %lu entries %lu windows %lu rounds %lu | us win %.1f round %.1f "
                    "ins %.1f total %.1f\n", idx[k], (unsigned long)d[0], (unsigned long)d[1], (unsigned long)d[2],
                    (unsigned long)d[3], d[4] / 100.0, d[5] / 100.0, d[6] / 100.0, d[7] / 100.0);
        }
    }
    return MUMS_OK;
}

// SetMatchLog under ParallelMemHash (the patched 2-argument AddHashEntry logs every insert,
// MemHash.cpp:238-241), one OpenMP thread: for every chunk, its SearchRange's
// inserts into the thread table in call order (the replay's log events of the chunk's
// probes), then MergeTable's (ParallelMemHash.cpp:105-121): the chunk's new entries that
// survive the re-add, bucket by bucket in vector order.  An entry can only enter the global
// table at its own chunk's merge, and the final table holds exactly the surviving entries in
// that order, so the merge lines of chunk c are the final table's entries created in chunk c.
int compat_log_order(mums_ctx* ctx, uint32_t Tb, hipStream_t st) {
    const uint64_t n = ctx->log_n;
    const uint32_t nch = ctx->compat_pfirst.empty() ? 0 : (uint32_t)ctx->compat_pfirst.size() - 1;
    std::vector<uint64_t> ev(n);
    if (n) HIPCHK(hipMemcpyAsync(ev.data(), ctx->logA.p, n * 8, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> ts(Tb), tb(Tb);
    HIPCHK(hipMemcpyAsync(ts.data(), ctx->tsize.p, (size_t)Tb * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(tb.data(), ctx->emit_base, (size_t)Tb * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint64_t end = 0;
    for (uint32_t b = 0; b < Tb; ++b)
        if (ts[b]) end = std::max<uint64_t>(end, (uint64_t)tb[b] + ts[b]);
    std::vector<uint32_t> tbl(end);
    if (end) HIPCHK(hipMemcpy(tbl.data(), ctx->emit_tbl, end * 4, hipMemcpyDeviceToHost));
    auto chunk_of_probe = [&](uint64_t k) -> uint32_t {
        if (!nch) return 0;
        const auto it = std::upper_bound(ctx->compat_pfirst.begin(), ctx->compat_pfirst.end() - 1, (uint32_t)k);
        return (uint32_t)(it - ctx->compat_pfirst.begin()) - 1;
    };
    uint32_t maxid = 0;
    for (uint64_t i = 0; i < n; ++i) maxid = std::max(maxid, (uint32_t)(ev[i] & 0xFFFFFFFFull));
    std::vector<uint32_t> made(maxid + 1u, 0);   // chunk that created each pool entry
    std::vector<std::vector<uint32_t>> lines(std::max<uint32_t>(nch, 1));
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t cid = (uint32_t)(ev[i] & 0xFFFFFFFFull), c = chunk_of_probe(ev[i] >> 32);
        made[cid] = c;
        lines[c].push_back(cid);
    }
    std::vector<std::vector<uint32_t>> merged(lines.size());
    for (uint32_t b = 0; b < Tb; ++b)
        for (uint32_t j = 0; j < ts[b]; ++j) {
            const uint32_t cid = tbl[(uint64_t)tb[b] + j];
            if (cid > maxid) return fail(ctx, MUMS_E_HIP, "compat match log: an entry without an insert (internal error)");
            merged[made[cid]].push_back(cid);
        }
    ctx->log_ids.clear();
    for (size_t c = 0; c < lines.size(); ++c) {
        ctx->log_ids.insert(ctx->log_ids.end(), lines[c].begin(), lines[c].end());
        ctx->log_ids.insert(ctx->log_ids.end(), merged[c].begin(), merged[c].end());
    }
    ctx->log_n = ctx->log_ids.size();
    return MUMS_OK;
}

// FindMatches above find_chunk() probes (BASELINE config 5: 2.5e9): chains labelled per
// slice of find_chunk() probes (key order) into per-slice entries, merged by content
// (chains.hip), then the replay of the kept probes (launch_replay_kept).
// Per-probe memory: rows, chain_of, tbl, spill, the bucket order and one keep flag.
uint64_t find_chunk() {
    uint64_t c = 1ull << 28;
    if (const char* e = getenv("MUMS_DEV_FIND_CHUNK")) c = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    return c;
}

// Chains of the P probe rows v (key order) labelled slice by slice (find_chunk() probes
// each, key order) into per-slice entries: ctx->pool_loc (*nloc_out x (G + 2) words),
// ctx->fkloc (each entry's first probe, global index) and ctx->chain_of (probe -> entry).
// A chain whose probes fall into k slices has k equal entries (merge_slices).
template <int MG>
int label_slices(mums_ctx* ctx, MatProbes v, const uint32_t* packed, const MatchParams& mp, hipStream_t st,
                 uint64_t* nloc_out) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t P = ctx->P, C = find_chunk();
    const int G = ctx->gt.G;
    const size_t W = (size_t)(G + 2) * 8;
    uint32_t* chain_of = ctx->chain_of.as<uint32_t>();
    uint64_t nloc = 0;
    for (uint64_t k0 = 0; k0 < P; k0 += C) {
        const uint64_t n = std::min(C, P - k0);
        if (ctx->pool_loc.cap < (nloc + n + 1) * W) {   // grow, keeping the entries so far
            DevBuf nb;
            HIPCHK(nb.ensure(std::max((nloc + n + 1) * W, ctx->pool_loc.cap + ctx->pool_loc.cap / 4)));
            if (nloc) HIPCHK(hipMemcpyAsync(nb.p, ctx->pool_loc.p, nloc * W, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
            ctx->pool_loc.release();
            ctx->pool_loc = nb;
        }
        if (ctx->fkloc.cap < (nloc + n + 1) * 4) {
            DevBuf nb;
            HIPCHK(nb.ensure(std::max((nloc + n + 1) * 4, ctx->fkloc.cap + ctx->fkloc.cap / 4)));
            if (nloc) HIPCHK(hipMemcpyAsync(nb.p, ctx->fkloc.p, nloc * 4, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
            ctx->fkloc.release();
            ctx->fkloc = nb;
        }
        MatProbes vc = v;
        vc.rows = v.rows + k0 * (uint64_t)(G + 1);
        HIPCHK((launch_chains<MG, MatProbes>(vc, nullptr, n, ctx->gt, mp, ctx->ss, packed, ctx->chain_tmp.p, ctx->tmp.p,
                                        ctx->radix_tmp.p, chain_of + k0,
                                        ctx->pool_loc.as<int64_t>() + nloc * (uint64_t)(G + 2), &dc->nchains, st, dc,
                                        nullptr, ctx->fkloc.as<uint32_t>() + nloc, (uint32_t)k0)));
        uint32_t nc = 0;
        HIPCHK(hipMemcpyAsync(&nc, &dc->nchains, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (nloc + nc >= (1ull << 31)) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^31 seed chains in one FindMatches");
        HIPCHK(launch_add_offset(chain_of + k0, n, (uint32_t)nloc, st));
        nloc += nc;
    }
    *nloc_out = nloc;
    return MUMS_OK;
}

// The nloc per-slice (or per-rank) entries in ctx->pool_loc / ctx->fkloc merged by content
// into ctx->pool / ctx->fk (chain_of remapped; *nch_out merged chains), then the replay of
// the kept probes (launch_replay_kept) and the match log.
template <int MG>
int replay_merged(mums_ctx* ctx, MatProbes v, const MatchParams& mp, hipStream_t st, uint64_t nloc) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t P = ctx->P;
    const int G = ctx->gt.G;
    const size_t W = (size_t)(G + 2) * 8;
    uint32_t* chain_of = ctx->chain_of.as<uint32_t>();
    HIPCHK(ctx->chain_tmp.ensure(chain_merge_tmp_bytes(nloc)));
    HIPCHK(ctx->pool.ensure((nloc + 1) * W));
    HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(nloc + 1)));
    HIPCHK(ctx->fk.ensure((nloc + 1) * 4));
    HIPCHK(launch_chain_merge(ctx->pool_loc.as<int64_t>(), nloc, G, chain_of, P, ctx->pool.as<int64_t>(),
                              ctx->chain_tmp.p, ctx->radix_tmp.p, ctx->tmp.p, &dc->nchains, st,
                              ctx->fkloc.as<uint32_t>(), ctx->fk.as<uint32_t>()));
    ctx->walk_events = false;
    HIPCHK(hipEventRecord(ctx->ev[EV_CHAINS], st));
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t nch = ctx->hc.nchains;
    HIPCHK(ctx->chain_tmp.ensure(nch * 112 + 64 * 256));   // the replay's chain keys / ranks
    HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(nch + 1)));
    uint64_t* mlog = nullptr;
    ctx->log_n = 0;
    if (ctx->match_log) {
        HIPCHK(ctx->logA.ensure((P + 1) * 8));
        HIPCHK(ctx->logB.ensure((P + 1) * 8));
        mlog = ctx->logB.as<uint64_t>();
    }
    const uint32_t lds_cap = std::max<uint32_t>(64, std::min<uint32_t>(ctx->hc.max_bucket, kReplayLdsIds));
    HIPCHK((launch_replay_kept<MG, MatProbes>(v, ctx->gt, mp, ctx->L, P, ctx->pool.as<int64_t>(), chain_of,
                                         ctx->fk.as<uint32_t>(), (uint32_t)nch, ctx->chain_tmp.p, ctx->radix_tmp.p,
                                         ctx->tmp.p, lds_cap, ctx->tsize.as<uint32_t>(), ctx->counters.p, nullptr, st,
                                         mlog, &ctx->emit_tbl, &ctx->emit_base, devbuf_alloc, &ctx->cbuf)));
    if (mlog) {
        HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const uint64_t n = ctx->hc.log_n;
        HIPCHK(ctx->logvA.ensure((n + 1) * 4));
        HIPCHK(ctx->logvB.ensure((n + 1) * 4));
        int buf = 0;
        if (n) HIPCHK(radix_sort<uint64_t>(mlog, nullptr, n, 64, ctx->logA.as<uint64_t>(), ctx->logvA.as<uint32_t>(),
                                           ctx->logB.as<uint64_t>(), ctx->logvB.as<uint32_t>(), ctx->radix_tmp.p, &buf,
                                           st));
        if (buf) std::swap(ctx->logA, ctx->logB);
        ctx->log_n = n;
    }
    return MUMS_OK;
}

template <int MG>
int find_rows_chunked(mums_ctx* ctx, MatProbes v, const uint32_t* packed, const MatchParams& mp, hipStream_t st) {
    if (ctx->prelabelled) return replay_merged<MG>(ctx, v, mp, st, ctx->prelab_n);   // chains labelled by the ranks
    uint64_t nloc = 0;
    int rc = label_slices<MG>(ctx, v, packed, mp, st, &nloc);
    if (rc) return rc;
    return replay_merged<MG>(ctx, v, mp, st, nloc);
}

// chunked: find_tail's decision (P > find_chunk()), made once per call so the rows it
// materialized (64-bit rows for the sliced path, int32 rows only in the one-pass path)
// are the ones the chain kernels read
int find_rows_dispatch(mums_ctx* ctx, MatProbes v, const uint32_t* packed, const MatchParams& mp, hipStream_t st,
                       bool chunked) {
    const int G = ctx->gt.G;
    if (chunked) {
        if (!v.rows) return fail(ctx, MUMS_E_HIP, "sliced FindMatches needs 64-bit probe rows (internal error)");
        if (G <= 4) return find_rows_chunked<4>(ctx, v, packed, mp, st);
        if (G <= 8) return find_rows_chunked<8>(ctx, v, packed, mp, st);
        if (G <= 16) return find_rows_chunked<16>(ctx, v, packed, mp, st);
        if (G <= 32) return find_rows_chunked<32>(ctx, v, packed, mp, st);
        return find_rows_chunked<64>(ctx, v, packed, mp, st);
    }
    if (G <= 4) return find_rows<4>(ctx, v, packed, mp, st);
    if (G <= 8) return find_rows<8>(ctx, v, packed, mp, st);
    if (G <= 16) return find_rows<16>(ctx, v, packed, mp, st);
    if (G <= 32) return find_rows<32>(ctx, v, packed, mp, st);
    return find_rows<64>(ctx, v, packed, mp, st);
}

// the probes of the seed stage as rows (one build_probe each) in ctx->mprobe
template <typename View>
int materialize_dispatch(mums_ctx* ctx, View sv, const MatchParams& mp, hipStream_t st, int64_t* rows = nullptr) {
    const int G = ctx->gt.G;
    const uint64_t P = ctx->P;
    ctx->rows_narrow = false;
    // find_tail's own rows (ctx->fused_keys) as int32 starts when every start fits
    uint64_t mx = 0;
    for (int g = 0; g < G; ++g) mx = std::max<uint64_t>(mx, ctx->gt.n[g]);
    const char* wide_sw = getenv("MUMS_DEV_WIDE_ROWS");   // "1": 64-bit rows; "retry": the int32 rows flagged bad
    const bool force_retry = wide_sw && !strcmp(wide_sw, "retry");
    bool narrow = !rows && ctx->fused_keys && G <= 16 && mx + 2 < (1ull << 31) && (!wide_sw || force_retry);
    if (!rows) {   // into ctx->mprobe, else into the caller's (P + 1) rows
        HIPCHK(ctx->mprobe.ensure((P + 1) * (size_t)(G + 1) * 8));
        rows = ctx->mprobe.as<int64_t>();
    }
    uint64_t* lk = ctx->fused_keys ? chain_lkey_slot(ctx->chain_tmp.p, P, G) : nullptr;
    uint32_t* fs = ctx->fused_keys ? ctx->fsk.as<uint32_t>() : nullptr;
    uint32_t* lh = nullptr;   // the line sort's records and hashes instead of the line keys
    if (ctx->fused_keys && chain_line_records(P, ctx->gt)) chain_line_slots(ctx->chain_tmp.p, P, G, &lk, &lh);
    for (int pass = 0; pass < 2; ++pass) {
        int32_t* r32 = narrow ? (int32_t*)rows : nullptr;
        if (narrow) HIPCHK(hipMemsetAsync(fs + P, 0, 4, st));
        if (G <= 4) HIPCHK((launch_materialize<4, View>(sv, ctx->probe_info, P, ctx->gt, mp, ctx->L, rows, st, lk, fs, lh, r32)));
        else if (G <= 8) HIPCHK((launch_materialize<8, View>(sv, ctx->probe_info, P, ctx->gt, mp, ctx->L, rows, st, lk, fs, lh, r32)));
        else if (G <= 16) HIPCHK((launch_materialize<16, View>(sv, ctx->probe_info, P, ctx->gt, mp, ctx->L, rows, st, lk, fs, lh, r32)));
        else if (G <= 32) HIPCHK((launch_materialize<32, View>(sv, ctx->probe_info, P, ctx->gt, mp, ctx->L, rows, st, lk, fs, lh)));
        else HIPCHK((launch_materialize<64, View>(sv, ctx->probe_info, P, ctx->gt, mp, ctx->L, rows, st, lk, fs, lh)));
        if (!narrow) break;
        uint32_t bad = 0;
        HIPCHK(hipMemcpyAsync(&bad, fs + P, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (force_retry) bad = 1;
        if (!bad) {
            ctx->rows_narrow = true;
            break;
        }
        narrow = false;   // a start or offset the int32 rows do not restate: the 64-bit rows
    }
    return MUMS_OK;
}

int materialize_seeds(mums_ctx* ctx, const MatchParams& mp, hipStream_t st) {
    if (ctx->compat_rec) return materialize_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, mp, st);
    if (ctx->packed_path && ctx->rec_ib == 33)
        return materialize_dispatch<RecViewT<33>>(ctx, RecViewT<33>{ctx->sorted_rec}, mp, st);
    if (ctx->packed_path) return materialize_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, mp, st);
    if (ctx->key64)
        return materialize_dispatch<PairView<uint64_t>>(
            ctx, PairView<uint64_t>{(const uint64_t*)ctx->sorted_key, ctx->sorted_idx}, mp, st);
    return materialize_dispatch<PairView<uint32_t>>(
        ctx, PairView<uint32_t>{(const uint32_t*)ctx->sorted_key, ctx->sorted_idx}, mp, st);
}

// FindMatches after the bucket sort (ctx->P probes, ctx->sorted_ids / sorted_buckets):
// workspace, bucket ranges, [rows()] materialize, chains + replay, MatchList (A10-A12)
// stream_rows: rows() is materialize_seeds (the seed stage's probes from its merged stream):
// in the single-pass path it also writes the line keys and first starts (ctx->fused_keys)
template <typename Rows>
int find_tail(mums_ctx* ctx, const MatchParams& mp, const uint32_t* packed, Rows&& rows, hipStream_t st,
              bool stream_rows = false) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const int G = ctx->gt.G;
    const uint32_t Tb = ctx->table_size;
    HIPCHK(ctx->bstart.ensure((size_t)Tb * 4));
    HIPCHK(ctx->bend.ensure((size_t)Tb * 4));
    HIPCHK(ctx->tsize.ensure((size_t)Tb * 4));
    HIPCHK(ctx->obase.ensure((size_t)Tb * 4 + 64));
    if (ctx->P >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes in one FindMatches");
    const uint64_t fchunk = find_chunk();   // read once: the env switch may change between calls
    // prelabelled (sharded FindMatches): the ranks labelled the chains of their own probes;
    // their entries are merged and replayed like the slices of the sliced path
    const bool chunked = ctx->P > fchunk || ctx->prelabelled;
    HIPCHK(ctx->chain_of.ensure((ctx->P + 1) * (chunked ? 4 : 12)));   // find_rows: 3 words per line position
    // the replay keeps only the chain-first / suspicious probes (launch_replay_kept): its
    // summaries, bucket vectors and spill live in ctx->cbuf, sized by their count
    for (DevBuf* b : {&ctx->tbl, &ctx->spill, &ctx->summ}) b->release();
    if (chunked) {   // find_rows_chunked: chains per slice, merged
        ctx->pool.release();
    } else {
        HIPCHK(ctx->pool.ensure((ctx->P + 1) * (size_t)(G + 2) * 8));
        HIPCHK(ctx->chain_tmp.ensure(chain_tmp_bytes(ctx->P + 1, Tb, G)));
    }
    HIPCHK(ctx->radix_tmp.ensure(std::max(radix_tmp_bytes(ctx->P + 1),
                                          chain_radix_tmp_bytes(std::min<uint64_t>(ctx->P, find_chunk()) + 1))));
    HIPCHK(ctx->tmp.ensure(std::max(scan_tmp_bytes(ctx->P + 1), scan_tmp_bytes(Tb))));
    HIPCHK(hipMemsetAsync(ctx->bstart.p, 0, (size_t)Tb * 4, st));
    HIPCHK(hipMemsetAsync(ctx->bend.p, 0, (size_t)Tb * 4, st));
    HIPCHK(hipMemsetAsync(ctx->tsize.p, 0, (size_t)Tb * 4, st));
    if (ctx->sorted_buckets || ctx->P == 0) {
        HIPCHK(hipMemsetAsync(&dc->max_bucket, 0, 4, st));
        HIPCHK(launch_bucket_ranges(ctx->sorted_buckets, ctx->P, ctx->bstart.as<uint32_t>(),
                                    ctx->bend.as<uint32_t>(), &dc->max_bucket, st));
    } else {   // no bucket order (finish_seeds): the replay sizes its LDS vectors from the kept probes
        if (chunked) return fail(ctx, MUMS_E_HIP, "sliced FindMatches without the probes' bucket order (internal error)");
        HIPCHK(hipMemsetAsync(&dc->max_bucket, 0xFF, 4, st));
    }
    ctx->emit_tbl = ctx->tbl.as<uint32_t>();
    ctx->emit_base = ctx->bstart.as<uint32_t>();
    if (ctx->P == 0) HIPCHK(hipEventRecord(ctx->ev[EV_CHAINS], st));
    if (ctx->P > 0) {
        MatProbes v{};
        // the seed stage's own probes, one pass: rows plus line keys and first starts
        ctx->fused_keys = stream_rows && !chunked;
        if (ctx->fused_keys) HIPCHK(ctx->fsk.ensure((ctx->P + 1) * 4));
        int rc = rows(&v);
        ctx->fused_keys = false;
        if (rc) return rc;
        if (stream_rows && !chunked) v.fs = ctx->fsk.as<uint32_t>();
        if (stream_rows && !chunked && ctx->rows_narrow) {
            v.rows32 = (const int32_t*)ctx->mprobe.p;
            v.stride32 = line_row_stride(G);
            v.L32 = ctx->L;
            v.rows = nullptr;
        }
        if (chunked) {   // the rows hold all FindMatches reads: keep the bucket order only
            // the dead records (recA / recB, when the packed path sized them) are the arena
            // of the sliced FindMatches: bucket order and summaries in recB, chain scratch
            // in recA; buffers that do not fit there are allocated (and the rest freed)
            auto inside = [](const DevBuf& b, const void* q) {
                return b.p && (const char*)q >= (const char*)b.p && (const char*)q < (const char*)b.p + b.cap;
            };
            const bool arena = ctx->packed_path && !inside(ctx->recA, v.rows) && !inside(ctx->recB, v.rows) &&
                               !inside(ctx->recA, packed) && !inside(ctx->recB, packed);
            ctx->sorted_ids = nullptr;   // the replay needs no bucket order of all probes
            ctx->sorted_buckets = nullptr;
            ctx->probe_info = nullptr;
            ctx->sorted_rec = nullptr;
            ctx->sorted_key = nullptr;
            ctx->sorted_idx = nullptr;
            ctx->rowtmp.drop_view();
            // (prelabelled: only the merge of the received entries; the replay sizes its own)
            const size_t cbytes = ctx->prelabelled ? chain_merge_tmp_bytes(ctx->prelab_n + 1)
                                                   : chain_tmp_bytes(std::min<uint64_t>(ctx->P, fchunk) + 1, Tb, G);
            // a kept tie workspace holding the rows (run_pipeline_chunked) holds the chain
            // scratch behind them
            const bool in_tie = ctx->rowsall.borrowed && ctx->tiebuf.p && ctx->rowsall.p == ctx->tiebuf.p &&
                                ctx->chain_tmp.borrow(ctx->tiebuf, ctx->rowsall.cap, cbytes);
            if (!in_tie && !(arena && ctx->chain_tmp.borrow(ctx->recA, 0, cbytes)))
                HIPCHK(ctx->chain_tmp.ensure(cbytes));
            for (DevBuf* b : {&ctx->pbuf, &ctx->tiles, &ctx->rowtmp, &ctx->kA, &ctx->kB, &ctx->vA, &ctx->vB,
                              &ctx->ckey, &ctx->mprobe})
                if (!(b->p && (char*)v.rows >= (char*)b->p && (char*)v.rows < (char*)b->p + b->cap)) b->release();
            if (!arena) {
                ctx->recA.release();
                ctx->recB.release();
            }
        }
        rc = find_rows_dispatch(ctx, v, packed, mp, st, chunked);
        if (rc) return rc;
        if (ctx->pcompat) {   // ParallelMemHash::MergeTable (ParallelMemHash.cpp:105-121)
            HIPCHK(hipMemcpyAsync(ctx->obase.p, ctx->tsize.p, (size_t)Tb * 4, hipMemcpyDeviceToDevice, st));
            HIPCHK(exclusive_scan_u32(ctx->obase.as<uint32_t>(), Tb, ctx->tmp.p, &dc->nmatches, st));
            uint32_t tot = 0;
            HIPCHK(hipMemcpyAsync(&tot, &dc->nmatches, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            HIPCHK(ctx->cmerge.ensure((size_t)Tb * 4 + 64));
            HIPCHK(launch_compat_merge(ctx->tsize.as<uint32_t>(), ctx->emit_base, ctx->emit_tbl,
                                       ctx->pool.as<int64_t>(), G, Tb, &dc->collisions, ctx->obase.as<uint32_t>(), tot,
                                       ctx->cmerge.as<uint32_t>(), st));
        }
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_REPLAY], st));
    HIPCHK(hipMemcpyAsync(ctx->obase.p, ctx->tsize.p, (size_t)Tb * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(exclusive_scan_u32(ctx->obase.as<uint32_t>(), Tb, ctx->tmp.p, &dc->nmatches, st));
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->hc.err & 4u) return fail(ctx, MUMS_E_HIP, "bucket replay: an insert broke the rank order (internal error)");
    ctx->M = ctx->hc.nmatches;
    HIPCHK(ctx->out_len.ensure((ctx->M + 1) * 8));
    HIPCHK(ctx->out_s.ensure((ctx->M + 1) * (size_t)G * 8));
    HIPCHK(launch_emit(ctx->obase.as<uint32_t>(), ctx->emit_base, ctx->emit_tbl,
                       ctx->pool.as<int64_t>(), G, Tb, ctx->M, ctx->out_len.as<uint64_t>(), ctx->out_s.as<int64_t>(),
                       st));
    HIPCHK(hipEventRecord(ctx->ev[EV_OUTPUT], st));
    ctx->log_ids.clear();
    if (ctx->match_log && ctx->pcompat) {
        const int rc = compat_log_order(ctx, Tb, st);
        if (rc) return rc;
    }
    ctx->stage_done = MUMS_STAGE_ALL;
    return MUMS_OK;
}

// probe / slot arrays of the groups stage (one grow-only device buffer)
struct ProbeSpace {
    uint64_t* probe_info;
    uint64_t* slot_info;
    uint32_t* probe_bucket;
    uint32_t* bucketB;
    uint32_t* idsA;
    uint32_t* idsB;
    uint32_t* slot_bucket;
};

int ensure_probe_space(mums_ctx* ctx, uint64_t N, uint64_t ntiles_groups, ProbeSpace* ps) {
    const uint64_t pcap = (N / 2 + 2) & ~1ull;   // even: bucketB is 8-B aligned (finish_seeds)
    const uint64_t nslots = group_slot_count(ntiles_groups);
    HIPCHK(ctx->partials.ensure((3 * group_blocks(ntiles_groups, true) + 128) * 4));
    HIPCHK(ctx->pbuf.ensure(pcap * (8 + 4 * 4) + nslots * 12 + 256));
    char* pb = (char*)ctx->pbuf.p;
    ps->probe_info = (uint64_t*)pb;
    ps->slot_info = ps->probe_info + pcap;
    ps->probe_bucket = (uint32_t*)(ps->slot_info + nslots);
    ps->bucketB = ps->probe_bucket + pcap;
    ps->idsA = ps->bucketB + pcap;
    ps->idsB = ps->idsA + pcap;
    ps->slot_bucket = ps->idsB + pcap;
    return MUMS_OK;
}

// word offsets of the packed genomes and key-kernel tiles for the genomes of table t
// (sets t.woff / t.tfirst); returns the tile count, *words = packed words
uint32_t layout_packed(GenomeTable& t, uint64_t* words) {
    uint64_t wsum = 0;
    uint32_t T = 0;
    for (int g = 0; g < t.G; ++g) {
        t.woff[g] = wsum;
        wsum += (packed_words(t.n[g]) + 3) & ~3ull;
        t.tfirst[g] = T;
        T += (uint32_t)((t.n[g] + kSeedTile - 1) / kSeedTile);
    }
    t.woff[t.G] = wsum;
    for (int g = t.G; g <= kMaxG; ++g) t.tfirst[g] = T;
    *words = wsum;
    return T;
}

// Keys stage, packed path (rows A2-A4): pack the context's own genomes (table lgt, whose
// bases are GLOBAL seed-mer indices), histogram the top B key bits per tile, then scatter
// the (ckey_low << 32 | global index) records stably into their MSD buckets in out.
// Bucket starts -> bstart[0 .. 2^B] (device).
// side > 0 (keys wider than 32 + 8 bits, w20-21): the scatter runs on the top 8 bits into
// scratch (ctx->recB) with the next `side` key bits in ctx->side, and msd_split partitions
// the 256 buckets into the 2^B buckets of out.
int keys_stage(mums_ctx* ctx, const GenomeTable& lgt, uint32_t T, int B, uint64_t n, uint64_t* out, uint32_t* bstart,
               hipStream_t st, int ib = 32, int side = 0) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    std::vector<const char*> ptrs(lgt.G);
    for (int g = 0; g < lgt.G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
    uint32_t* hist = ctx->hist.as<uint32_t>();
    if (side > 0) {
        if (B != 8 + side || out == ctx->recB.as<uint64_t>() || (ib != 32 && ib != 33))
            return fail(ctx, MUMS_E_INVALID, "msd split");
        HIPCHK(ctx->side.ensure(n + 64));
        HIPCHK(ctx->bst8.ensure((256 + 64) * 4));
        HIPCHK(ctx->recB.ensure(n * 8 + 64));
        HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, msd_split_tmp_bytes(n, 8))));
        HIPCHK(launch_seed_pack(ctx->ss, lgt, ptrs.data(), ctx->packed.as<uint32_t>(), 1, true, nullptr, 8, hist, T,
                                &dc->err, st));
        HIPCHK(exclusive_scan_u32(hist, (uint64_t)T << 8, ctx->tmp.p, nullptr, st));
        if (ib == 32) {
            HIPCHK(launch_seed_scatter(ctx->ss, lgt, ctx->packed.as<uint32_t>(), 8, hist, T, ctx->recB.as<uint64_t>(),
                                       st, ctx->side.as<uint8_t>(), side));
        } else {   // 33-bit indices (sharded above 2^32 seed-mers, w20-21): chunked.hip's scatter, one chunk
            HIPCHK(ctx->ctab.ensure(64));
            HIPCHK(hipMemsetAsync(ctx->ctab.p, 0, 64, st));
            HIPCHK(launch_seed_scatter_chunk(ctx->ss, lgt, ctx->packed.as<uint32_t>(), 8, hist, T, 0, 0,
                                             ctx->recB.as<uint64_t>(), st, ctx->ctab.as<uint64_t>(), 8,
                                             ctx->side.as<uint8_t>(), side));
        }
        HIPCHK(seg_bucket_starts(hist, T, 8, n, ctx->bst8.as<uint32_t>(), st));
        HIPCHK(msd_split(ctx->recB.as<uint64_t>(), ctx->side.as<uint8_t>(), out, n, 8, side, ctx->bst8.as<uint32_t>(),
                         bstart, ctx->tmp.p, st));
        return MUMS_OK;
    }
    HIPCHK(launch_seed_pack(ctx->ss, lgt, ptrs.data(), ctx->packed.as<uint32_t>(), 1, true, nullptr, B, hist, T,
                            &dc->err, st));
    if (B > 0) HIPCHK(exclusive_scan_u32(hist, (uint64_t)T << B, ctx->tmp.p, nullptr, st));
    if (ib == 32) {
        HIPCHK(launch_seed_scatter(ctx->ss, lgt, ctx->packed.as<uint32_t>(), B, hist, T, out, st));
    } else {   // 33-bit indices: every digit kept, one chunk at base 0 (chunked.hip's scatter)
        HIPCHK(ctx->ctab.ensure(64));
        HIPCHK(hipMemsetAsync(ctx->ctab.p, 0, 64, st));
        HIPCHK(launch_seed_scatter_chunk(ctx->ss, lgt, ctx->packed.as<uint32_t>(), B, hist, T, 0, 0, out, st,
                                         ctx->ctab.as<uint64_t>(), B));
    }
    HIPCHK(seg_bucket_starts(B > 0 ? hist : nullptr, T, B, n, bstart, st));
    return MUMS_OK;
}

// Workspace of the merge stage for n records in 2^mb buckets of key_bits key bits.
// the records are about to be written: end the views borrowed from them (sliced FindMatches)
void records_live(mums_ctx* ctx) {
    for (DevBuf* b : {&ctx->rowtmp, &ctx->sids, &ctx->summ, &ctx->chain_tmp}) b->drop_view();
}

int ensure_merge_space(mums_ctx* ctx, uint64_t n, int mb, int key_bits, ProbeSpace* ps) {
    records_live(ctx);
    const uint64_t ub = seg_tiles_upper(n, mb);
    HIPCHK(ctx->recA.ensure(n * 8 + 64));
    HIPCHK(ctx->recB.ensure(n * 8 + 64));
    HIPCHK(ctx->tiles.ensure(ub * sizeof(SegTile) + 64));
    HIPCHK(ctx->mstart.ensure(((1ull << mb) + 64) * 4));
    size_t tmpb = std::max(seg_tmp_bytes(n, mb), onesweep_tmp_bytes(n, mb, key_bits));
    tmpb = std::max(tmpb, std::max(scan_tmp_bytes(n), radix_tmp_bytes(n / 2 + 1)));
    tmpb = std::max(tmpb, scan_tmp_bytes((uint64_t)ctx->table_size));
    HIPCHK(ctx->tmp.ensure(tmpb));
    return ensure_probe_space(ctx, n, ub, ps);
}

int tie_fix_stream(mums_ctx* ctx, const RsStream& s, uint64_t n, hipStream_t st);
bool wants_tie_order(const mums_ctx* ctx);

// Merge stage (rows A5-A9): n records in recA, bucket-major over 2^mb buckets whose starts
// are in ctx->mstart -> stable sort on record key bits [32, 32 + key_bits) inside every
// bucket (the merged SortedMerList stream) -> equal-key groups -> accepted probes in key order.
int merge_stage(mums_ctx* ctx, uint64_t n, int mb, int key_bits, const MatchParams& mp, const ProbeSpace& ps,
                hipStream_t st, int ib = 32, uint64_t* rA = nullptr, uint64_t* rB = nullptr) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    if (!rA) rA = ctx->recA.as<uint64_t>();
    if (!rB) rB = ctx->recB.as<uint64_t>();
    SegTile* tiles = ctx->tiles.as<SegTile>();
    const uint32_t* bstart = ctx->mstart.as<uint32_t>();
    const uint64_t ub = seg_tiles_upper(n, mb);
    const bool prof = ctx->profiling;
    HIPCHK(build_seg_tiles_from_starts(bstart, mb, n, tiles, &dc->ntiles, ctx->tmp.p, st));
    int buf = 0;
    if (ib != 32 && !(n < (1ull << 30) && key_bits <= 32))
        return fail(ctx, MUMS_E_UNSUPPORTED, "33-bit records need < 2^30 records per merge");
    // default tolerances: a masked-key group's probe does not depend on its records' order
    const bool mask_parity = mp.repeat_tol == 0 && mp.enum_tol == 1;
    ctx->parity_masked = false;
    const bool onesweep = ctx->use_onesweep && n < (1ull << 30) && key_bits <= 32;
    // three 10-bit passes, parity bit unsorted (radix_wide.hip; 31 key bits with the 8-bit MSD)
    const bool wide = onesweep && mask_parity && ib == 32 && seg_wide_sort_enabled() && seg_wide_passes(key_bits) <= 3;
    if (wide) {
        HIPCHK(seg_onesweep_sort_wide(rA, rB, n, key_bits, mb, bstart, ctx->tmp.p, &dc->err, &buf, st,
                                      prof ? ctx->ev_ds : nullptr, 32));
        ctx->parity_masked = true;
    } else if (onesweep) {
        HIPCHK(seg_onesweep_sort(rA, rB, n, key_bits, mb, bstart, ctx->tmp.p, &dc->err, &buf, st,
                                 prof ? ctx->ev_ds : nullptr, ib, mask_parity));
        ctx->parity_masked = mask_parity && seg_onesweep_launches(key_bits) < (key_bits + 7) / 8;
    } else
        HIPCHK(seg_radix_sort(rA, rB, n, key_bits, tiles, ub, ctx->tmp.p, &buf, st, prof ? ctx->ev_ds : nullptr));
    ctx->sorted_buf = buf;
    ctx->sorted_rec = buf ? rB : rA;
    ctx->sort_passes = wide ? seg_wide_passes(key_bits) : onesweep ? seg_onesweep_launches(key_bits) : (key_bits + 7) / 8;
    HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
    if (wants_tie_order(ctx) && ib == 32 && !ctx->shard) {
        RsStream s{};
        s.kind = 0;
        s.rec = ctx->sorted_rec;
        s.bstart = bstart;
        s.B = mb;
        s.kbits = 2 * ctx->w + 1;
        const int rc = tie_fix_stream(ctx, s, n, st);
        if (rc) return rc;
    }
    if (ib == 33)
        return groups_dispatch<RecViewT<33>>(ctx, RecViewT<33>{ctx->sorted_rec}, tiles, ub, mp, ps.probe_info,
                                             ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
    return groups_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, tiles, ub, mp, ps.probe_info, ps.probe_bucket,
                                    ps.slot_info, ps.slot_bucket, st);
}

// After the groups stage: counters to the host, error flags, then the probes grouped
// by hash bucket (stable: key order kept inside a bucket; values = probe ids) (A10).
// find_follows: FindMatches runs next on this context; its one-pass replay (launch_replay_kept)
// orders only the kept probes by bucket, so the bucket order of all probes is skipped there
// (MUMS_DEV_KEEP_BUCKET_ORDER, read per call: sort them anyway)
int finish_seeds(mums_ctx* ctx, const ProbeSpace& ps, hipStream_t st, bool find_follows = false) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->hc.err & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
    if (ctx->hc.err & 2u) return fail(ctx, MUMS_E_HIP, "sort look-back timed out (internal error)");
    if (ctx->hc.err & 16u) return fail(ctx, MUMS_E_HIP, "sort segment fix-up list overflow (internal error)");
    ctx->P = ctx->hc.nprobes;
    ctx->probe_info = ps.probe_info;
    HIPCHK(hipEventRecord(ctx->ev[EV_GROUPS], st));
    int tbits = 1;
    while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)ctx->table_size) ++tbits;
    const uint64_t P = ctx->P;
    if (find_follows && P > 0 && P <= find_chunk() && !ctx->shard && !getenv("MUMS_DEV_KEEP_BUCKET_ORDER")) {
        ctx->sorted_buckets = nullptr;
        ctx->sorted_ids = nullptr;
        HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
        return MUMS_OK;
    }
    // the onesweep variant (MUMS_DEV_BUCKET_ONESWEEP) moves packed 8-B records: 2.36 vs 1.56 ms
    // on C3's 1e8 probes (u32 keys and ids in the radix passes move fewer bytes)
    const bool radix = getenv("MUMS_DEV_BUCKET_ONESWEEP") == nullptr;
    // (the seed sort's scratch holds the onesweep workspace: ctx->tmp is not regrown here, other
    // stages may hold pointers into it)
    if (!radix && P >= 4096 && P < (1ull << 30) && ps.slot_info + P <= (const uint64_t*)ps.probe_bucket &&
        ctx->tmp.cap >= onesweep_tmp_bytes(P, 0, tbits)) {
        // one onesweep sort of packed (bucket << 32 | probe) records: the dead slot array and
        // [bucketB, idsA] are the ping-pong pair, the sorted partition lands in probe_bucket / idsB
        uint64_t* rA = ps.slot_info;
        uint64_t* rB = (uint64_t*)ps.bucketB;
        HIPCHK(ctx->bst2.ensure(64));
        HIPCHK(launch_bucket_records(ps.probe_bucket, P, rA, st));
        HIPCHK(seg_bucket_starts(nullptr, 0, 0, P, ctx->bst2.as<uint32_t>(), st));
        int ob = 0;
        HIPCHK(seg_onesweep_sort(rA, rB, P, tbits, 0, ctx->bst2.as<uint32_t>(), ctx->tmp.p, &dc->err, &ob, st));
        HIPCHK(launch_bucket_split(ob ? rB : rA, P, ps.probe_bucket, ps.idsB, st));
        ctx->sorted_buckets = ps.probe_bucket;
        ctx->sorted_ids = ps.idsB;
    } else {
        int pout = 0;
        HIPCHK(radix_sort<uint32_t>(ps.probe_bucket, nullptr, P, tbits, ps.bucketB, ps.idsA, ps.probe_bucket,
                                    ps.idsB, ctx->tmp.p, &pout, st));
        ctx->sorted_buckets = pout ? ps.probe_bucket : ps.bucketB;
        ctx->sorted_ids = pout ? ps.idsB : ps.idsA;
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
    return MUMS_OK;
}

// per-run statistics (mums_stats) of the last seed stage [+ replay] over n records
void fill_stats(mums_ctx* ctx, uint64_t n) {
    struct ClearLast {   // the elapsed times below ignore their status: leave no sticky error behind
        ~ClearLast() { (void)hipGetLastError(); }
    } clear_last;
    mums_stats& s = ctx->st;
    s = mums_stats{};
    s.seedmers = n;
    s.groups = ctx->hc.ngroups;
    s.probes = ctx->P;
    s.repeat_limit_groups = ctx->hc.repeat_limit;
    s.restarts = ctx->restarts;
    auto el = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
        return (double)ms;
    };
    const size_t kb = ctx->key64 ? 8 : 4;
    const int passes = ctx->sort_passes;
    s.ms_keys = el(EV_START, EV_KEYS);
    s.ms_sort = el(EV_KEYS, EV_SORT);
    s.ms_groups = el(EV_SORT, EV_GROUPS);
    s.ms_buckets = el(EV_GROUPS, EV_BUCKETS);
    s.key_bytes = ctx->packed_path ? 8 : kb;
    s.sort_passes = (uint64_t)passes;
    if (ctx->profiling && n > 0) {
        for (int p = 0; p < passes; ++p) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ctx->ev_ds[2 * p], ctx->ev_ds[2 * p + 1]);
            s.ms_dominant += ms;
            // algorithmic bytes of one sort-pass launch: packed records read + written
            // (8 + 8); pairs: read K (+4 after pass 0) and write K + 4
            s.dominant_bytes += ctx->packed_path ? n * 16 : n * (kb + (p ? 4 : 0) + kb + 4);
        }
        s.dominant_launches = (uint64_t)passes;
    }
    s.chunks = ctx->nchunks;
    if (ctx->stage_done >= MUMS_STAGE_ALL) {
        s.mem_count = ctx->pcompat ? ctx->M : ctx->hc.entries;   // compat: entries of the merged table
        s.collision_count = ctx->hc.collisions;
        s.ms_chains = el(EV_BUCKETS, EV_CHAINS);
        s.ms_replay = el(EV_CHAINS, EV_REPLAY);
        s.chains = ctx->hc.nchains;
        s.ms_output = el(EV_REPLAY, EV_OUTPUT);
        s.ms_total = el(EV_START, EV_OUTPUT);
        s.chain_walk_words = ctx->hc.walk_words;
        s.chain_walks = ctx->hc.walk_items;
        const uint64_t row_b = ctx->rows_narrow ? 4ull * line_row_stride(ctx->gt.G) : 8ull * (ctx->gt.G + 1);
        s.chain_walk_bytes = ctx->hc.walk_wins * 28 + ctx->hc.walk_items * (row_b + 24);
        s.short_walk_words = ctx->hc.short_words;
        s.short_walks = ctx->hc.short_items;
        s.short_walk_bytes = ctx->hc.short_wins * 28 + ctx->hc.short_items * (row_b + 24);
        if (ctx->walk_events && ctx->P > 0)
            for (int p = 0; p < 2; ++p) {
                float ms = 0.f, ms_s = 0.f;
                (void)hipEventElapsedTime(&ms_s, ctx->ev_walk[3 * p], ctx->ev_walk[3 * p + 1]);
                (void)hipEventElapsedTime(&ms, ctx->ev_walk[3 * p + 1], ctx->ev_walk[3 * p + 2]);
                s.ms_chain_walks += ms;
                s.ms_short_walks += ms_s;
            }
    } else {
        s.ms_total = el(EV_START, EV_BUCKETS);
    }
}

bool have_start_points(const mums_ctx* ctx) {
    for (uint64_t x : ctx->start_points)
        if (x) return true;
    return false;
}

// The std::sort order of equal seed mers (MemorySML::Create, MemorySML.cpp:54) for the runs
// that matter (smlsort.hip): every run (d_sp == nullptr) or the runs the start points d_sp
// (rows x G SML indices) fall into.  ck: genome-major sorted keys over the slot space (=
// global seed-mer indices); the keys in position order come from ckf (per stream record)
// scattered by the record's global index (rec: packed records, else idx).  On return *tw
// holds the ids at the flagged slots in std::sort order; *flagged = 0 when nothing matters.
int tie_order(mums_ctx* ctx, uint64_t n, const uint64_t* ck, const uint64_t* ckf, const uint64_t* rec,
              const uint32_t* idx, const uint64_t* const* d_sp, const uint64_t* rows, int nsp, TieWs* tw,
              uint64_t* flagged, hipStream_t st) {
    const GenomeTable& gt = ctx->gt;
    *flagged = 0;
    if (n >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList tie order above 2^32 seed-mers");
    HIPCHK(tiebuf_ensure(ctx, tie_ws_bytes(n, gt.G)));
    *tw = tie_ws_layout(ctx->tiebuf.p, n, gt.G);
    HIPCHK(tie_set_genomes(*tw, gt.base, gt.m, st));
    HIPCHK(tie_clear_flags(*tw, st));
    if (nsp == 0) HIPCHK(tie_mark_all(*tw, ck, st));
    for (int k = 0; k < nsp; ++k) HIPCHK(tie_mark_starts(*tw, ck, d_sp[k], rows[k], st));
    HIPCHK(tie_prepare(*tw, flagged, st));
    if (*flagged == 0) return MUMS_OK;
    HIPCHK(tie_scatter_keys(*tw, ckf, rec, idx, st));
    HIPCHK(tie_replay(*tw, st));
    ctx->tie_slots += *flagged;
    return MUMS_OK;
}

// Every run of equal keys of the merged stream s (n records) in std::sort order: repeat /
// enumeration tolerance hash the first copies of a genome in SML order (MemHash.cpp:139-162,
// MatchFinder.cpp:342-393).  Rewrites the ids of the stream in place.
int tie_fix_stream(mums_ctx* ctx, const RsStream& s, uint64_t n, hipStream_t st) {
    HIPCHK(ctx->rsbuf.ensure(restart_ws_bytes(n, ctx->gt.G)));
    const RestartWs w = restart_ws_layout(ctx->rsbuf.p, n, ctx->gt.G);
    HIPCHK(launch_restart_smls(s, n, ctx->gt, w, st));
    TieWs tw{};
    uint64_t flagged = 0;
    int rc = tie_order(ctx, n, w.ck, w.ckf, s.kind == 0 ? s.rec : nullptr, s.kind == 0 ? nullptr : s.idx, nullptr,
                       nullptr, 0, &tw, &flagged, st);
    if (rc) return rc;
    if (flagged)
        HIPCHK(tie_writeback(tw, s.kind == 0 ? const_cast<uint64_t*>(s.rec) : nullptr,
                             s.kind == 0 ? nullptr : const_cast<uint32_t*>(s.idx), w.inv, st));
    ctx->ties_fixed = true;
    return MUMS_OK;
}

// repeat / enumeration tolerance see the order of a genome's copies (PairwiseMatchFinder
// hashes single-copy genomes only)
bool wants_tie_order(const mums_ctx* ctx) { return !ctx->pairwise && (ctx->repeat_tol > 0 || ctx->enum_tol > 1); }

int progress_packed(mums_ctx* ctx, const uint64_t* rec, const uint32_t* bstart, int B, uint64_t n, hipStream_t st,
                    const RestartWs* pw = nullptr, uint64_t* ck_build = nullptr);
int progress_pairs(mums_ctx* ctx, const RestartWs* pw, hipStream_t st);
// the pair path's (key, index) stream without a restart: its SMLs built for LogProgress
int progress_pair_stream(mums_ctx* ctx, const RsStream& s, uint64_t n, hipStream_t st);

// MER_REPEAT_LIMIT restart (MatchFinder.cpp:253-277) and FindMatchSeeds start points
// (MemHash.cpp:117-127) on the merged stream s of n records (restart.hip): plan the
// restarts, then compact the live records in order into dst (records / keys + dst_idx;
// packed records also get their new bucket starts in dst_bstart).  *n_live = kept
// records; *changed = false when every record lives (the groups already stand).
int restart_fixup(mums_ctx* ctx, const RsStream& s, uint64_t n, void* dst_a, uint32_t* dst_idx, uint32_t* dst_bstart,
                  uint64_t* n_live, bool* changed, hipStream_t st) {
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    *changed = false;
    *n_live = n;
    ctx->restarts = 0;
    ctx->offset_log.clear();
    if (n >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "MER_REPEAT_LIMIT restart above 2^32 records");
    std::vector<uint64_t> S0(G, 0);
    for (int g = 0; g < G && g < (int)ctx->start_points.size(); ++g) S0[g] = ctx->start_points[g];
    HIPCHK(ctx->rsbuf.ensure(restart_ws_bytes(n, G)));
    const RestartWs w = restart_ws_layout(ctx->rsbuf.p, n, G);
    HIPCHK(launch_restart_smls(s, n, gt, w, st));
    // candidates: one per group above MER_REPEAT_LIMIT (counted by the groups stage)
    const uint64_t cap = ctx->hc.repeat_limit + 16;
    const uint64_t Gu = (uint64_t)G;
    const size_t plan_words = cap + 1 + 3 * cap * Gu + (cap + 1) / 2 + 2 * Gu + 16 + cap + 2 * cap * Gu;
    HIPCHK(ctx->rsplan.ensure(plan_words * 8 + sizeof(restart::PlanOut) + 256));
    uint64_t* d_list = ctx->rsplan.as<uint64_t>();
    unsigned long long* d_cnt = (unsigned long long*)(d_list + cap);
    uint64_t* d_pre = d_list + cap + 1;
    uint64_t* d_S = d_pre + 3 * cap * Gu + (cap + 1) / 2;
    uint64_t* d_S0 = d_S + Gu;
    restart::PlanOut* d_out = (restart::PlanOut*)(d_S0 + Gu);
    uint64_t* d_rkey = d_S0 + Gu + 16;
    uint64_t* d_rS = d_rkey + cap;
    uint64_t* d_rC = d_rS + cap * Gu;
    HIPCHK(launch_restart_cands(w, n, d_list, d_cnt, cap, st));
    unsigned long long C = 0;
    HIPCHK(hipMemcpyAsync(&C, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (C > cap) return fail(ctx, MUMS_E_HIP, "restart candidates exceed the groups stage's count (internal error)");
    std::vector<uint64_t> cand(C);
    if (C) {
        HIPCHK(hipMemcpy(cand.data(), d_list, C * 8, hipMemcpyDeviceToHost));
        std::sort(cand.begin(), cand.end());
        HIPCHK(hipMemcpyAsync(d_list, cand.data(), C * 8, hipMemcpyHostToDevice, st));
    }
    HIPCHK(hipMemcpyAsync(d_S, S0.data(), Gu * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_S0, S0.data(), Gu * 8, hipMemcpyHostToDevice, st));
    restart::PlanOut po{};
    po.cap = C;
    po.rkey = d_rkey;
    po.rS = d_rS;
    po.rC = d_rC;
    po.status = restart::kPlanOk;
    HIPCHK(hipMemcpyAsync(d_out, &po, sizeof(po), hipMemcpyHostToDevice, st));
    HIPCHK(launch_restart_plan(w, G, d_list, C, d_pre, d_S, d_out, st));
    HIPCHK(hipMemcpyAsync(&po, d_out, sizeof(po), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (po.status != restart::kPlanOk) return fail(ctx, MUMS_E_HIP, "restart plan table full (internal error)");
    ctx->restarts = po.nrestarts;
    ctx->offset_log.assign(po.nrestarts * Gu, 0);
    if (po.nrestarts) HIPCHK(hipMemcpy(ctx->offset_log.data(), d_rS, po.nrestarts * Gu * 8, hipMemcpyDeviceToHost));
    ctx->consumed_log.assign(po.nrestarts * Gu, 0);
    if (po.nrestarts) HIPCHK(hipMemcpy(ctx->consumed_log.data(), d_rC, po.nrestarts * Gu * 8, hipMemcpyDeviceToHost));
    if (ctx->progress_on) {   // the stream is still whole here (compaction below)
        const int rc = s.kind == 0 ? progress_packed(ctx, s.rec, s.bstart, s.B, n, st, &w) : progress_pairs(ctx, &w, st);
        if (rc) return rc;
    }
    if (po.nrestarts == 0 && !have_start_points(ctx)) return MUMS_OK;
    if (!ctx->ties_fixed) {
        // a start point inside a run of equal keys: which copies live depends on the SML's
        // std::sort order of that run (GetBreakpoint's FindMer + 1, MatchFinder.cpp:113-121)
        const uint64_t* sps[2] = {d_S0, d_rS};
        const uint64_t rws[2] = {1, po.nrestarts};
        TieWs tw{};
        uint64_t flagged = 0;
        int rc = tie_order(ctx, n, w.ck, w.ckf, s.kind == 0 ? s.rec : nullptr, s.kind == 0 ? nullptr : s.idx, sps,
                           rws, 2, &tw, &flagged, st);
        if (rc) return rc;
        if (flagged)
            HIPCHK(tie_writeback(tw, s.kind == 0 ? const_cast<uint64_t*>(s.rec) : nullptr,
                                 s.kind == 0 ? nullptr : const_cast<uint32_t*>(s.idx), w.inv, st));
    }
    uint32_t* d_total = (uint32_t*)d_cnt;
    HIPCHK(launch_restart_compact(s, n, G, w, d_rkey, po.nrestarts, d_rS, d_S0, dst_a, dst_idx, dst_bstart, d_total,
                                  st));
    uint32_t tot = 0;
    HIPCHK(hipMemcpyAsync(&tot, d_total, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *n_live = tot;
    *changed = true;
    return MUMS_OK;
}

// run_pipeline's restart stage: after the groups stage saw a group above MER_REPEAT_LIMIT
// (or with start points), fix the stream up and run the groups stage again on it.
int restart_stage(mums_ctx* ctx, const MatchParams& mp, const ProbeSpace& ps, hipStream_t st) {
    ctx->progress.clear();
    ctx->consumed_log.clear();
    if (!ctx->hc.repeat_limit && !have_start_points(ctx)) {
        ctx->restarts = 0;
        if (ctx->progress_on && ctx->packed_path)
            return progress_packed(ctx, ctx->sorted_rec, ctx->mstart.as<uint32_t>(), ctx->msd_bits, ctx->N, st, nullptr,
                                   ctx->sorted_buf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>());
        if (ctx->progress_on) {   // the pair path (seed weight > 21)
            RsStream ps{};
            ps.kind = ctx->key64 ? 2 : 1;
            ps.key = ctx->sorted_key;
            ps.idx = ctx->sorted_idx;
            return progress_pair_stream(ctx, ps, ctx->N, st);
        }
        return MUMS_OK;
    }
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t rep = ctx->hc.repeat_limit;
    const uint64_t N = ctx->N;
    RsStream s{};
    uint64_t nl = N;
    bool changed = false;
    int rc;
    if (ctx->packed_path) {
        const int B = ctx->msd_bits;
        s.kind = 0;
        s.rec = ctx->sorted_rec;
        s.bstart = ctx->mstart.as<uint32_t>();
        s.B = B;
        s.kbits = 2 * ctx->w + 1;
        uint64_t* dst = ctx->sorted_buf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>();
        if (ctx->parity_masked) {   // the restart replays SearchRange over the exact SML order
            HIPCHK(seg_parity_fix(const_cast<uint64_t*>(ctx->sorted_rec), dst, N, s.kbits - B, B, ctx->mstart.as<uint32_t>(), ctx->tmp.p,
                                  &dc->err, st));
            ctx->parity_masked = false;
        }
        HIPCHK(ctx->rsbst.ensure(((1ull << B) + 64) * 4));
        rc = restart_fixup(ctx, s, N, dst, nullptr, ctx->rsbst.as<uint32_t>(), &nl, &changed, st);
        if (rc || !changed) return rc;
        HIPCHK(hipMemcpyAsync(ctx->mstart.p, ctx->rsbst.p, ((1ull << B) + 1) * 4, hipMemcpyDeviceToDevice, st));
        ctx->sorted_buf ^= 1;
        ctx->sorted_rec = dst;
        SegTile* tiles = ctx->tiles.as<SegTile>();
        HIPCHK(build_seg_tiles_from_starts(ctx->mstart.as<uint32_t>(), B, nl, tiles, &dc->ntiles, ctx->tmp.p, st));
        HIPCHK(hipMemsetAsync(&dc->repeat_limit, 0, 8, st));
        rc = groups_dispatch<RecView>(ctx, RecView{dst}, tiles, seg_tiles_upper(nl, B), mp, ps.probe_info,
                                      ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
    } else {
        const size_t kb = ctx->key64 ? 8 : 4;
        (void)kb;
        s.kind = ctx->key64 ? 2 : 1;
        s.key = ctx->sorted_key;
        s.idx = ctx->sorted_idx;
        void* dk = ctx->sorted_buf ? ctx->kA.p : ctx->kB.p;
        uint32_t* dv = ctx->sorted_buf ? ctx->vA.as<uint32_t>() : ctx->vB.as<uint32_t>();
        rc = restart_fixup(ctx, s, N, dk, dv, nullptr, &nl, &changed, st);
        if (rc || !changed) return rc;
        ctx->sorted_buf ^= 1;
        ctx->sorted_key = dk;
        ctx->sorted_idx = dv;
        SegTile* tiles = ctx->tiles.as<SegTile>();
        const uint64_t nt = (nl + kSegTile - 1) / kSegTile;
        HIPCHK(launch_flat_tiles(nl, tiles, st));
        HIPCHK(hipMemsetAsync(&dc->repeat_limit, 0, 8, st));
        if (ctx->key64)
            rc = groups_dispatch<PairView<uint64_t>>(ctx, PairView<uint64_t>{(const uint64_t*)dk, dv}, tiles, nt, mp,
                                                     ps.probe_info, ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
        else
            rc = groups_dispatch<PairView<uint32_t>>(ctx, PairView<uint32_t>{(const uint32_t*)dk, dv}, tiles, nt, mp,
                                                     ps.probe_info, ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
    }
    if (rc) return rc;
    rc = finish_seeds(ctx, ps, st);
    if (rc) return rc;
    // the report counts the groups above MER_REPEAT_LIMIT of the whole stream
    HIPCHK(h2d_sync(&dc->repeat_limit, &rep, 8, ctx->stream));
    ctx->hc.repeat_limit = rep;
    return MUMS_OK;
}

// keys -> sorted stream -> probes -> bucket-sorted probes [-> replay -> MatchList]
int run_pipeline(mums_ctx* ctx, int stage) {
    hipStream_t st = ctx->stream;
    const int G = (int)ctx->genomes.size();
    const uint64_t N = ctx->N;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    GenomeTable& gt = ctx->gt;

    uint64_t words = 0;
    const uint32_t T = layout_packed(gt, &words);
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const SeedSpec& ss = ctx->ss;

    const int kbits = 2 * ctx->w + 1;
    ctx->packed_path = kbits <= 32 + kMaxMsdBits;
    ctx->msd_bits = ctx->packed_path ? std::max(0, kbits - 32) : 0;
    if (const char* e = getenv("MUMS_DEV_MSD_BITS"))   // development knob (sort layout experiments)
        if (ctx->packed_path) ctx->msd_bits = std::min(kMaxMsdBits, std::max(ctx->msd_bits, atoi(e)));
    // the three-pass sort (MUMS_DEV_SORT3) sorts 30 bits: the 8-bit MSD scatter leaves 31 key
    // bits in a w19 record, the parity bit stays unsorted (default tolerances only)
    if (ctx->packed_path && seg_wide_sort_enabled() && ctx->msd_bits < 8 && kbits - 8 <= 31 && kbits > 8 &&
        ctx->repeat_tol == 0 && ctx->enum_tol == 1)
        ctx->msd_bits = 8;
    const int B = ctx->msd_bits;
    // keys wider than 32 + 8 bits: an 8-bit scatter + side bytes + msd_split (msdsplit.hip)
    // instead of a 2^B-digit scatter (write runs of ~2 records per tile at w21)
    const int side = (ctx->packed_path && B > 8 && !getenv("MUMS_DEV_MSD_BITS") && !getenv("MUMS_DEV_NO_SPLIT"))
                         ? B - 8 : 0;
    const size_t kb = ctx->key64 ? 8 : 4;
    ProbeSpace ps{};
    if (ctx->packed_path) {
        HIPCHK(ctx->hist.ensure(((uint64_t)T << B) * 4 + 64));
        HIPCHK(ctx->tmp.ensure(scan_tmp_bytes((uint64_t)T << B)));
        int rc0 = ensure_merge_space(ctx, N, B, kbits - B, &ps);
        if (rc0) return rc0;
        HIPCHK(ctx->tmp.ensure(std::max(scan_tmp_bytes((uint64_t)T << B), ctx->tmp.cap)));
    } else {
        const uint64_t ntiles_groups = (N + kSegTile - 1) / kSegTile;
        HIPCHK(ctx->ckey.ensure(N * kb + 64));
        HIPCHK(ctx->kA.ensure(N * kb + 64));
        HIPCHK(ctx->kB.ensure(N * kb + 64));
        HIPCHK(ctx->vA.ensure(N * 4 + 64));
        HIPCHK(ctx->vB.ensure(N * 4 + 64));
        HIPCHK(ctx->tiles.ensure(ntiles_groups * sizeof(SegTile) + 64));
        size_t tmpb = std::max(scan_tmp_bytes(N), radix_tmp_bytes(N));
        tmpb = std::max(tmpb, scan_tmp_bytes((uint64_t)ctx->table_size));
        HIPCHK(ctx->tmp.ensure(tmpb));
        int rc0 = ensure_probe_space(ctx, N, ntiles_groups, &ps);
        if (rc0) return rc0;
    }

    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    const bool prof = ctx->profiling;
    if (prof && !ctx->ev_ds[0])
        for (int i = 0; i < 16; ++i) HIPCHK(hipEventCreate(&ctx->ev_ds[i]));

    int rc = MUMS_OK;
    if (ctx->packed_path) {
        rc = keys_stage(ctx, gt, T, B, N, ctx->recA.as<uint64_t>(), ctx->mstart.as<uint32_t>(), st, 32, side);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        rc = merge_stage(ctx, N, B, kbits - B, mp, ps, st);
    } else {
        std::vector<const char*> ptrs(G);
        for (int g = 0; g < G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
        HIPCHK(launch_seed_pack(ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 0, ctx->key64, ctx->ckey.p, 0,
                                nullptr, T, &dc->err, st));
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        int buf = 0;
        SegTile* tiles = ctx->tiles.as<SegTile>();
        const uint64_t ntiles_groups = (N + kSegTile - 1) / kSegTile;
        HIPCHK(launch_flat_tiles(N, tiles, st));
        if (ctx->key64) {
            HIPCHK(radix_sort<uint64_t>(ctx->ckey.as<uint64_t>(), nullptr, N, kbits, ctx->kA.as<uint64_t>(),
                                        ctx->vA.as<uint32_t>(), ctx->kB.as<uint64_t>(), ctx->vB.as<uint32_t>(),
                                        ctx->tmp.p, &buf, st, prof ? ctx->ev_ds : nullptr));
        } else {
            HIPCHK(radix_sort<uint32_t>(ctx->ckey.as<uint32_t>(), nullptr, N, kbits, ctx->kA.as<uint32_t>(),
                                        ctx->vA.as<uint32_t>(), ctx->kB.as<uint32_t>(), ctx->vB.as<uint32_t>(),
                                        ctx->tmp.p, &buf, st, prof ? ctx->ev_ds : nullptr));
        }
        ctx->sorted_buf = buf;
        ctx->sorted_key = buf ? ctx->kB.p : ctx->kA.p;
        ctx->sorted_idx = buf ? ctx->vB.as<uint32_t>() : ctx->vA.as<uint32_t>();
        ctx->sort_passes = (kbits + 7) / 8;
        HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
        if (wants_tie_order(ctx)) {
            RsStream s{};
            s.kind = ctx->key64 ? 2 : 1;
            s.key = ctx->sorted_key;
            s.idx = ctx->sorted_idx;
            rc = tie_fix_stream(ctx, s, N, st);
            if (rc) return rc;
        }
        if (ctx->key64)
            rc = groups_dispatch<PairView<uint64_t>>(ctx, PairView<uint64_t>{(const uint64_t*)ctx->sorted_key,
                                                                             ctx->sorted_idx},
                                                     tiles, ntiles_groups, mp, ps.probe_info, ps.probe_bucket,
                                                     ps.slot_info, ps.slot_bucket, st);
        else
            rc = groups_dispatch<PairView<uint32_t>>(ctx, PairView<uint32_t>{(const uint32_t*)ctx->sorted_key,
                                                                             ctx->sorted_idx},
                                                     tiles, ntiles_groups, mp, ps.probe_info, ps.probe_bucket,
                                                     ps.slot_info, ps.slot_bucket, st);
    }
    if (rc) return rc;
    rc = finish_seeds(ctx, ps, st, stage >= MUMS_STAGE_ALL);
    if (rc) return rc;
    rc = restart_stage(ctx, mp, ps, st);
    if (rc) return rc;
    ctx->stage_done = MUMS_STAGE_SEEDS;

    if (stage >= MUMS_STAGE_ALL) {
        rc = find_tail(ctx, mp, ctx->packed.as<uint32_t>(), [&](MatProbes* v) {
            const int r = materialize_seeds(ctx, mp, st);
            v->rows = ctx->mprobe.as<int64_t>();
            return r;
        }, st, true);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));

    fill_stats(ctx, N);
    return MUMS_OK;
}

// Seed pattern (default from the mean genome length, MatchList.h:351-357; checks of
// SortedMerList::Create :788-798) and the global genome table for genome lengths lens.
int prepare_run(mums_ctx* ctx, const std::vector<uint64_t>& lens) {
    records_live(ctx);
    ctx->stage_done = 0;
    ctx->compat_rec = false;
    ctx->ties_fixed = false;
    ctx->tie_slots = 0;
    ctx->restarts = 0;
    ctx->offset_log.clear();
    ctx->log_host = false;
    ctx->M = ctx->P = 0;
    const int G = (int)lens.size();
    uint64_t total = 0;
    for (uint64_t n : lens) total += n;
    uint64_t pat = ctx->seed;
    if (pat == 0) {
        uint32_t wdef = mums_default_seed_weight(G ? total / (uint64_t)G : 0);
        pat = (uint64_t)mums_get_seed((int)wdef, 0);
    }
    const int L = seed_len(pat), w = __builtin_popcountll(pat);
    if (L == 0) return fail(ctx, MUMS_E_INVALID, "Can't have 0 seed length");
    if (L > 32) return fail(ctx, MUMS_E_INVALID, "Mer size is too large");
    if (w > 31) return fail(ctx, MUMS_E_UNSUPPORTED, "seed weight 32 not supported");
    ctx->pattern = pat;
    ctx->L = L;
    ctx->w = w;
    ctx->key64 = (2 * w + 1) > 32;
    GenomeTable& gt = ctx->gt;
    gt = GenomeTable{};
    gt.G = G;
    uint64_t N = 0;
    for (int g = 0; g < G; ++g) {
        gt.n[g] = lens[g];
        gt.m[g] = gt.n[g] < (uint64_t)L ? 0 : gt.n[g] - L + 1;
        gt.base[g] = N;
        N += gt.m[g];
    }
    gt.base[G] = N;
    for (int g = G + 1; g <= kMaxG; ++g) gt.base[g] = N;
    genome_lookup_init(gt);
    if (N >= (1ull << 33))
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^33 seed-mers per context");
    ctx->N = N;
    ctx->ss = make_seed_spec(pat, L, w);
    return MUMS_OK;
}

// ParallelMemHash::FindMatches (ParallelMemHash.cpp:42-103) compat pipeline (compat.hip):
// pair path; one sort of (genome, ckey) gives the G SortedMerLists, the chunk starts
// follow GetBreakpoint, and a second sort of (chunk, ckey) yields the chunk-major probe
// order; groups / probes / chains / replay are the serial kernels, then MergeTable.
// ParallelMemHash chunks with a seed group above MER_REPEAT_LIMIT (ParallelMemHash.cpp:97-100):
// the chunk's SearchRange returns false at the group (MatchFinder.cpp:253-277), the return
// value is ignored and MergeTable still runs, so the chunk keeps exactly the AddHashEntry
// calls before that group and the later chunks are unaffected.  On the chunk-major stream
// (sorted_key / sorted_idx, N records) every (chunk, masked key) group of more than 1000
// records is a candidate; compat_fire_kernel decides per candidate whether the check fires
// inside its chunk (restart_plan.h head order, buffers from the chunk start); the first
// firing group of a chunk drops the stream from its first record to the chunk's end.
// ctx->crall holds the genome-major SML keys.  *n_live = records kept.
int progress_compat(mums_ctx* ctx, uint32_t nch, const std::vector<uint64_t>& hcs, hipStream_t st);

// ctx->crall (the genome-major SML keys without the genome bits) on first use: the packed
// path's partition leaves it out unless the tie replay or the MER_REPEAT_LIMIT plan needs it
int compat_ck_ready(mums_ctx* ctx, hipStream_t st) {
    if (!ctx->compat_ck_src) return MUMS_OK;
    HIPCHK(launch_compat_strip(ctx->compat_ck_src, ctx->crall.as<uint64_t>(), ctx->N, ctx->compat_ck_mask, st));
    ctx->compat_ck_src = nullptr;
    return MUMS_OK;
}

// the candidate list of compat_truncate in ctx->rsplan: list (cap words) and its counter
int compat_cand_slots(mums_ctx* ctx, uint32_t nch, uint64_t** list, unsigned long long** cnt, uint64_t* cap_out) {
    const int G = ctx->gt.G;
    const uint64_t cap = ctx->N / (restart::kRepeatLimit + 1) + 16;
    const uint64_t words = cap * (4 + (uint64_t)G) + 2 * (uint64_t)(G + 1) + 16 + 3 * ((uint64_t)nch + 1);
    HIPCHK(ctx->rsplan.ensure(words * 8 + 256));
    *list = ctx->rsplan.as<uint64_t>();
    *cnt = (unsigned long long*)(*list + 3 * cap + 2 * (uint64_t)(G + 1));
    *cap_out = cap;
    return MUMS_OK;
}

// cands_ready: the candidates were collected with the packed records (launch_compat_recs)
int compat_truncate(mums_ctx* ctx, uint32_t nch, const uint64_t* cs, int kbits, uint64_t* n_live, hipStream_t st,
                    bool cands_ready = false) {
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t N = ctx->N;
    *n_live = N;
    ctx->restarts = 0;
    uint64_t* d_list = nullptr;
    unsigned long long* d_cnt = nullptr;
    uint64_t cap = 0;
    int rc0 = compat_cand_slots(ctx, nch, &d_list, &d_cnt, &cap);
    if (rc0) return rc0;
    uint64_t* d_cend = d_list + cap;
    uint32_t* d_fire = (uint32_t*)(d_cend + cap);
    uint64_t* d_dm = d_list + 3 * cap;   // (d_fire takes cap/2 words of that third block)
    uint64_t* d_db = d_dm + G + 1;
    uint64_t* d_rng = d_db + G + 1 + 16;
    uint64_t* d_cons = d_rng + 3 * ((uint64_t)nch + 1);   // cap x (G + 1)
    ctx->compat_cons.clear();
    const uint64_t* key2 = (const uint64_t*)ctx->sorted_key;
    if (!cands_ready) HIPCHK(launch_compat_cands(key2, N, d_list, d_cnt, cap, st));
    unsigned long long C = 0;
    HIPCHK(hipMemcpyAsync(&C, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (C > cap) return fail(ctx, MUMS_E_HIP, "compat: candidate list overflow (internal error)");
    if (C == 0) return MUMS_OK;
    std::vector<uint64_t> cand(C);
    HIPCHK(hipMemcpy(cand.data(), d_list, C * 8, hipMemcpyDeviceToHost));
    std::sort(cand.begin(), cand.end());
    std::vector<uint64_t> hm(G + 1, 0), hb(G + 1, 0);
    for (int g = 0; g < G; ++g) { hm[g] = gt.m[g]; hb[g] = gt.base[g]; }
    HIPCHK(hipMemcpyAsync(d_list, cand.data(), C * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_dm, hm.data(), (G + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_db, hb.data(), (G + 1) * 8, hipMemcpyHostToDevice, st));
    if ((rc0 = compat_ck_ready(ctx, st))) return rc0;
    const restart::PlanData d{G, d_dm, d_db, ctx->crall.as<uint64_t>()};
    HIPCHK(launch_compat_fire(d, key2, N, kbits, d_list, C, cs, nch, d_fire, d_cend, d_cons, st));
    std::vector<uint32_t> fire(C);
    std::vector<uint64_t> cend(C), cons(C * (uint64_t)(G + 1));
    HIPCHK(hipMemcpyAsync(fire.data(), d_fire, C * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(cend.data(), d_cend, C * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(cons.data(), d_cons, cons.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    // candidates are in stream order = (chunk, key) order: the first firing one of a chunk cuts it
    std::vector<uint64_t> rlo, rhi, rpre;
    uint64_t dropped = 0;
    for (uint64_t c = 0; c < C; ++c) {
        if (!fire[c] || (!rhi.empty() && cand[c] < rhi.back())) continue;   // chunk already cut
        if (ctx->compat_cons.empty()) ctx->compat_cons.assign((uint64_t)nch * G, ~0ull);
        const uint64_t* cz = &cons[c * (uint64_t)(G + 1)];
        std::copy(cz, cz + G, ctx->compat_cons.begin() + cz[G] * (uint64_t)G);   // the cut chunk's consumption
        rlo.push_back(cand[c]);
        rhi.push_back(cend[c]);
        rpre.push_back(dropped);
        dropped += cend[c] - cand[c];
    }
    ctx->restarts = rlo.size();
    if (rlo.empty()) return MUMS_OK;
    const uint32_t R = (uint32_t)rlo.size();
    uint64_t* d_rlo = d_rng;
    uint64_t* d_rhi = d_rlo + R;
    uint64_t* d_rpre = d_rhi + R;
    HIPCHK(hipMemcpyAsync(d_rlo, rlo.data(), R * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_rhi, rhi.data(), R * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_rpre, rpre.data(), R * 8, hipMemcpyHostToDevice, st));
    uint64_t* k_out = ctx->sorted_buf ? ctx->kA.as<uint64_t>() : ctx->kB.as<uint64_t>();
    uint32_t* v_out = ctx->sorted_buf ? ctx->vA.as<uint32_t>() : ctx->vB.as<uint32_t>();
    HIPCHK(launch_compat_drop(key2, ctx->sorted_idx, N, d_rlo, d_rhi, d_rpre, R, k_out, v_out, st));
    HIPCHK(hipStreamSynchronize(st));   // (rlo / rhi / rpre are host temporaries)
    ctx->sorted_buf ^= 1;
    ctx->sorted_key = k_out;
    ctx->sorted_idx = v_out;
    *n_live = N - dropped;
    return MUMS_OK;
}

// compat over ranks: keep only this rank's chunks [nch * r / R, nch * (r + 1) / R) of the live
// chunk-major stream (the oracle's rank model, oracle/mums_oracle.c parallel_compat_search):
// its search then starts from empty tables at its first chunk.  The MER_REPEAT_LIMIT cuts were
// decided per chunk before (compat_truncate), so they are unchanged.
int compat_keep_chunks(mums_ctx* ctx, uint32_t nch, int kbits, uint64_t* n_live, hipStream_t st) {
    const uint32_t c0 = (uint32_t)((uint64_t)nch * ctx->compat_rank / ctx->compat_ranks);
    const uint32_t c1 = (uint32_t)((uint64_t)nch * (ctx->compat_rank + 1) / ctx->compat_ranks);
    const uint64_t n = *n_live;
    const uint64_t* key2 = (const uint64_t*)ctx->sorted_key;
    uint64_t* d_rng = nullptr;
    {
        uint64_t* d_list = nullptr;
        unsigned long long* d_cnt = nullptr;
        uint64_t cap = 0;
        int rc = compat_cand_slots(ctx, nch, &d_list, &d_cnt, &cap);
        if (rc) return rc;
        d_rng = (uint64_t*)(d_cnt + 2);   // 8 words behind the candidate counter
    }
    HIPCHK(launch_compat_chunk_span(key2, n, kbits, c0, c1, d_rng, st));
    uint64_t span[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(span, d_rng, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (span[0] == 0 && span[1] == n) return MUMS_OK;
    const uint64_t rng[6] = {0, span[1], span[0], n, 0, span[0]};   // rlo[2], rhi[2], rpre[2]
    HIPCHK(hipMemcpyAsync(d_rng + 2, rng, sizeof(rng), hipMemcpyHostToDevice, st));
    uint64_t* k_out = ctx->sorted_buf ? ctx->kA.as<uint64_t>() : ctx->kB.as<uint64_t>();
    uint32_t* v_out = ctx->sorted_buf ? ctx->vA.as<uint32_t>() : ctx->vB.as<uint32_t>();
    HIPCHK(launch_compat_drop(key2, ctx->sorted_idx, n, d_rng + 2, d_rng + 4, d_rng + 6, 2, k_out, v_out, st));
    HIPCHK(hipStreamSynchronize(st));   // (rng is a host temporary)
    ctx->sorted_buf ^= 1;
    ctx->sorted_key = k_out;
    ctx->sorted_idx = v_out;
    *n_live = span[1] - span[0];
    return MUMS_OK;
}

int run_pipeline_compat(mums_ctx* ctx, int stage) {
    hipStream_t st = ctx->stream;
    const int G = (int)ctx->genomes.size();
    const uint64_t N = ctx->N;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    GenomeTable& gt = ctx->gt;
    const int kbits = 2 * ctx->w + 1;
    int gbits = 0;
    while ((1 << gbits) < G) ++gbits;
    if (kbits + gbits > 63) return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: seed weight too large");
    ctx->packed_path = false;
    ctx->key64 = true;
    ctx->msd_bits = 0;
    ctx->progress.clear();
    const uint64_t kmask = (1ull << kbits) - 1;

    uint64_t words = 0;
    const uint32_t T = layout_packed(gt, &words);
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t ntiles_groups = (N + kSegTile - 1) / kSegTile;
    HIPCHK(ctx->ckey.ensure(N * 8 + 64));
    HIPCHK(ctx->kA.ensure(N * 8 + 64));
    HIPCHK(ctx->kB.ensure(N * 8 + 64));
    HIPCHK(ctx->vA.ensure(N * 4 + 64));
    HIPCHK(ctx->vB.ensure(N * 4 + 64));
    HIPCHK(ctx->cval.ensure(N * 4 + 64));
    HIPCHK(ctx->tiles.ensure(ntiles_groups * sizeof(SegTile) + 64));
    size_t tmpb = std::max(scan_tmp_bytes(N), radix_tmp_bytes(N));
    tmpb = std::max(tmpb, scan_tmp_bytes((uint64_t)ctx->table_size));
    HIPCHK(ctx->tmp.ensure(tmpb));
    ProbeSpace ps{};
    int rc = ensure_probe_space(ctx, N, ntiles_groups, &ps);
    if (rc) return rc;

    int mx = -1;   // the longest SML by Length() = sequence length (ParallelMemHash.cpp:64-73)
    uint64_t maxlen = 0;
    for (int g = 0; g < G; ++g)
        if (gt.n[g] > maxlen) { maxlen = gt.n[g]; mx = g; }
    const uint64_t chunk = ctx->chunk_size;
    const uint32_t cap = (uint32_t)std::min<uint64_t>(2 * (maxlen / chunk) + 4, 1u << 24);
    HIPCHK(ctx->ctab.ensure((size_t)cap * (G + 1) * 8 + 64));
    uint64_t* cs = ctx->ctab.as<uint64_t>();
    uint64_t* bm = cs + (size_t)cap * G;
    uint32_t* d_nch = (uint32_t*)(bm + cap);

    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    HIPCHK(hipMemsetAsync(cs, 0, (size_t)cap * G * 8, st));
    int buf = 0;
    const uint64_t* sk = nullptr;
    const uint32_t* sv = nullptr;
    // the G SortedMerLists, genome-major: from the MemHash path's packed records (scatter into
    // 2^B MSD buckets + onesweep passes, then a stable partition by genome) where they fit,
    // else one 64-bit (genome, ckey) radix sort.  MUMS_DEV_COMPAT_RADIX (read per call): the
    // radix sort always.
    const int B = std::max(0, kbits - 32);
    const bool packed_sml = B <= 7 && N > 0 && N < (1ull << 30) && !getenv("MUMS_DEV_COMPAT_RADIX");
    const bool all_ties = wants_tie_order(ctx);
    ctx->compat_ck_src = nullptr;
    DevBuf dst;            // the sorted stream's bucket starts (packed_sml)
    CrStream pstream{};    // the sorted stream (packed_sml): also the source of the chunk-major order
    // lean: the chunk starts and the chunk-major records come from the sorted stream alone
    // (compat_fast_chunks, cr_compat_direct) where no later step reads the SMLs or key2 arrays;
    // the genome-major SMLs are built only when one of them declines.  MUMS_DEV_COMPAT_SML /
    // MUMS_DEV_COMPAT_PART (read per call): the SML chunking / the partition path always.
    const bool lean = packed_sml && !all_ties && N < (1ull << 32) && ctx->compat_ranks <= 1 && !ctx->match_log &&
                      !ctx->progress_on && !getenv("MUMS_DEV_COMPAT_PAIRS") && !getenv("MUMS_DEV_COMPAT_GID_SCAN") &&
                      !getenv("MUMS_DEV_COMPAT_PART");
    bool have_sml = !packed_sml, sml_idx = !packed_sml;   // genome-major keys (kA) / indices (vA) written
    auto build_sml = [&](bool idx) -> hipError_t {   // from the sorted stream (packed_sml)
        hipError_t e = launch_cr_partition(pstream, gt, ctx->crcnt.as<uint32_t>(), kbits, ctx->kA.as<uint64_t>(),
                                           idx ? ctx->vA.as<uint32_t>() : nullptr, nullptr, st);
        have_sml = true;
        sml_idx = sml_idx || idx;
        ctx->compat_ck_src = ctx->kA.as<uint64_t>();
        ctx->compat_ck_mask = kmask;
        return e;
    };
    HIPCHK(ctx->crall.ensure(N * 8 + 64));
    if (packed_sml) {
        HIPCHK(ctx->hist.ensure(((uint64_t)T << B) * 4 + 64));
        HIPCHK(ctx->recA.ensure(N * 8 + 64));
        HIPCHK(ctx->recB.ensure(N * 8 + 64));
        HIPCHK(ctx->mstart.ensure(((1ull << B) + 64) * 4));
        const uint64_t nblk = cr_blocks(N);
        HIPCHK(ctx->tmp.ensure(std::max({ctx->tmp.cap, onesweep_tmp_bytes(N, B, kbits - B),
                                         scan_tmp_bytes((uint64_t)T << B), scan_tmp_bytes(nblk + 2)})));
        HIPCHK(ctx->crcnt.ensure((uint64_t)G * (nblk + 1) * 4 + 256));
        int rc0 = keys_stage(ctx, gt, T, B, N, ctx->recA.as<uint64_t>(), ctx->mstart.as<uint32_t>(), st);
        if (rc0) return rc0;
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        int ob = 0;
        HIPCHK(seg_onesweep_sort(ctx->recA.as<uint64_t>(), ctx->recB.as<uint64_t>(), N, kbits - B, B,
                                 ctx->mstart.as<uint32_t>(), ctx->tmp.p, &dc->err, &ob, st));
        const uint64_t nd = 1ull << B;
        std::vector<uint32_t> h32(nd + 1);
        HIPCHK(hipMemcpyAsync(h32.data(), ctx->mstart.p, (nd + 1) * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::vector<uint64_t> h64(nd + 1);
        for (uint64_t d = 0; d <= nd; ++d) h64[d] = B ? h32[d] : (d ? N : 0);
        HIPCHK(dst.ensure((nd + 1) * 8 + 64));
        HIPCHK(hipMemcpyAsync(dst.p, h64.data(), (nd + 1) * 8, hipMemcpyHostToDevice, st));
        pstream = CrStream{ob ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>(), dst.as<uint64_t>(), (uint32_t)nd, N};
        pstream.kb = (uint32_t)(kbits - B);
        pstream.ib = 32;
        HIPCHK(launch_cr_counts(pstream, gt, ctx->crcnt.as<uint32_t>(), ctx->tmp.p, st));
        // the chunking reads the SML keys only: the indices (tie replay) and crall (the
        // MER_REPEAT_LIMIT plan, LogProgress) are written when a later step needs them
        if (all_ties) {
            HIPCHK(launch_cr_partition(pstream, gt, ctx->crcnt.as<uint32_t>(), kbits, ctx->kA.as<uint64_t>(),
                                       ctx->vA.as<uint32_t>(), ctx->crall.as<uint64_t>(), st));
            have_sml = sml_idx = true;
        } else if (!lean) {
            HIPCHK(build_sml(false));
        }
        sk = ctx->kA.as<uint64_t>();
        sv = ctx->vA.as<uint32_t>();
    } else {
        std::vector<const char*> ptrs(G);
        for (int g = 0; g < G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
        HIPCHK(launch_seed_pack(ctx->ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 0, true, ctx->ckey.p, 0, nullptr,
                                T, &dc->err, st));
        HIPCHK(launch_genome_keys(ctx->ckey.as<uint64_t>(), N, gt, kbits, st));
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        HIPCHK(radix_sort<uint64_t>(ctx->ckey.as<uint64_t>(), nullptr, N, kbits + gbits, ctx->kA.as<uint64_t>(),
                                    ctx->vA.as<uint32_t>(), ctx->kB.as<uint64_t>(), ctx->vB.as<uint32_t>(), ctx->tmp.p,
                                    &buf, st));
        sk = buf ? ctx->kB.as<uint64_t>() : ctx->kA.as<uint64_t>();
        sv = buf ? ctx->vB.as<uint32_t>() : ctx->vA.as<uint32_t>();
    }
    uint32_t nch = 1;
    std::vector<uint64_t> hcs((size_t)G, 0);   // chunk starts (nch x G)
    bool fast_chunks = false;   // chunk starts from the sorted stream, no split (compat_fast_chunks)
    if (mx >= 0 && !have_sml) {
        const uint64_t nmx = gt.n[mx], kmax = nmx ? (nmx - 1) / chunk : 0;
        if (kmax + 1 <= cap && (kmax == 0 || kmax * chunk < gt.m[mx]) && !getenv("MUMS_DEV_COMPAT_SML")) {
            HIPCHK(launch_compat_fast_chunks(pstream, gt, ctx->crcnt.as<uint32_t>(), mx, chunk, ctx->L,
                                             (uint32_t)(kmax + 1), cs, &dc->scratch32, st));
            uint32_t h[2] = {0, 0};
            HIPCHK(hipMemcpyAsync(&h[0], &dc->scratch32, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(&h[1], &dc->err, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (h[1] & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
            if (getenv("MUMS_DEV_COMPAT_DEBUG")) fprintf(stderr, "compat fast chunks: flags %u\n", h[0]);
            if (h[0] == 0) {
                fast_chunks = true;
                nch = (uint32_t)(kmax + 1);
                hcs.assign((size_t)nch * G, 0);
                HIPCHK(hipMemcpyAsync(hcs.data(), cs, hcs.size() * 8, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                for (uint32_t k = 1; k < nch; ++k)
                    for (int g = 0; g < G; ++g)
                        if (hcs[(size_t)k * G + g] < hcs[(size_t)(k - 1) * G + g])
                            return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: decreasing chunk starts "
                                                                 "(overlapping chunk ranges) not reproduced");
            }
        }
        if (!fast_chunks) {
            HIPCHK(hipMemsetAsync(cs, 0, (size_t)cap * G * 8, st));
            HIPCHK(build_sml(false));
        }
    }
    if (mx >= 0 && !fast_chunks) {
        HIPCHK(launch_compat_breaks(sk, gt, kmask, mx, chunk, cs, bm, cap, d_nch, &dc->err, st));
        uint32_t h[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(&h[0], d_nch, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&h[1], &dc->err, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (h[1] & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
        if (h[1] & 4u)
            return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: a masked-key group spans a whole chunk "
                                                 "(the reference's chunking loop does not terminate)");
        if (h[1] & 8u)
            return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: chunk breakpoint past the SML end "
                                                 "(out-of-range SortedMerList::operator[] in the reference)");
        nch = h[0];
        HIPCHK(launch_compat_find(sk, gt, kmask, mx, ctx->L, cs, bm, nch, st));
        hcs.assign((size_t)nch * G, 0);
        HIPCHK(hipMemcpyAsync(hcs.data(), cs, hcs.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (uint32_t k = 1; k < nch; ++k)
            for (int g = 0; g < G; ++g)
                if (hcs[(size_t)k * G + g] < hcs[(size_t)(k - 1) * G + g])
                    return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: decreasing chunk starts "
                                                         "(overlapping chunk ranges) not reproduced");
    }
    ctx->nchunks = nch;
    bool reordered = false;   // an equal-key run of a genome moved into std::sort order
    if (N) {   // SML order of the runs the chunk starts fall into (all runs under repeat tolerance)
        const uint64_t* sps[1] = {cs};
        const uint64_t rws[1] = {nch};
        TieWs tw{};
        uint64_t flagged = 0;
        const bool all = all_ties;
        bool split = !fast_chunks;   // a chunk start inside a run of equal keys: its SML order matters
        if (!all && !fast_chunks) {
            HIPCHK(launch_compat_split(sk, gt, cs, nch, &dc->scratch32, st));
            uint32_t h = 0;
            HIPCHK(hipMemcpyAsync(&h, &dc->scratch32, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            split = h != 0;
        }
        if (split && packed_sml && !sml_idx) HIPCHK(build_sml(true));   // the SMLs' indices for the replay
        if (split) {
            rc = tie_order(ctx, N, sk, sk, nullptr, sv, all ? nullptr : sps, all ? nullptr : rws, all ? 0 : 1, &tw,
                           &flagged, st);
            if (rc) return rc;
        }
        if (flagged) HIPCHK(tie_slots_out(tw, const_cast<uint32_t*>(sv), st));
        reordered = flagged != 0;
        ctx->ties_fixed = all;
    }
    int cbits = 0;
    while (((uint64_t)1 << cbits) < (uint64_t)nch) ++cbits;
    if (kbits + cbits > 64) return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat: too many chunks");
    // the chunk-major stream: from the sorted stream by a stable partition by chunk when its
    // order inside equal keys is the SMLs' (no run reordered), else a (chunk, ckey) radix sort
    // of the SMLs.  The genome-major SMLs' keys (genome bits off, ctx->crall) survive for the
    // MER_REPEAT_LIMIT plan below.
    // Direct form (the common case): compat_recs' packed records straight from the sorted
    // stream when every block boundary is closed under the chunk order (chunked.hip); any flag
    // falls back to the partition below.  It needs no key2 / index arrays, so it is taken only
    // where no later step reads them: no chunk cut (flag 4 screens runs above
    // MER_REPEAT_LIMIT), no rank split, match log or LogProgress.  MUMS_DEV_COMPAT_PART (read
    // per call): the partition always.
    uint64_t* drec = nullptr;
    if (packed_sml && !reordered && N < (1ull << 32) && ctx->compat_ranks <= 1 && !ctx->match_log &&
        !ctx->progress_on && !getenv("MUMS_DEV_COMPAT_PAIRS") && !getenv("MUMS_DEV_COMPAT_GID_SCAN") &&
        !getenv("MUMS_DEV_COMPAT_PART")) {
        uint64_t* out = pstream.rec == ctx->recA.as<uint64_t>() ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>();
        const size_t wsb = (cr_direct_ws_bytes(N) + 255) & ~(size_t)255;
        HIPCHK(ctx->ckey.ensure(std::max<size_t>(N * 8 + 64, wsb + 64)));
        uint32_t* d_flags = (uint32_t*)((char*)ctx->ckey.p + wsb);
        HIPCHK(launch_cr_compat_direct(pstream, gt, ctx->crcnt.as<uint32_t>(), cs, nch, kbits, out, ctx->kB.as<uint64_t>(),
                                       (uint8_t*)ctx->vB.p, ctx->ckey.p, d_flags, st));
        uint32_t hf[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(hf, d_flags, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (getenv("MUMS_DEV_COMPAT_DEBUG"))
            fprintf(stderr, "compat direct: flags %u, %u units, %u chunks\n", hf[0], hf[1], nch);
        if (hf[0] == 0) drec = out;
    }
    if (!drec && !have_sml) HIPCHK(build_sml(false));   // (the MER_REPEAT_LIMIT plan may read them)
    if (drec) {
        buf = 1;   // (key2 / index arrays not built: nothing below reads them)
    } else if (packed_sml && !reordered && cr_chunk_part_fits(N, nch)) {
        HIPCHK(ctx->ckey.ensure(cr_chunk_part_cnt_words(N, nch) * 4 + 64));   // the (chunk, block) counts
        HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(cr_chunk_part_cnt_words(N, nch)))));
        HIPCHK(launch_cr_chunk_part(pstream, gt, ctx->crcnt.as<uint32_t>(), cs, nch, kbits, ctx->ckey.as<uint32_t>(),
                                    ctx->tmp.p, ctx->kB.as<uint64_t>(), ctx->vB.as<uint32_t>(), st));
        buf = 1;
    } else {
        if (!sml_idx) HIPCHK(build_sml(true));
        HIPCHK(launch_compat_chunk_keys(sk, sv, N, gt, kbits, cs, nch, ctx->ckey.as<uint64_t>(),
                                        ctx->cval.as<uint32_t>(), ctx->crall.as<uint64_t>(), st));
        ctx->compat_ck_src = nullptr;   // crall written here; the radix sort below reuses kA
        HIPCHK(radix_sort<uint64_t>(ctx->ckey.as<uint64_t>(), ctx->cval.as<uint32_t>(), N, kbits + cbits,
                                    ctx->kA.as<uint64_t>(), ctx->vA.as<uint32_t>(), ctx->kB.as<uint64_t>(),
                                    ctx->vB.as<uint32_t>(), ctx->tmp.p, &buf, st));
    }
    ctx->sorted_buf = buf;
    ctx->sorted_key = buf ? ctx->kB.p : ctx->kA.p;
    ctx->sorted_idx = buf ? ctx->vB.as<uint32_t>() : ctx->vA.as<uint32_t>();
    ctx->sort_passes = (kbits + cbits + 7) / 8;
    uint64_t n_live = N;
    // the chunk-major stream as packed records for the packed-record probe / materialize
    // kernels (group keys compared for equality only: launch_compat_recs), built in the same
    // pass as MER_REPEAT_LIMIT's candidate list, again after a chunk was cut;
    // MUMS_DEV_COMPAT_PAIRS (read per call): the (key2, index) pair kernels,
    // MUMS_DEV_COMPAT_GID_SCAN: group keys numbered by the scan
    ctx->compat_rec = N < (1ull << 32) && !getenv("MUMS_DEV_COMPAT_PAIRS");
    const bool gid_scan = getenv("MUMS_DEV_COMPAT_GID_SCAN") != nullptr;
    if (ctx->compat_rec) {
        HIPCHK(ctx->recA.ensure(N * 8 + 64));
        HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(N + 1))));
        uint64_t* d_list = nullptr;
        unsigned long long* d_cnt = nullptr;
        uint64_t cap = 0;
        if ((rc = compat_cand_slots(ctx, nch, &d_list, &d_cnt, &cap))) return rc;
        if (drec) {   // no candidates: the direct form screened every masked-key run
            HIPCHK(hipMemsetAsync(d_cnt, 0, 8, st));
            ctx->sorted_rec = drec;
        } else {
            HIPCHK(launch_compat_recs((const uint64_t*)ctx->sorted_key, ctx->sorted_idx, N, kbits,
                                      ctx->recA.as<uint64_t>(), &dc->scratch32, ctx->ckey.as<uint32_t>(), ctx->tmp.p,
                                      gid_scan, d_list, d_cnt, cap, st));
            ctx->sorted_rec = ctx->recA.as<uint64_t>();
        }
    }
    rc = compat_truncate(ctx, nch, cs, kbits, &n_live, st, ctx->compat_rec);
    if (rc) return rc;
    if (ctx->compat_ranks > 1 && (rc = compat_keep_chunks(ctx, nch, kbits, &n_live, st))) return rc;
    if (ctx->compat_ranks > 1 && n_live == 0) {   // no chunk (or no live record) in this rank's range
        ctx->P = 0;
        ctx->M = 0;
        ctx->stage_done = stage >= MUMS_STAGE_ALL ? MUMS_STAGE_ALL : MUMS_STAGE_SEEDS;
        for (int e = EV_SORT; e <= EV_OUTPUT; ++e) HIPCHK(hipEventRecord(ctx->ev[e], st));
        HIPCHK(hipStreamSynchronize(st));
        HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
        fill_stats(ctx, N);
        return MUMS_OK;
    }
    if (ctx->compat_rec && n_live != N)   // records of the cut stream
        HIPCHK(launch_compat_recs((const uint64_t*)ctx->sorted_key, ctx->sorted_idx, n_live, kbits,
                                  ctx->recA.as<uint64_t>(), &dc->scratch32, ctx->ckey.as<uint32_t>(), ctx->tmp.p,
                                  gid_scan, nullptr, nullptr, 0, st));
    if (ctx->progress_on && (rc = progress_compat(ctx, nch, hcs, st))) return rc;
    HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
    SegTile* tiles = ctx->tiles.as<SegTile>();
    HIPCHK(launch_flat_tiles(n_live, tiles, st));
    if (ctx->compat_rec)
        rc = groups_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, tiles, (n_live + kSegTile - 1) / kSegTile, mp,
                                      ps.probe_info, ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
    else
        rc = groups_dispatch<PairView<uint64_t>>(
            ctx, PairView<uint64_t>{(const uint64_t*)ctx->sorted_key, ctx->sorted_idx}, tiles,
            (n_live + kSegTile - 1) / kSegTile, mp, ps.probe_info, ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
    if (rc) return rc;
    rc = finish_seeds(ctx, ps, st, stage >= MUMS_STAGE_ALL);
    if (rc) return rc;
    ctx->compat_pfirst.clear();
    if (ctx->match_log) {   // the probes of every chunk (the match log's per-chunk order)
        DevBuf pf;
        HIPCHK(pf.ensure(((uint64_t)nch + 1) * 4 + 64));
        HIPCHK(launch_compat_probe_chunks(ctx->probe_info, ctx->P, (const uint64_t*)ctx->sorted_key, kbits, nch,
                                          pf.as<uint32_t>(), st));
        ctx->compat_pfirst.resize((size_t)nch + 1);
        HIPCHK(hipMemcpyAsync(ctx->compat_pfirst.data(), pf.p, ((uint64_t)nch + 1) * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    ctx->stage_done = MUMS_STAGE_SEEDS;
    if (stage >= MUMS_STAGE_ALL) {
        rc = find_tail(ctx, mp, ctx->packed.as<uint32_t>(), [&](MatProbes* v) {
            const int r = materialize_seeds(ctx, mp, st);
            v->rows = ctx->mprobe.as<int64_t>();
            return r;
        }, st, true);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
    fill_stats(ctx, N);
    return MUMS_OK;
}

int run_pipeline_pairwise(mums_ctx* ctx, int stage);   // after sort_row_keys below
int run_pipeline_chunked(mums_ctx* ctx, int stage);

int check_ctx(mums_ctx* ctx) {
    if (!ctx) return MUMS_E_INVALID;
    ctx->err.clear();
    return MUMS_OK;
}

// MSD bits of the sharded key exchange: at least the packed-record split (2w+1-32),
// else 8 (256 key ranges to balance over the ranks), never the parity bit.
int shard_msd_bits(int w) {
    const int kbits = 2 * w + 1;
    return std::min(kMaxMsdBits, std::max(kbits - 32, std::min(8, kbits - 1)));
}

int ceil_log2(uint64_t x) {
    int b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

// sharded mode: global table from the layout, local table (owned genomes, global bases)
int prepare_shard(mums_ctx* ctx) {
    if (!ctx->shard) return fail(ctx, MUMS_E_INVALID, "no shard layout (mums_shard_layout)");
    const uint32_t nl = (uint32_t)ctx->genomes.size();
    if (!ctx->slice) {
        if (ctx->shard_first + nl > ctx->shard_len.size())
            return fail(ctx, MUMS_E_INVALID, "owned genomes exceed the shard layout");
        for (uint32_t i = 0; i < nl; ++i)
            if (ctx->genomes[i].n != ctx->shard_len[ctx->shard_first + i])
                return fail(ctx, MUMS_E_INVALID, "owned genome length differs from the shard layout");
    }
    int rc = prepare_run(ctx, ctx->shard_len);
    if (rc) return rc;
    // the sharded merge / find build MemHash's MatchParams: a ParallelMemHash compat or
    // PairwiseMatchFinder context would silently get MemHash's MatchList
    if (ctx->pcompat)
        return fail(ctx, MUMS_E_UNSUPPORTED, "sharded mode: ParallelMemHash compat runs single-GPU only");
    if (ctx->match_log)   // (compat contexts: ctx_compat_rank_find)
        return fail(ctx, MUMS_E_UNSUPPORTED, "sharded MemHash: no match log (ParallelMemHash compat ranks only)");
    if (2 * ctx->w + 1 > 32 + kMaxMsdBits)
        return fail(ctx, MUMS_E_UNSUPPORTED, "sharded mode needs 2w+1 <= 43 (packed records)");
    GenomeTable& l = ctx->lgt;
    l = GenomeTable{};
    if (ctx->slice) {   // one genome slice: its SML positions [slice_begin, slice_end)
        const uint32_t g = ctx->slice_genome;
        const uint64_t mg = ctx->gt.m[g], b0 = ctx->slice_begin, b1 = ctx->slice_end;
        if (g >= (uint32_t)ctx->gt.G || b0 > b1 || b1 > mg || nl != 1)
            return fail(ctx, MUMS_E_INVALID, "bad genome slice");
        const uint64_t want = (b1 > b0) ? std::min<uint64_t>(ctx->gt.n[g], b1 + ctx->L - 1) - b0 : 0;
        if (ctx->genomes[0].n != want)
            return fail(ctx, MUMS_E_INVALID, "slice ASCII must hold bases [begin, end + L - 1) of its genome");
        l.G = 1;
        l.n[0] = want;
        l.m[0] = b1 - b0;
        l.base[0] = ctx->gt.base[g] + b0;
        for (int k = 1; k <= kMaxG; ++k) l.base[k] = l.base[0] + l.m[0];
    } else {
        l.G = (int)nl;
        for (uint32_t i = 0; i < nl; ++i) {
            l.n[i] = ctx->gt.n[ctx->shard_first + i];
            l.m[i] = ctx->gt.m[ctx->shard_first + i];
            l.base[i] = ctx->gt.base[ctx->shard_first + i];
        }
        for (int g = (int)nl; g <= kMaxG; ++g) l.base[g] = ctx->gt.base[ctx->shard_first + nl];
    }
    ctx->packed_path = true;
    ctx->msd_bits = shard_msd_bits(ctx->w);
    // records: 32-bit global indices up to 2^32 seed-mers, 33-bit beyond (the key part
    // then holds 2w+1-B = 31 bits: w19 with B = 8)
    const bool big = ctx->gt.base[ctx->gt.G] >= 0xFFFFFFF0ull || getenv("MUMS_DEV_SHARD_IB33") != nullptr;
    ctx->rec_ib = big ? 33 : 32;
    ctx->shard_side = 0;
    if (big && 2 * ctx->w + 1 - 31 > 8 && 2 * ctx->w + 1 - 31 <= 12) {
        // w20-21 (getDefaultSeedWeight of 3 Gbp genomes, SeedMasks.h:389-401): 31 key bits in
        // the record, 8 MSD bits scattered + 2-4 side bits split before the exchange (msdsplit.hip)
        ctx->msd_bits = 2 * ctx->w + 1 - 31;
        ctx->shard_side = ctx->msd_bits - 8;
    } else if (big && (2 * ctx->w + 1 - ctx->msd_bits != 31 || ctx->msd_bits > 8)) {
        return fail(ctx, MUMS_E_UNSUPPORTED, "sharded mode above 2^32 seed-mers needs seed weight 19-21");
    }
    return MUMS_OK;
}

}  // namespace

extern "C" {

int mums_abi_version(void) { return MUMS_ABI_VERSION; }

int mums_ctx_create(int device, mums_ctx** out) {
    if (!out) return MUMS_E_INVALID;
    *out = nullptr;
    if (!have_device()) return MUMS_E_NODEVICE;
    mums_ctx* ctx = new mums_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { delete ctx; return MUMS_E_HIP; }
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete ctx; return MUMS_E_HIP; }
    ctx->own_stream = true;
    for (int i = 0; i < EV_COUNT; ++i) (void)hipEventCreate(&ctx->ev[i]);
    for (int i = 0; i < 6; ++i) (void)hipEventCreate(&ctx->ev_walk[i]);
    *out = ctx;
    return MUMS_OK;
}

int mums_ctx_destroy(mums_ctx* ctx) {
    if (!ctx) return MUMS_E_INVALID;
    (void)hipSetDevice(ctx->device);
    mums_clear(ctx);
    DevBuf* bufs[] = {&ctx->packed, &ctx->recA, &ctx->recB, &ctx->hist, &ctx->tiles, &ctx->ckey, &ctx->kA,
                      &ctx->kB, &ctx->vA, &ctx->vB, &ctx->tmp, &ctx->partials, &ctx->counters, &ctx->bstart,
                      &ctx->bend, &ctx->tsize, &ctx->obase, &ctx->pool, &ctx->tbl, &ctx->out_len, &ctx->out_s,
                      &ctx->pbuf, &ctx->keybuf, &ctx->mstart, &ctx->chain_tmp, &ctx->chain_of,
                      &ctx->radix_tmp, &ctx->spill, &ctx->summ, &ctx->dbgbuf, &ctx->mprobe, &ctx->rowtmp,
                      &ctx->cval, &ctx->ctab, &ctx->smlk0, &ctx->smlkA, &ctx->smlkB, &ctx->smlvA,
                      &ctx->smlvB, &ctx->smltmp, &ctx->flen, &ctx->fs, &ctx->rowsall, &ctx->rsbuf,
                      &ctx->rsplan, &ctx->rsbst, &ctx->pool_loc, &ctx->cbuf, &ctx->sids,
                      &ctx->logA, &ctx->logB, &ctx->logvA, &ctx->logvB, &ctx->tiebuf, &ctx->fk, &ctx->fkloc,
                      &ctx->crbuf, &ctx->crcnt, &ctx->crlive, &ctx->crruns, &ctx->crall, &ctx->fsk, &ctx->bst2,
                      &ctx->side, &ctx->bst8, &ctx->cbst, &ctx->dsarr, &ctx->labx, &ctx->rkpool0, &ctx->rkpool1,
                      &ctx->rku32, &ctx->ascii_all};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i < EV_COUNT; ++i)
        if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
    for (int i = 0; i < 16; ++i)
        if (ctx->ev_ds[i]) (void)hipEventDestroy(ctx->ev_ds[i]);
    for (int i = 0; i < 6; ++i)
        if (ctx->ev_walk[i]) (void)hipEventDestroy(ctx->ev_walk[i]);
    if (ctx->compat_sub) (void)mums_ctx_destroy(ctx->compat_sub);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return MUMS_OK;
}

int mums_set_stream(mums_ctx* ctx, void* s) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!s) return fail(ctx, MUMS_E_INVALID, "null stream");
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    ctx->stream = (hipStream_t)s;
    ctx->own_stream = false;
    return MUMS_OK;
}

int mums_set_seed(mums_ctx* ctx, uint64_t pattern) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    ctx->seed = pattern;
    return MUMS_OK;
}

int mums_set_params(mums_ctx* ctx, uint32_t repeat_tol, uint32_t enum_tol, uint32_t table_size) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (table_size == 0 || table_size > 0x7FFFFFFFu)
        return fail(ctx, MUMS_E_INVALID, "table size must be in [1, 2^31)");
    ctx->repeat_tol = repeat_tol;
    ctx->enum_tol = enum_tol;
    ctx->table_size = table_size;
    return MUMS_OK;
}

int mums_set_mask(mums_ctx* ctx, int masked, uint64_t seq_mask) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    ctx->masked = masked ? 1 : 0;
    ctx->seq_mask = seq_mask;
    return MUMS_OK;
}

int mums_add_genome(mums_ctx* ctx, const char* ascii, uint64_t n) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!ascii && n) return fail(ctx, MUMS_E_INVALID, "Null gnSequence pointer");  // MatchFinder.cpp:63-65
    if (ctx->genomes.size() >= (size_t)kMaxG)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 64 genomes per context");
    HIPCHK(hipSetDevice(ctx->device));
    char* d = nullptr;
    HIPCHK(hipMalloc(&d, n + 16));
    if (n) HIPCHK(h2d_sync(d, ascii, n, ctx->stream));
    ctx->genomes.push_back({d, n, true});
    ctx->stage_done = 0;
    return MUMS_OK;
}

int mums_add_genome_device(mums_ctx* ctx, const void* d_ascii, uint64_t n) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!d_ascii && n) return fail(ctx, MUMS_E_INVALID, "Null gnSequence pointer");
    if (ctx->genomes.size() >= (size_t)kMaxG)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 64 genomes per context");
    ctx->genomes.push_back({(const char*)d_ascii, n, false});
    ctx->stage_done = 0;
    return MUMS_OK;
}

int mums_genome_device(mums_ctx* ctx, uint32_t genome, const void** d_ascii, uint64_t* n) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!d_ascii || !n) return fail(ctx, MUMS_E_INVALID, "null output pointer");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    *d_ascii = ctx->genomes[genome].d_ptr;
    *n = ctx->genomes[genome].n;
    return MUMS_OK;
}

int mums_clear(mums_ctx* ctx) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    (void)hipSetDevice(ctx->device);
    for (auto& g : ctx->genomes)
        if (g.owned && g.d_ptr) (void)hipFree((void*)g.d_ptr);
    ctx->genomes.clear();
    ctx->stage_done = 0;
    ctx->M = ctx->P = ctx->N = 0;
    ctx->st = mums_stats{};
    return MUMS_OK;
}

int mums_find_stage(mums_ctx* ctx, int stage) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    if (ctx->shard) return fail(ctx, MUMS_E_INVALID, "context is in sharded mode: use mums_shard_keys/merge");
    HIPCHK(hipSetDevice(ctx->device));
    std::vector<uint64_t> lens;
    for (auto& g : ctx->genomes) lens.push_back(g.n);
    int rc = prepare_run(ctx, lens);
    if (rc) return rc;
    if (ctx->genomes.empty()) {
        ctx->stage_done = MUMS_STAGE_ALL;
        ctx->st = mums_stats{};
        return MUMS_OK;
    }
    const bool big = ctx->N >= 0xFFFFFFF0ull || getenv("MUMS_DEV_CHUNK_RECORDS") != nullptr;
    if (big && ctx->pcompat)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed-mers: ParallelMemHash compat not supported");
    if (ctx->pcompat && ctx->enum_tol > 1)
        return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat with enumeration tolerance > 1");
    if (!ctx->start_points.empty() && ctx->start_points.size() != ctx->genomes.size())   // MatchFinder.cpp:197-199
        return fail(ctx, MUMS_E_INVALID, "start points: one per sequence required");
    if (have_start_points(ctx) && ctx->pcompat)
        // ParallelMemHash has no FindMatchesFromPosition of its own: the inherited MemHash one
        // (MemHash.cpp:117-127) runs SearchRange into ParallelMemHash::AddHashEntry's thread
        // table (ParallelMemHash.cpp:123-127), which only FindMatches sizes (:85-86) and merges:
        // undefined behaviour in the reference, refused here
        return fail(ctx, MUMS_E_UNSUPPORTED, "start points (FindMatchesFromPosition) in the ParallelMemHash compat mode: "
                                             "the reference hashes them into an unsized thread table");
    // the chunked mode may keep its (config-5-sized) tie workspace between seed-stage-only
    // calls; any other pipeline sizes its own
    if (!big && ctx->tiebuf_kept) release_tiebuf(ctx);
    if ((ctx->pairwise || ctx->enum_tol > 1) && !big) return run_pipeline_pairwise(ctx, stage);
    if (ctx->pcompat) return run_pipeline_compat(ctx, stage);
    return big ? run_pipeline_chunked(ctx, stage) : run_pipeline(ctx, stage);
}

int mums_set_start_points(mums_ctx* ctx, const uint64_t* start_points, uint32_t count) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (count && !start_points) return fail(ctx, MUMS_E_INVALID, "null start points");
    ctx->start_points.assign(start_points, start_points + count);
    return MUMS_OK;
}

int mums_get_offset_log(mums_ctx* ctx, uint64_t* out, uint64_t cap_rows, uint64_t* rows, uint32_t* seq_count) {
    if (check_ctx(ctx) || !rows) return MUMS_E_INVALID;
    const uint64_t G = (uint64_t)ctx->gt.G, R = G ? ctx->offset_log.size() / G : 0;
    *rows = R;
    if (seq_count) *seq_count = (uint32_t)G;
    if (!out || cap_rows == 0) return MUMS_OK;
    if (cap_rows < R) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    std::copy(ctx->offset_log.begin(), ctx->offset_log.end(), out);
    return MUMS_OK;
}

int mums_set_pairwise(mums_ctx* ctx, int enable) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    ctx->pairwise = enable != 0;
    return MUMS_OK;
}

int mums_set_parallel_compat(mums_ctx* ctx, int enable, uint64_t chunk_size) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (enable && chunk_size == 0) chunk_size = 200000;   // CHUNK_SIZE, ParallelMemHash.cpp:51
    ctx->pcompat = enable != 0;
    ctx->chunk_size = chunk_size ? chunk_size : 200000;
    return MUMS_OK;
}

int mums_find(mums_ctx* ctx) { return mums_find_stage(ctx, MUMS_STAGE_ALL); }

int mums_result_count(mums_ctx* ctx, uint64_t* count, uint32_t* seq_count) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (count) *count = ctx->M;
    if (seq_count) *seq_count = (uint32_t)ctx->gt.G;   // all genomes of the problem (sharded: not only the owned)
    return MUMS_OK;
}

int mums_result_copy(mums_ctx* ctx, uint64_t* lengths, int64_t* starts) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (ctx->M == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    const size_t G = (size_t)ctx->gt.G;
    if (lengths) HIPCHK(hipMemcpy(lengths, ctx->out_len.p, ctx->M * 8, hipMemcpyDeviceToHost));
    if (starts) HIPCHK(hipMemcpy(starts, ctx->out_s.p, ctx->M * G * 8, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

int mums_mem_table_count(mums_ctx* ctx, uint32_t* counts, uint32_t table_size) {
    if (check_ctx(ctx) || !counts) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (table_size != ctx->table_size) return fail(ctx, MUMS_E_INVALID, "table_size differs from the context's");
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->P == 0 && ctx->M == 0) {   // nothing hashed (the table buffers may be unset)
        std::fill(counts, counts + table_size, 0u);
        return MUMS_OK;
    }
    HIPCHK(hipMemcpy(counts, ctx->tsize.p, (size_t)table_size * 4, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

int mums_get_stats(mums_ctx* ctx, mums_stats* out) {
    if (check_ctx(ctx) || !out) return MUMS_E_INVALID;
    *out = ctx->st;
    return MUMS_OK;
}

const char* mums_last_error(mums_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mums_set_profiling(mums_ctx* ctx, int enable) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    ctx->profiling = enable != 0;
    return MUMS_OK;
}

int mums_copy_seed_keys(mums_ctx* ctx, uint32_t genome, uint64_t* out, uint64_t cap) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not computed yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    const uint64_t m = ctx->gt.m[genome];
    if (cap < m) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    if (m == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(ctx->keybuf.ensure(m * 8));
    HIPCHK(launch_keys_of_genome(ctx->ss, ctx->packed.as<uint32_t>() + ctx->gt.woff[genome], m,
                                 ctx->keybuf.as<uint64_t>(), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(out, ctx->keybuf.p, m * 8, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

int mums_copy_seed_keys_range(mums_ctx* ctx, uint32_t genome, uint64_t first, uint64_t count, uint64_t* out) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not computed yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    const uint64_t m = ctx->gt.m[genome];
    if (first > m || count > m - first) return fail(ctx, MUMS_E_INVALID, "position range outside the genome's SML");
    if (count == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    // keys of positions [first & ~15, first + count) from the word holding position first
    const uint64_t a = first & ~15ull, mm = first + count - a;
    HIPCHK(ctx->keybuf.ensure(mm * 8));
    HIPCHK(launch_keys_of_genome(ctx->ss, ctx->packed.as<uint32_t>() + ctx->gt.woff[genome] + a / 16, mm,
                                 ctx->keybuf.as<uint64_t>(), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(out, ctx->keybuf.as<uint64_t>() + (first - a), count * 8, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

// One genome's SortedMerList on the device (MemorySML::Create, MemorySML.cpp:45-60):
// its ckeys from the packed genome, stably sorted (ties by position) -> *sk, *sv.
int genome_sml(mums_ctx* ctx, uint32_t genome, const uint64_t** sk, const uint32_t** sv) {
    const uint64_t m = ctx->gt.m[genome];
    hipStream_t st = ctx->stream;
    HIPCHK(ctx->smlk0.ensure(m * 8 + 64));
    HIPCHK(ctx->smlkA.ensure(m * 8 + 64));
    HIPCHK(ctx->smlkB.ensure(m * 8 + 64));
    HIPCHK(ctx->smlvA.ensure(m * 4 + 64));
    HIPCHK(ctx->smlvB.ensure(m * 4 + 64));
    HIPCHK(ctx->smltmp.ensure(std::max(radix_tmp_bytes(m + 1), occ_tmp_bytes(m + 1))));
    int buf = 0;
    if (m) {
        HIPCHK(launch_keys_of_genome(ctx->ss, ctx->packed.as<uint32_t>() + ctx->gt.woff[genome], m,
                                     ctx->smlk0.as<uint64_t>(), st, false));
        HIPCHK(radix_sort<uint64_t>(ctx->smlk0.as<uint64_t>(), nullptr, m, 2 * ctx->w + 1, ctx->smlkA.as<uint64_t>(),
                                    ctx->smlvA.as<uint32_t>(), ctx->smlkB.as<uint64_t>(), ctx->smlvB.as<uint32_t>(),
                                    ctx->smltmp.p, &buf, st));
    }
    *sk = buf ? ctx->smlkB.as<uint64_t>() : ctx->smlkA.as<uint64_t>();
    *sv = buf ? ctx->smlvB.as<uint32_t>() : ctx->smlvA.as<uint32_t>();
    if (m > 1) {   // equal mers in std::sort order (MemorySML.cpp:54; smlsort.hip)
        if (m >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList of more than 2^32 seed-mers");
        HIPCHK(tiebuf_ensure(ctx, tie_ws_bytes(m, 1)));
        const TieWs tw = tie_ws_layout(ctx->tiebuf.p, m, 1);
        const uint64_t b0 = 0;
        HIPCHK(tie_set_genomes(tw, &b0, &m, st));
        HIPCHK(tie_clear_flags(tw, st));
        HIPCHK(tie_mark_all(tw, *sk, st));
        uint64_t flagged = 0;
        HIPCHK(tie_prepare(tw, &flagged, st));
        if (flagged) {
            HIPCHK(hipMemcpyAsync(tw.K, ctx->smlk0.p, m * 8, hipMemcpyDeviceToDevice, st));
            HIPCHK(tie_replay(tw, st));
            HIPCHK(tie_slots_out(tw, const_cast<uint32_t*>(*sv), st));
        }
    }
    return MUMS_OK;
}

int mums_build_sml(mums_ctx* ctx, uint32_t genome, uint32_t* positions, uint64_t cap) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not sorted yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    const uint64_t m = ctx->gt.m[genome];
    if (cap < m) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t* sk = nullptr;
    const uint32_t* sv = nullptr;
    int rc = genome_sml(ctx, genome, &sk, &sv);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (m) HIPCHK(hipMemcpy(positions, sv, m * 4, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

int mums_seed_occurrence(mums_ctx* ctx, uint32_t genome, float* freq, uint64_t cap) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not computed yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    const uint64_t m = ctx->gt.m[genome], n = ctx->gt.n[genome];
    if (cap < n) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    if (n >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "genome longer than 2^32");
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t* sk = nullptr;
    const uint32_t* sv = nullptr;
    int rc = genome_sml(ctx, genome, &sk, &sv);
    if (rc) return rc;
    HIPCHK(ctx->keybuf.ensure(n * 4 + 64));
    HIPCHK(launch_seed_occurrence(sk, sv, m, n, ctx->L, ctx->smltmp.p, ctx->keybuf.as<float>(), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (n) HIPCHK(hipMemcpy(freq, ctx->keybuf.p, n * 4, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

// ---- on-disk SortedMerList, DNAFileSML format version 5 ------------
// File = SMLHeader (SortedMerList.h:48-63, written raw: FileSML.cpp:336) + the 2-bit
// sequence words (binary_seq_len = ceil(2n/32) + 2, :340) + SMLLength() uint32 positions in
// SML order (:344-345).  Header values as dmSML's InitSML writes them (dmSML/sml.c:9-24).
// Layout on x86-64 with libGenome's one-byte boolean: 2352 bytes.
struct SmlHeaderV5 {
    uint32_t version;
    uint32_t alphabet_bits;
    uint64_t seed;
    uint32_t seed_length;
    uint32_t seed_weight;
    uint64_t length;
    uint32_t unique_mers;
    uint32_t word_size;
    uint8_t little_endian;
    int16_t id;
    uint8_t circular;
    uint8_t translation_table[255];   // UINT8_MAX entries
    char description[2048];           // DESCRIPTION_SIZE
};
static_assert(sizeof(SmlHeaderV5) == 2352, "SMLHeader layout");
static_assert(offsetof(SmlHeaderV5, id) == 42 && offsetof(SmlHeaderV5, circular) == 44 &&
              offsetof(SmlHeaderV5, translation_table) == 45 && offsetof(SmlHeaderV5, description) == 300,
              "SMLHeader field offsets");
constexpr uint32_t kDnaFileSmlVersion = 5;   // DNAFileSML::FormatVersion (DNAFileSML.h:58-62)

void basic_dna_table(uint8_t* t) {   // SortedMerList::CreateBasicDNATable (SortedMerList.cpp:29-47)
    memset(t, 0, 255);
    const char* c1 = "cCbByY";
    const char* c2 = "gGsSkK";
    for (const char* p = c1; *p; ++p) t[(uint8_t)*p] = 1;
    for (const char* p = c2; *p; ++p) t[(uint8_t)*p] = 2;
    t['t'] = 3;
    t['T'] = 3;
}

int mums_write_sml(mums_ctx* ctx, uint32_t genome, const char* path, const char* description) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not computed yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    if (!path) return fail(ctx, MUMS_E_INVALID, "null path");
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t n = ctx->gt.n[genome], m = ctx->gt.m[genome];
    const uint64_t words = packed_words(n);
    const uint64_t* sk = nullptr;
    const uint32_t* sv = nullptr;
    int rc = genome_sml(ctx, genome, &sk, &sv);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    std::vector<uint32_t> w(words), pos(m);
    HIPCHK(hipMemcpy(w.data(), ctx->packed.as<uint32_t>() + ctx->gt.woff[genome], words * 4, hipMemcpyDeviceToHost));
    if (m) HIPCHK(hipMemcpy(pos.data(), sv, m * 4, hipMemcpyDeviceToHost));
    SmlHeaderV5 h;
    memset(&h, 0, sizeof(h));
    h.version = kDnaFileSmlVersion;
    h.alphabet_bits = 2;
    h.seed = ctx->pattern;
    h.seed_length = (uint32_t)ctx->L;
    h.seed_weight = (uint32_t)ctx->w;
    h.length = n;
    h.unique_mers = 0xFFFFFFFFu;   // NO_UNIQUE_COUNT (SortedMerList.h:36)
    h.word_size = 32;
    h.little_endian = 1;
    basic_dna_table(h.translation_table);
    if (description) strncpy(h.description, description, sizeof(h.description) - 1);
    FILE* f = fopen(path, "wb");
    if (!f) return fail(ctx, MUMS_E_INVALID, "Unable to open file for writing.");   // FileSML.cpp:125
    bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
    ok = ok && fwrite(w.data(), 4, words, f) == words;
    ok = ok && (m == 0 || fwrite(pos.data(), 4, m, f) == m);
    ok = (fclose(f) == 0) && ok;
    if (!ok) return fail(ctx, MUMS_E_INVALID, "Error writing sorted mer list to disk.");   // FileSML.cpp:349
    return MUMS_OK;
}

// FileSML::LoadFile (FileSML.cpp:46-110): header check, then the 2-bit sequence becomes a
// context-owned genome (unpacked on the device; ExtendMatch and the keys only ever see
// the 2-bit codes, so A/C/G/T re-pack to the same words).  *seed_out = header.seed.
int mums_add_genome_sml(mums_ctx* ctx, const char* path, uint64_t* seed_out) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!path) return fail(ctx, MUMS_E_INVALID, "null path");
    if (ctx->genomes.size() >= (size_t)kMaxG)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 64 genomes per context");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(ctx, MUMS_E_INVALID, "Unable to open file.");   // FileSML.cpp:51
    SmlHeaderV5 h;
    if (fread(&h, sizeof(h), 1, f) != 1) { fclose(f); return fail(ctx, MUMS_E_INVALID, "Unable to read file."); }
    if (h.version != kDnaFileSmlVersion) { fclose(f); return fail(ctx, MUMS_E_INVALID, "Unsupported file format."); }
    if (h.alphabet_bits != 2 || h.circular) {
        fclose(f);
        return fail(ctx, MUMS_E_UNSUPPORTED, "only linear DNA sorted mer lists are supported");
    }
    const uint64_t n = h.length, words = packed_words(n);
    std::vector<uint32_t> w(words);
    const bool ok = fread(w.data(), 4, words, f) == words;
    fclose(f);
    if (!ok) return fail(ctx, MUMS_E_INVALID, "Error reading sequence data.");   // FileSML.cpp:86
    HIPCHK(hipSetDevice(ctx->device));
    char* d = nullptr;
    uint32_t* dw = nullptr;
    HIPCHK(hipMalloc(&d, n + 16));
    HIPCHK(hipMalloc(&dw, words * 4 + 16));
    HIPCHK(h2d_sync(dw, w.data(), words * 4, ctx->stream));
    HIPCHK(launch_unpack(dw, n, d, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipFree(dw));
    ctx->genomes.push_back({d, n, true});
    ctx->stage_done = 0;
    if (seed_out) *seed_out = h.seed;
    return MUMS_OK;
}

// MultiplicityFilter / LengthFilter (MatchList.h:636-664) on the context's MatchList
int match_filter(mums_ctx* ctx, uint32_t mult, uint64_t min_len) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    HIPCHK(hipSetDevice(ctx->device));
    const int G = ctx->gt.G;
    const uint64_t M = ctx->M;
    hipStream_t st = ctx->stream;
    HIPCHK(ctx->flen.ensure((M + 1) * 8));
    HIPCHK(ctx->fs.ensure((M + 1) * (size_t)G * 8 + 8));
    HIPCHK(ctx->smltmp.ensure(filter_tmp_bytes(M + 1) + 64));
    uint32_t* d_kept = (uint32_t*)ctx->smltmp.p;
    HIPCHK(launch_match_filter(ctx->out_len.as<uint64_t>(), ctx->out_s.as<int64_t>(), M, G, mult, min_len,
                               (char*)ctx->smltmp.p + 256, d_kept, ctx->flen.as<uint64_t>(), ctx->fs.as<int64_t>(),
                               st));
    uint32_t kept = 0;
    HIPCHK(hipMemcpyAsync(&kept, d_kept, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::swap(ctx->out_len, ctx->flen);
    std::swap(ctx->out_s, ctx->fs);
    ctx->M = kept;
    return MUMS_OK;
}

int mums_multiplicity_filter(mums_ctx* ctx, uint32_t mult) {
    if (mult == 0) return check_ctx(ctx) ? MUMS_E_INVALID : fail(ctx, MUMS_E_INVALID, "multiplicity 0");
    return match_filter(ctx, mult, 0);
}

int mums_length_filter(mums_ctx* ctx, uint64_t min_len) { return match_filter(ctx, 0, min_len); }

extern "C++" {
hipStream_t mums::ctx_stream(mums_ctx* ctx) { return ctx->stream; }
uint32_t mums::ctx_repeat_tol(mums_ctx* ctx) { return ctx->repeat_tol; }
bool mums::ctx_merge_chunked(mums_ctx* ctx) { return ctx->merge_chunked; }
bool mums::ctx_tie_all(mums_ctx* ctx) { return wants_tie_order(ctx); }
int mums::ctx_device(mums_ctx* ctx) { return ctx->device; }
int mums::ctx_table_genomes(mums_ctx* ctx, uint32_t* table_size, uint32_t* genomes) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    *table_size = ctx->table_size;
    *genomes = (uint32_t)ctx->gt.G;
    return MUMS_OK;
}

// ---- ParallelMemHash compat over ranks (shard_comm.hip compat_shard_run) ----------------
bool mums::ctx_pcompat(mums_ctx* ctx) { return ctx && ctx->pcompat; }

int mums::ctx_compat_layout(mums_ctx* ctx, uint32_t* first, uint32_t* nown, std::vector<uint64_t>* lens) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!ctx->shard) return fail(ctx, MUMS_E_INVALID, "no shard layout (mums_shard_layout)");
    if (ctx->slice)
        return fail(ctx, MUMS_E_UNSUPPORTED, "sharded ParallelMemHash compat: genome blocks only (no position slices)");
    if (ctx->pairwise || ctx->enum_tol > 1)
        return fail(ctx, MUMS_E_UNSUPPORTED, "ParallelMemHash compat with PairwiseMatchFinder / enumeration tolerance > 1");
    if (!ctx->start_points.empty())
        return fail(ctx, MUMS_E_UNSUPPORTED, "start points (FindMatchesFromPosition) in the ParallelMemHash compat mode");
    const uint32_t nl = (uint32_t)ctx->genomes.size();
    if (ctx->shard_first + nl > ctx->shard_len.size())
        return fail(ctx, MUMS_E_INVALID, "owned genomes exceed the shard layout");
    for (uint32_t i = 0; i < nl; ++i)
        if (ctx->genomes[i].n != ctx->shard_len[ctx->shard_first + i])
            return fail(ctx, MUMS_E_INVALID, "owned genome length differs from the shard layout");
    *first = ctx->shard_first;
    *nown = nl;
    *lens = ctx->shard_len;
    return MUMS_OK;
}

int mums::ctx_compat_rank_find(mums_ctx* ctx, const char* const* d_ascii, const uint64_t* lens, int G, uint32_t rank,
                               uint32_t ranks, int stage) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    if (!ctx->compat_sub) {
        mums_ctx* sub = nullptr;
        const int rc = mums_ctx_create(ctx->device, &sub);
        if (rc) return fail(ctx, rc, "compat rank context");
        ctx->compat_sub = sub;
    }
    mums_ctx* sub = ctx->compat_sub;
    (void)mums_clear(sub);
    if (mums_set_stream(sub, ctx->stream)) return fail(ctx, MUMS_E_HIP, "compat rank context stream");
    sub->seed = ctx->seed;
    sub->repeat_tol = ctx->repeat_tol;
    sub->enum_tol = ctx->enum_tol;
    sub->table_size = ctx->table_size;
    sub->masked = ctx->masked;
    sub->seq_mask = ctx->seq_mask;
    sub->pcompat = true;
    sub->chunk_size = ctx->chunk_size;
    sub->progress_on = ctx->progress_on;
    sub->profiling = ctx->profiling;
    sub->match_log = false;
    sub->compat_rank = rank;
    sub->compat_ranks = ranks;
    for (int g = 0; g < G; ++g)
        if (mums_add_genome_device(sub, d_ascii[g], lens[g])) return fail(ctx, MUMS_E_INVALID, sub->err);
    const int rc = mums_find_stage(sub, stage);
    if (rc) return fail(ctx, rc, sub->err);
    ctx->gt = sub->gt;
    ctx->st = sub->st;
    ctx->progress = sub->progress;
    ctx->nchunks = sub->nchunks;
    ctx->M = 0;
    ctx->stage_done = MUMS_STAGE_SEEDS;   // the MatchList: after the owners' merge
    ctx->log_host = ctx->match_log;
    ctx->log_n = 0;
    ctx->log_hlen.clear();
    ctx->log_hs.clear();
    // SetMatchLog (MemHash.cpp:238-241) over the ranks: the log is the one-thread schedule's --
    // each chunk's thread-table inserts against the WHOLE global table before it (the thread table
    // is a copy of it after every MergeTable, ParallelMemHash.cpp:117) -- which a rank that
    // searched its chunks from its own earlier chunks only does not have (with long bucket vectors
    // a seed finds, or misses, an earlier rank's entry around its lower_bound).  Rank 0 holds
    // every genome (the all-gather above), so it restates the log with the one-context compat
    // search; the other ranks' parts are empty and the ranks' MatchList is unchanged.
    if (ctx->match_log && rank == 0 && stage >= MUMS_STAGE_ALL) {
        mums_ctx* lc = nullptr;
        int r2 = mums_ctx_create(ctx->device, &lc);
        if (r2) return fail(ctx, r2, "compat match log context");
        std::unique_ptr<mums_ctx, int (*)(mums_ctx*)> hold(lc, mums_ctx_destroy);
        if (mums_set_stream(lc, ctx->stream)) return fail(ctx, MUMS_E_HIP, "compat match log context stream");
        lc->seed = ctx->seed;
        lc->repeat_tol = ctx->repeat_tol;
        lc->enum_tol = ctx->enum_tol;
        lc->table_size = ctx->table_size;
        lc->masked = ctx->masked;
        lc->seq_mask = ctx->seq_mask;
        lc->pcompat = true;
        lc->chunk_size = ctx->chunk_size;
        lc->match_log = true;
        for (int g = 0; g < G; ++g)
            if (mums_add_genome_device(lc, d_ascii[g], lens[g])) return fail(ctx, MUMS_E_INVALID, lc->err);
        if ((r2 = mums_find_stage(lc, MUMS_STAGE_ALL))) return fail(ctx, r2, lc->err);
        uint64_t n = 0;
        if ((r2 = mums_match_log_copy(lc, nullptr, nullptr, 0, &n))) return fail(ctx, r2, lc->err);
        ctx->log_hlen.resize(n);
        ctx->log_hs.resize(n * (uint64_t)G);
        if (n && (r2 = mums_match_log_copy(lc, ctx->log_hlen.data(), ctx->log_hs.data(), n, &n)))
            return fail(ctx, r2, lc->err);
        ctx->log_n = n;
    }
    return MUMS_OK;
}

int mums::ctx_compat_rank_export(mums_ctx* ctx, uint64_t* bucket_counts, int64_t* d_rows, uint64_t* M) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    mums_ctx* sub = ctx->compat_sub;
    if (!sub || sub->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no compat rank search");
    const uint32_t Tb = sub->table_size;
    *M = sub->M;
    if (sub->M == 0) {
        std::fill(bucket_counts, bucket_counts + Tb, 0ull);
        return MUMS_OK;
    }
    HIPCHK(hipSetDevice(ctx->device));
    std::vector<uint32_t> ts(Tb);
    HIPCHK(hipMemcpy(ts.data(), sub->tsize.p, (size_t)Tb * 4, hipMemcpyDeviceToHost));
    for (uint32_t b = 0; b < Tb; ++b) bucket_counts[b] = ts[b];
    if (d_rows)
        HIPCHK(launch_rank_rows(sub->obase.as<uint32_t>(), sub->emit_base, sub->emit_tbl, sub->pool.as<int64_t>(),
                                sub->gt.G, Tb, sub->M, d_rows, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return MUMS_OK;
}

// MergeTable of the W sources' tables into one, source after source (compat_ranks.hip): the
// union kernels per step, the exact sequential merge for the buckets whose union fails a check
int mums::ctx_compat_rank_merge(mums_ctx* ctx, const int64_t* d_rows, uint32_t W, const uint64_t* counts, uint32_t nb) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int G = ctx->gt.G;
    const uint64_t rowb = 8ull * (G + 2);
    uint64_t total = 0;
    std::vector<uint64_t> src_n(W, 0);
    for (uint32_t s = 0; s < W; ++s)
        for (uint32_t j = 0; j < nb; ++j) src_n[s] += counts[(uint64_t)s * nb + j];
    for (uint32_t s = 0; s < W; ++s) total += src_n[s];
    if (total >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "compat rank merge: more than 2^32 entries per owner");
    // test hook (read per call): every bucket through the exact sequential merge
    const bool all_exact = getenv("MUMS_DEV_COMPAT_RANK_EXACT") != nullptr;
    const bool dbg = getenv("MUMS_DEV_COMPAT_RANK_DEBUG") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(ctx->rkpool0.ensure((total + 1) * rowb));
    HIPCHK(ctx->rkpool1.ensure((total + 1) * rowb));
    const uint64_t words = 3 * (total + 1) + 8 * ((uint64_t)nb + 2) + 64;
    HIPCHK(ctx->rku32.ensure(words * 4));
    HIPCHK(ctx->tmp.ensure(std::max({ctx->tmp.cap, scan_tmp_bytes(total + 2), scan_tmp_bytes((uint64_t)nb + 2)})));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    uint32_t* u = ctx->rku32.as<uint32_t>();
    uint32_t* lbA = u;
    uint32_t* nd = lbA + (total + 1);
    uint32_t* tblcat = nd + (total + 1);
    uint32_t* offA = tblcat + (total + 1);
    uint32_t* offB = offA + (nb + 2);
    uint32_t* catoff = offB + (nb + 2);
    uint32_t* tsz = catoff + (nb + 2);
    uint32_t* ff = tsz + (nb + 2);
    uint32_t* bad = ff + (nb + 2);
    uint32_t* newoff = bad + (nb + 2);
    int64_t* cur = ctx->rkpool0.as<int64_t>();
    int64_t* nxt = ctx->rkpool1.as<int64_t>();
    uint64_t nA = 0, src_off = 0, coll = 0;
    HIPCHK(hipMemsetAsync(offA, 0, (size_t)(nb + 1) * 4, st));
    std::vector<uint32_t> hoff(nb + 1);
    for (uint32_t s = 0; s < W; ++s) {
        const uint64_t nB = src_n[s];
        hoff[0] = 0;
        for (uint32_t j = 0; j < nb; ++j) hoff[j + 1] = hoff[j] + (uint32_t)counts[(uint64_t)s * nb + j];
        HIPCHK(hipMemcpyAsync(offB, hoff.data(), (size_t)(nb + 1) * 4, hipMemcpyHostToDevice, st));
        if (nB)   // pool = [A rows | B rows]
            HIPCHK(hipMemcpyAsync(cur + nA * (G + 2), d_rows + src_off * (G + 2), nB * rowb, hipMemcpyDeviceToDevice, st));
        src_off += nB;
        HIPCHK(hipMemsetAsync(bad, all_exact ? 0x01 : 0x00, (size_t)(nb + 1) * 4, st));
        HIPCHK(hipMemsetAsync(nd + nB, 0, 4, st));
        HIPCHK(launch_rank_lb(cur, G, (uint32_t)nA, offA, offB, nb, (uint32_t)nB, lbA, nd, bad, st));
        HIPCHK(exclusive_scan_u32(nd, nB + 1, ctx->tmp.p, &dc->scratch32, st));   // nd -> prefix (nB + 1 words)
        HIPCHK(launch_rank_place(cur, G, (uint32_t)nA, offA, offB, nb, (uint32_t)nB, lbA, nd, catoff, tsz, tblcat, st));
        const uint32_t ncat = (uint32_t)(nA + nB);
        HIPCHK(launch_rank_check(cur, G, catoff, tsz, nb, ncat, tblcat, bad, st));
        HIPCHK(launch_rank_exact_init((uint32_t)nA, offA, offB, catoff, nb, ncat, bad, tblcat, tsz, ff, st));
        HIPCHK(launch_compat_merge_from(tsz, catoff, tblcat, cur, G, nb, ff, &dc->collisions, st));
        HIPCHK(hipMemcpyAsync(newoff, tsz, (size_t)nb * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemsetAsync(newoff + nb, 0, 4, st));
        HIPCHK(exclusive_scan_u32(newoff, (uint64_t)nb + 1, ctx->tmp.p, &dc->scratch32, st));
        uint32_t nF = 0;
        HIPCHK(hipMemcpyAsync(&nF, newoff + nb, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(launch_rank_gather(cur, G, catoff, tsz, nb, ncat, tblcat, newoff, nxt, st));
        HIPCHK(hipMemcpyAsync(offA, newoff, (size_t)(nb + 1) * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        if (dbg) {   // development: per source, the buckets that took the exact merge
            std::vector<uint32_t> hb(nb);
            HIPCHK(hipMemcpy(hb.data(), bad, (size_t)nb * 4, hipMemcpyDeviceToHost));
            uint64_t nbad = 0;
            for (uint32_t v : hb) nbad += v != 0;
            fprintf(stderr, "compat rank merge: source %u A %lu B %lu -> %u entries, %lu of %u buckets exact, %.2f ms\n", s,
                    (unsigned long)nA, (unsigned long)nB, nF, (unsigned long)nbad, nb,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        coll += nA + nB - nF;
        nA = nF;
        std::swap(cur, nxt);
    }
    ctx->M = nA;
    HIPCHK(ctx->out_len.ensure((ctx->M + 1) * 8));
    HIPCHK(ctx->out_s.ensure((ctx->M + 1) * (size_t)G * 8));
    HIPCHK(launch_rank_list(cur, G, ctx->M, ctx->out_len.as<uint64_t>(), ctx->out_s.as<int64_t>(), st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->st.mem_count = ctx->M;
    ctx->st.collision_count += coll;   // the rank's own search + this owner's re-adds
    ctx->stage_done = MUMS_STAGE_ALL;
    return MUMS_OK;
}
}

// MemHash::SetMatchLog (MemHash.h:149; written at MemHash.cpp:238-241)
int mums_set_progress_log(mums_ctx* ctx, int enable) {
    if (!ctx) return MUMS_E_INVALID;
    ctx->progress_on = enable != 0;
    ctx->progress.clear();
    return MUMS_OK;
}

int mums_progress_log_copy(mums_ctx* ctx, char* text, uint64_t capacity, uint64_t* length) {
    if (!ctx) return MUMS_E_INVALID;
    if (length) *length = ctx->progress.size();
    if (text && capacity) {
        const uint64_t k = std::min<uint64_t>(capacity - 1, ctx->progress.size());
        std::memcpy(text, ctx->progress.data(), k);
        text[k] = 0;
    }
    return MUMS_OK;
}

int mums_set_match_log(mums_ctx* ctx, int enable) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    ctx->match_log = enable != 0;
    return MUMS_OK;
}

int mums_match_log_copy(mums_ctx* ctx, uint64_t* lengths, int64_t* starts, uint64_t capacity, uint64_t* count) {
    if (check_ctx(ctx) || !count) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (!ctx->match_log)
        return fail(ctx, MUMS_E_INVALID, "the match log was not enabled for this FindMatches (mums_set_match_log)");
    *count = ctx->log_n;
    if (!lengths && !starts) return MUMS_OK;
    if (capacity < ctx->log_n) return fail(ctx, MUMS_E_INVALID, "match log capacity too small");
    if (ctx->log_n == 0) return MUMS_OK;
    const int G = ctx->gt.G;
    if (ctx->log_host) {   // a compat rank's log (ctx_compat_rank_find)
        for (uint64_t i = 0; i < ctx->log_n; ++i) {
            if (lengths) lengths[i] = ctx->log_hlen[i];
            if (starts) std::copy(&ctx->log_hs[i * (uint64_t)G], &ctx->log_hs[(i + 1) * (uint64_t)G], starts + i * (uint64_t)G);
        }
        return MUMS_OK;
    }
    HIPCHK(hipSetDevice(ctx->device));
    std::vector<uint32_t> ids(ctx->log_n);   // pool entries of the inserted chains, in log order
    if (ctx->pcompat) {
        ids = ctx->log_ids;
    } else {
        std::vector<uint64_t> ev(ctx->log_n);
        HIPCHK(hipMemcpy(ev.data(), ctx->logA.p, ctx->log_n * 8, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < ctx->log_n; ++i) ids[i] = (uint32_t)(ev[i] & 0xFFFFFFFFull);
    }
    const uint64_t nid = (uint64_t)*std::max_element(ids.begin(), ids.end()) + 1;
    std::vector<int64_t> pool(nid * (uint64_t)(G + 2));   // one copy of the entries referenced
    HIPCHK(hipMemcpy(pool.data(), ctx->pool.as<int64_t>(), pool.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < ctx->log_n; ++i) {
        const int64_t* e = &pool[(uint64_t)ids[i] * (G + 2)];
        if (lengths) lengths[i] = (uint64_t)e[0];
        if (starts) std::copy(e + 2, e + 2 + G, starts + i * (uint64_t)G);
    }
    return MUMS_OK;
}

// EliminateOverlaps (Aligner.cpp:62-176) on the context's MatchList, in place
int mums_eliminate_overlaps(mums_ctx* ctx) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (ctx->M >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "EliminateOverlaps of more than 2^32 matches");
    HIPCHK(hipSetDevice(ctx->device));
    const int G = ctx->gt.G;
    uint64_t n = 0;
    HIPCHK(eliminate_overlaps_device(ctx->eo, ctx->out_len.as<uint64_t>(), ctx->out_s.as<int64_t>(), ctx->M, G, &n,
                                     ctx->stream));
    HIPCHK(ctx->flen.ensure((n + 1) * 8));
    HIPCHK(ctx->fs.ensure((n + 1) * (size_t)G * 8 + 8));
    HIPCHK(eo_gather(ctx->eo, G, ctx->flen.as<uint64_t>(), ctx->fs.as<int64_t>(), ctx->stream));
    std::swap(ctx->out_len, ctx->flen);
    std::swap(ctx->out_s, ctx->fs);
    ctx->M = n;
    return MUMS_OK;
}

// a caller's MatchList becomes the context's result (filters / EliminateOverlaps input)
int mums_load_matches(mums_ctx* ctx, uint32_t seq_count, uint64_t count, const uint64_t* lengths,
                      const int64_t* starts) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (seq_count == 0 || (count && (!lengths || !starts))) return fail(ctx, MUMS_E_INVALID, "bad MatchList");
    if (!ctx->genomes.empty() && seq_count != ctx->genomes.size())
        return fail(ctx, MUMS_E_INVALID, "MatchList sequence count differs from the context's genomes");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(ctx->out_len.ensure((count + 1) * 8));
    HIPCHK(ctx->out_s.ensure((count + 1) * (size_t)seq_count * 8 + 8));
    if (count) {
        HIPCHK(h2d_sync(ctx->out_len.p, lengths, count * 8, ctx->stream));
        HIPCHK(h2d_sync(ctx->out_s.p, starts, count * (size_t)seq_count * 8, ctx->stream));
    }
    ctx->gt.G = (int)seq_count;
    ctx->M = count;
    ctx->P = 0;
    ctx->stage_done = MUMS_STAGE_ALL;
    return MUMS_OK;
}

// test entry point: the device replay of libstdc++ std::sort (overlaps.hip) on host keys
int mums_debug_std_sort(mums_ctx* ctx, const uint64_t* keys, uint64_t n, int depth_override, uint32_t* ids) {
    if (check_ctx(ctx) || (n && (!keys || !ids))) return MUMS_E_INVALID;
    if (n >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "n >= 2^32");
    if (n == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(ctx->flen.ensure(n * 8 + 8));
    HIPCHK(ctx->fs.ensure(n * 4 + 8));
    HIPCHK(h2d_sync(ctx->flen.p, keys, n * 8, ctx->stream));
    HIPCHK(eo_sort_ids(ctx->eo, ctx->flen.as<uint64_t>(), (uint32_t)n, depth_override, ctx->fs.as<uint32_t>(),
                       ctx->stream));
    HIPCHK(hipMemcpy(ids, ctx->fs.p, n * 4, hipMemcpyDeviceToHost));
    return MUMS_OK;
}

// ---- sharded seed stage -------------------------------------------

int mums_shard_layout(mums_ctx* ctx, uint32_t genomes_total, uint32_t first_genome, const uint64_t* lengths) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (genomes_total > (uint32_t)kMaxG) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 64 genomes");
    if (first_genome > genomes_total || (genomes_total && !lengths))
        return fail(ctx, MUMS_E_INVALID, "bad shard layout");
    ctx->shard = true;
    ctx->slice = false;
    ctx->shard_first = first_genome;
    ctx->shard_len.assign(lengths, lengths + genomes_total);
    ctx->stage_done = 0;
    return MUMS_OK;
}

int mums_shard_slice(mums_ctx* ctx, uint32_t genomes_total, const uint64_t* lengths, uint32_t genome,
                     uint64_t pos_begin, uint64_t pos_end) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (genomes_total > (uint32_t)kMaxG) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 64 genomes");
    if (genome >= genomes_total || !lengths || pos_begin > pos_end) return fail(ctx, MUMS_E_INVALID, "bad slice");
    ctx->shard = true;
    ctx->slice = true;
    ctx->shard_first = genome;
    ctx->slice_genome = genome;
    ctx->slice_begin = pos_begin;
    ctx->slice_end = pos_end;
    ctx->shard_len.assign(lengths, lengths + genomes_total);
    ctx->stage_done = 0;
    return MUMS_OK;
}

int mums_shard_msd_bits(mums_ctx* ctx, uint32_t* msd_bits, uint64_t* local_records) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    int rc = prepare_shard(ctx);
    if (rc) return rc;
    if (msd_bits) *msd_bits = (uint32_t)ctx->msd_bits;
    if (local_records) {
        uint64_t n = 0;
        for (int g = 0; g < ctx->lgt.G; ++g) n += ctx->lgt.m[g];
        *local_records = n;
    }
    return MUMS_OK;
}

int mums_shard_keys(mums_ctx* ctx, uint64_t* d_records, uint64_t capacity, uint64_t* bucket_counts) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = prepare_shard(ctx);
    if (rc) return rc;
    GenomeTable& l = ctx->lgt;
    uint64_t n = 0;
    for (int g = 0; g < l.G; ++g) n += l.m[g];
    if (n > capacity || (n && !d_records)) return fail(ctx, MUMS_E_INVALID, "record buffer too small");
    if (!bucket_counts) return fail(ctx, MUMS_E_INVALID, "null bucket_counts");
    const int B = ctx->msd_bits;
    const uint64_t nb = 1ull << B;
    hipStream_t st = ctx->stream;
    uint64_t words = 0;
    const uint32_t T = layout_packed(l, &words);
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    HIPCHK(ctx->hist.ensure(((uint64_t)T << B) * 4 + 64));
    HIPCHK(ctx->tmp.ensure(scan_tmp_bytes(((uint64_t)T << B) + 1)));
    HIPCHK(ctx->mstart.ensure((nb + 64) * 4));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    std::vector<uint32_t> hs(nb + 1, 0);
    if (l.G > 0 && n > 0) {
        rc = keys_stage(ctx, l, T, B, n, d_records, ctx->mstart.as<uint32_t>(), st, ctx->rec_ib, ctx->shard_side);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(hs.data(), ctx->mstart.p, (nb + 1) * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->hc.err & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
    for (uint64_t b = 0; b < nb; ++b) bucket_counts[b] = (n > 0) ? (uint64_t)hs[b + 1] - hs[b] : 0;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ctx->ev[EV_START], ctx->ev[EV_KEYS]);
    ctx->shard_keys_ms = ms;
    return MUMS_OK;
}

}  // extern "C"

namespace {
// One segment of a whole merged stream (a chunk of the chunked mode, a rank's key range of
// the sharded mode): records [lo, hi), bucket-major over nb local buckets.
struct RestartSeg {
    uint64_t lo, hi;
    uint32_t nb;
};

int stream_restart(mums_ctx* ctx, uint64_t* srec, uint64_t* other, const std::vector<uint64_t>& dstart, uint32_t kb,
                   uint32_t ib, const std::vector<RestartSeg>& segs,
                   const std::function<int(uint32_t, uint32_t*)>& bst_in, uint32_t* d_bst_out,
                   std::vector<uint64_t>& n_live, bool* live_out, hipStream_t st);

// stats of a sharded merge over n records: the regroup copy counts as sort, the keys stage
// is mums_shard_keys' (owned genomes)
void shard_merge_stats(mums_ctx* ctx, uint64_t n) {
    fill_stats(ctx, n);
    float rg = 0.f;
    (void)hipEventElapsedTime(&rg, ctx->ev[EV_START], ctx->ev[EV_KEYS]);
    ctx->st.ms_sort += rg;
    ctx->st.ms_keys = ctx->shard_keys_ms;
}
// The key chunks of a sharded merge above one onesweep merge (2^30 records): runs of
// consecutive local buckets of < cap records each, in key order ({b0, b1} pairs over the
// merge's nbuckets real buckets; bst: local bucket starts).  Empty when a bucket alone is
// too big.
uint64_t shard_chunk_cap() {
    uint64_t cap = (1ull << 30) - 4096;
    if (const char* e = getenv("MUMS_DEV_CHUNK_RECORDS")) cap = std::min<uint64_t>(cap, strtoull(e, nullptr, 10));
    return cap;
}
std::vector<std::pair<uint32_t, uint32_t>> shard_key_chunks(const std::vector<uint32_t>& bst, uint32_t nbuckets,
                                                            uint64_t cap) {
    std::vector<std::pair<uint32_t, uint32_t>> out;
    uint32_t b0 = 0;
    while (b0 < nbuckets) {
        uint32_t b1 = b0;
        while (b1 < nbuckets && (uint64_t)bst[b1 + 1] - bst[b0] < cap) ++b1;
        if (b1 == b0) return {};
        out.push_back({b0, b1});
        b0 = b1;
    }
    return out;
}

// The groups stage of every key chunk of a chunked sharded stream rec (local bucket starts
// bst) in key order: the seed-stage counts over all chunks (ctx->P = their probes); rows:
// every chunk's probe rows appended to ctx->rowsall (the sharded FindMatches' input).
int shard_groups_chunked(mums_ctx* ctx, uint64_t* rec, const std::vector<uint32_t>& bst, const ProbeSpace& ps,
                         bool rows, hipStream_t st) {
    const int mb = ctx->shard_mb, G = ctx->gt.G;
    const uint32_t nbk = 1u << mb;
    const auto chunks = shard_key_chunks(bst, ctx->shard_kcount, shard_chunk_cap());
    if (chunks.empty() && ctx->shard_kcount)
        return fail(ctx, MUMS_E_UNSUPPORTED, "one MSD bucket holds more than 2^30 records");
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    const size_t W = (size_t)(G + 1) * 8;
    uint64_t P_total = 0, groups = 0;
    ctx->fused_keys = false;
    for (const auto& ch : chunks) {
        const uint32_t b0 = ch.first, b1 = ch.second;
        const uint64_t o = bst[b0], nc = (uint64_t)bst[b1] - o;
        std::vector<uint32_t> sub(nbk + 1);
        for (uint32_t b = 0; b <= nbk; ++b) sub[b] = b < b0 ? 0u : (b < b1 ? bst[b] - (uint32_t)o : (uint32_t)nc);
        HIPCHK(hipMemcpyAsync(ctx->mstart.p, sub.data(), sub.size() * 4, hipMemcpyHostToDevice, st));
        SegTile* tiles = ctx->tiles.as<SegTile>();
        HIPCHK(build_seg_tiles_from_starts(ctx->mstart.as<uint32_t>(), mb, nc, tiles, &dc->ntiles, ctx->tmp.p, st));
        const uint64_t ub = seg_tiles_upper(nc, mb);
        int rc;
        if (ctx->rec_ib == 33)
            rc = groups_dispatch<RecViewT<33>>(ctx, RecViewT<33>{rec + o}, tiles, ub, mp, ps.probe_info,
                                               ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
        else
            rc = groups_dispatch<RecView>(ctx, RecView{rec + o}, tiles, ub, mp, ps.probe_info, ps.probe_bucket,
                                          ps.slot_info, ps.slot_bucket, st);
        if (rc) return rc;
        rc = finish_seeds(ctx, ps, st);
        if (rc) return rc;
        const uint64_t Pc = ctx->P;
        if (rows && Pc) {
            if (P_total + Pc >= (1ull << 32) - 64)
                return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes on one rank");
            if (ctx->rowsall.cap < (P_total + Pc + 1) * W) {   // grow, keeping the rows so far
                DevBuf nb;
                HIPCHK(nb.ensure((P_total + Pc + 1) * W * 5 / 4));
                if (P_total) HIPCHK(hipMemcpyAsync(nb.p, ctx->rowsall.p, P_total * W, hipMemcpyDeviceToDevice, st));
                HIPCHK(hipStreamSynchronize(st));
                ctx->rowsall.release();
                ctx->rowsall = nb;
            }
            int64_t* dst = ctx->rowsall.as<int64_t>() + P_total * (uint64_t)(G + 1);
            if (ctx->rec_ib == 33) rc = materialize_dispatch<RecViewT<33>>(ctx, RecViewT<33>{rec + o}, mp, st, dst);
            else rc = materialize_dispatch<RecView>(ctx, RecView{rec + o}, mp, st, dst);
            if (rc) return rc;
        }
        P_total += Pc;
        groups += ctx->hc.ngroups;
    }
    HIPCHK(hipStreamSynchronize(st));
    ctx->P = P_total;
    ctx->st.probes = P_total;
    ctx->st.groups = groups;
    ctx->sorted_rec = rec;
    return MUMS_OK;
}

// the sharded FindMatches reads its probe rows from ctx->rowsall (built once per merge /
// restart) for a chunked merge and under enumeration tolerance > 1
int enum_count_check(mums_ctx* ctx, hipStream_t st);   // (after sort_row_keys below)

bool shard_rows_from_all(const mums_ctx* ctx) { return ctx->merge_chunked || ctx->enum_tol > 1 || ctx->pairwise; }

// Enumeration tolerance > 1 (and PairwiseMatchFinder's pairs) on a sharded rank (MemHash::EnumerateMatches, MemHash.cpp:139-162 ->
// MatchFinder::EnumerateMatches' odometer, MatchFinder.cpp:342-393): one probe row per
// AddHashEntry call of every group of the rank's key range, in key order (pairwise.hip
// en_count / en_emit over the records as full-key pairs, the run order already the std::sort
// order: mums_shard_tie_*).  ctx->P = the rows.
int shard_enum_rows(mums_ctx* ctx, hipStream_t st) {
    const uint64_t n = ctx->live_n;   // the live stream (after a restart: its live records)
    const int G = ctx->gt.G;
    const bool pw = ctx->pairwise;    // PairwiseMatchFinder (PairwiseMatchFinder.cpp:37-73): pair rows
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, pw ? 0 : ctx->masked, pw ? 0 : ctx->seq_mask};
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint32_t nb = (uint32_t)ctx->live_bst.size() - 1;
    const bool ib33 = ctx->rec_ib == 33;   // above 2^32 seed-mers: 64-bit indices
    HIPCHK(ctx->ckey.ensure(n * 8 + 64));
    HIPCHK(ctx->cval.ensure((ib33 ? 3 : 2) * (n + 64) * 4 + (uint64_t)(nb + 1) * 4));
    uint32_t* idx = ctx->cval.as<uint32_t>();
    uint32_t* ncalls = idx + (ib33 ? 2 : 1) * (n + 64);
    uint32_t* d_bst = ncalls + n + 64;
    HIPCHK(hipMemcpyAsync(d_bst, ctx->live_bst.data(), (uint64_t)(nb + 1) * 4, hipMemcpyHostToDevice, st));
    const int kb_rec = 2 * ctx->w + 1 - ctx->msd_bits;
    if (ib33)
        HIPCHK(launch_rec_pairs33(ctx->sorted_rec, n, d_bst, nb, ctx->shard_kfirst, kb_rec, ctx->ckey.as<uint64_t>(),
                                  (uint64_t*)idx, st));
    else
        HIPCHK(launch_rec_pairs(ctx->sorted_rec, n, d_bst, nb, ctx->shard_kfirst, kb_rec, ctx->ckey.as<uint64_t>(), idx,
                                st));
    const PairView<uint64_t> v{ctx->ckey.as<uint64_t>(), idx};
    const PairView<uint64_t, uint64_t> v64{ctx->ckey.as<uint64_t>(), (const uint64_t*)idx};
    HIPCHK(hipMemsetAsync(&dc->repeat_limit, 0, 8, st));
    if (pw && ib33) HIPCHK(launch_pairwise_count(v64, n, ctx->gt, ncalls, dc, st));
    else if (pw) HIPCHK(launch_pairwise_count(v, n, ctx->gt, ncalls, dc, st));
    else if (ib33) HIPCHK(launch_enum_count(v64, n, ctx->gt, mp, ncalls, dc, st));
    else HIPCHK(launch_enum_count(v, n, ctx->gt, mp, ncalls, dc, st));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(n + 1))));
    uint32_t* total = &dc->nprobes;
    HIPCHK(ctx->rowtmp.ensure((n + 64) * 4 + 4096));
    uint32_t* off = (uint32_t*)ctx->rowtmp.p;
    HIPCHK(hipMemcpyAsync(off, ncalls, n * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(exclusive_scan_u32(off, n, ctx->tmp.p, total, st));
    uint32_t P = 0;
    HIPCHK(hipMemcpyAsync(&P, total, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (int rc = enum_count_check(ctx, st)) return rc;
    HIPCHK(ctx->rowsall.ensure(((uint64_t)P + 1) * (G + 1) * 8));
    int64_t* rows = ctx->rowsall.as<int64_t>();
    if (pw && ib33) HIPCHK(launch_pairwise_emit(v64, n, ctx->gt, ctx->L, ncalls, off, rows, st));
    else if (pw) HIPCHK(launch_pairwise_emit(v, n, ctx->gt, ctx->L, ncalls, off, rows, st));
    else if (ib33) HIPCHK(launch_enum_emit(v64, n, ctx->gt, mp, ctx->L, ncalls, off, rows, st));
    else HIPCHK(launch_enum_emit(v, n, ctx->gt, mp, ctx->L, ncalls, off, rows, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->P = P;
    ctx->st.probes = P;
    ctx->shard_rows_built = true;
    return MUMS_OK;
}

// a chunked merge's probe rows for the sharded FindMatches (once per merge / restart)
int shard_chunk_rows(mums_ctx* ctx, hipStream_t st) {
    if (!shard_rows_from_all(ctx) || ctx->shard_rows_built) return MUMS_OK;
    if (ctx->enum_tol > 1 || ctx->pairwise) return shard_enum_rows(ctx, st);
    ProbeSpace ps{};
    int rc = ensure_probe_space(ctx, ctx->shard_n, seg_tiles_upper(ctx->shard_n, ctx->shard_mb), &ps);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, sizeof(DevCounters), st));
    rc = shard_groups_chunked(ctx, const_cast<uint64_t*>(ctx->sorted_rec), ctx->shard_bst, ps, true, st);
    if (rc) return rc;
    ctx->shard_rows_built = true;
    return MUMS_OK;
}

// the groups stage again over the nl live records at dst (bucket starts bst, 2^shard_mb + 1):
// the end of a sharded restart (mums_shard_restart_apply / _finish)
int shard_regroup(mums_ctx* ctx, uint64_t* dst, uint64_t nl, const std::vector<uint32_t>& bst, const ProbeSpace& ps,
                  uint64_t restarts, const uint64_t* offset_log, hipStream_t st) {
    const int mb = ctx->shard_mb;
    ctx->sorted_buf ^= 1;
    ctx->sorted_rec = dst;
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const uint64_t rep = ctx->hc.repeat_limit;
    if (ctx->merge_chunked) {   // the live stream's key chunks (seed-stage counts; rows on export)
        ctx->shard_bst = bst;
        ctx->shard_n = nl;
        ctx->live_n = nl;
        ctx->live_bst = bst;
        ctx->shard_rows_built = false;
        HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
        const int rc = shard_groups_chunked(ctx, dst, bst, ps, false, st);
        if (rc) return rc;
        const uint64_t P = ctx->P, groups = ctx->st.groups;
        ctx->hc.repeat_limit = rep;
        ctx->restarts = restarts;
        ctx->offset_log.assign(offset_log, offset_log + restarts * (uint64_t)ctx->gt.G);
        ctx->shard_restart_pending = false;
        shard_merge_stats(ctx, nl);
        ctx->P = P;
        ctx->st.probes = P;
        ctx->st.groups = groups;
        return MUMS_OK;
    }
    HIPCHK(hipMemcpyAsync(ctx->mstart.p, bst.data(), bst.size() * 4, hipMemcpyHostToDevice, st));
    ctx->live_n = nl;
    ctx->live_bst = bst;
    SegTile* tiles = ctx->tiles.as<SegTile>();
    HIPCHK(build_seg_tiles_from_starts(ctx->mstart.as<uint32_t>(), mb, nl, tiles, &dc->ntiles, ctx->tmp.p, st));
    HIPCHK(hipMemsetAsync(&dc->repeat_limit, 0, 8, st));
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    const uint64_t ub = seg_tiles_upper(nl, mb);
    int rc;
    if (ctx->rec_ib == 33)
        rc = groups_dispatch<RecViewT<33>>(ctx, RecViewT<33>{dst}, tiles, ub, mp, ps.probe_info, ps.probe_bucket,
                                           ps.slot_info, ps.slot_bucket, st);
    else
        rc = groups_dispatch<RecView>(ctx, RecView{dst}, tiles, ub, mp, ps.probe_info, ps.probe_bucket, ps.slot_info,
                                      ps.slot_bucket, st);
    if (rc) return rc;
    rc = finish_seeds(ctx, ps, st);
    if (rc) return rc;
    HIPCHK(h2d_sync(&dc->repeat_limit, &rep, 8, ctx->stream));   // the report: the whole range's groups
    ctx->hc.repeat_limit = rep;
    ctx->restarts = restarts;
    ctx->offset_log.assign(offset_log, offset_log + restarts * (uint64_t)ctx->gt.G);
    ctx->shard_restart_pending = false;
    HIPCHK(hipStreamSynchronize(st));
    shard_merge_stats(ctx, ctx->shard_n);
    return MUMS_OK;
}
}  // namespace

extern "C" {

int mums_shard_merge(mums_ctx* ctx, const uint64_t* d_records, uint32_t nsources, uint32_t first_bucket,
                     uint32_t nbuckets, const uint64_t* counts) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = prepare_shard(ctx);
    if (rc) return rc;
    const int B = ctx->msd_bits;
    if (nsources == 0 || (uint64_t)first_bucket + nbuckets > (1ull << B) || (nbuckets && !counts))
        return fail(ctx, MUMS_E_INVALID, "bad shard merge arguments");
    if (!ctx->start_points.empty() && ctx->start_points.size() != (size_t)ctx->gt.G)   // MatchFinder.cpp:197-199
        return fail(ctx, MUMS_E_INVALID, "start points: one per sequence (all genomes of the shard layout) required");
    ctx->shard_restart_pending = false;
    hipStream_t st = ctx->stream;
    // chunk table: received source-major (each source's buckets in order) -> bucket-major
    std::vector<uint64_t> tot(nbuckets, 0), chunks;
    uint64_t n = 0;
    for (uint32_t s = 0; s < nsources; ++s)
        for (uint32_t b = 0; b < nbuckets; ++b) tot[b] += counts[(uint64_t)s * nbuckets + b];
    for (uint32_t b = 0; b < nbuckets; ++b) n += tot[b];
    if (n && !d_records) return fail(ctx, MUMS_E_INVALID, "null record buffer");
    if (n >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 records per shard");
    const int mb = ceil_log2(nbuckets);
    std::vector<uint32_t> bst((1ull << mb) + 1, (uint32_t)n);
    {
        std::vector<uint64_t> srcoff(nsources + 1, 0);
        for (uint32_t s = 0; s < nsources; ++s) {
            uint64_t c = 0;
            for (uint32_t b = 0; b < nbuckets; ++b) c += counts[(uint64_t)s * nbuckets + b];
            srcoff[s + 1] = srcoff[s] + c;
        }
        std::vector<uint64_t> inner(nsources, 0);   // running offset inside each source's block
        uint64_t dst = 0;
        for (uint32_t b = 0; b < nbuckets; ++b) {
            bst[b] = (uint32_t)dst;
            for (uint32_t s = 0; s < nsources; ++s) {
                const uint64_t len = counts[(uint64_t)s * nbuckets + b];
                if (len) {
                    chunks.push_back(srcoff[s] + inner[s]);
                    chunks.push_back(dst);
                    chunks.push_back(len);
                }
                inner[s] += len;
                dst += len;
            }
        }
    }
    ProbeSpace ps{};
    rc = ensure_merge_space(ctx, n, mb, 2 * ctx->w + 1 - B, &ps);
    if (rc) return rc;
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    HIPCHK(ctx->keybuf.ensure(std::max<size_t>(chunks.size(), 1) * 8));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    if (ctx->profiling && !ctx->ev_ds[0])
        for (int i = 0; i < 16; ++i) HIPCHK(hipEventCreate(&ctx->ev_ds[i]));
    HIPCHK(h2d_sync(ctx->keybuf.p, chunks.data(), chunks.size() * 8, ctx->stream));
    HIPCHK(h2d_sync(ctx->mstart.p, bst.data(), bst.size() * 4, ctx->stream));
    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    HIPCHK(launch_regroup(d_records, ctx->recA.as<uint64_t>(), ctx->keybuf.as<uint64_t>(),
                          (uint32_t)(chunks.size() / 3), n, st));
    HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    ctx->N = n;
    // a key range above one onesweep merge (2^30 records: BASELINE config 5 on 2 or 4 GPUs)
    // is merged in chunks of consecutive buckets, in key order (seed-stage counts only)
    uint64_t cap = (1ull << 30) - 4096;
    if (const char* e = getenv("MUMS_DEV_CHUNK_RECORDS")) cap = std::min<uint64_t>(cap, strtoull(e, nullptr, 10));
    ctx->merge_chunked = n >= cap;
    uint64_t P_total = 0, groups = 0;
    if (!ctx->merge_chunked) {
        rc = merge_stage(ctx, n, mb, 2 * ctx->w + 1 - B, mp, ps, st, ctx->rec_ib);
        if (rc) return rc;
        rc = finish_seeds(ctx, ps, st);
        if (rc) return rc;
    } else {
        const uint32_t nbk = 1u << mb;
        uint32_t b0 = 0;
        while (b0 < nbuckets) {
            uint32_t b1 = b0;
            while (b1 < nbuckets && (uint64_t)bst[b1 + 1] - bst[b0] < cap) ++b1;
            if (b1 == b0) return fail(ctx, MUMS_E_UNSUPPORTED, "one MSD bucket holds more than 2^30 records");
            const uint64_t o = bst[b0], nc = (uint64_t)bst[b1] - o;
            std::vector<uint32_t> sub(nbk + 1);
            for (uint32_t b = 0; b <= nbk; ++b)
                sub[b] = b < b0 ? 0u : (b < b1 ? (uint32_t)(bst[b] - o) : (uint32_t)nc);
            HIPCHK(h2d_sync(ctx->mstart.p, sub.data(), sub.size() * 4, ctx->stream));
            rc = merge_stage(ctx, nc, mb, 2 * ctx->w + 1 - B, mp, ps, st, ctx->rec_ib, ctx->recA.as<uint64_t>() + o,
                             ctx->recB.as<uint64_t>() + o);
            if (rc) return rc;
            rc = finish_seeds(ctx, ps, st);
            if (rc) return rc;
            P_total += ctx->P;
            groups += ctx->hc.ngroups;
            b0 = b1;
        }
        // every chunk sorted in place with the same pass count: the whole range's stream
        ctx->sorted_rec = ctx->sorted_buf ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>();
    }
    ctx->shard_rows_built = false;
    // a group above MER_REPEAT_LIMIT (or start points): the restart moves start points of
    // every later key, on every rank -> planned on the whole stream (mums_shard_restart_*)
    ctx->restarts = 0;
    ctx->offset_log.clear();
    // (repeat tolerance: every run of equal keys in std::sort order, mums_shard_tie_*, first)
    // (LogProgress: the text is restated by the gathered plan on rank 0, over the whole stream)
    ctx->shard_restart_pending =
        ctx->hc.repeat_limit > 0 || have_start_points(ctx) || wants_tie_order(ctx) || ctx->progress_on;
    ctx->shard_mb = mb;
    ctx->shard_n = n;
    ctx->shard_kfirst = first_bucket;
    ctx->shard_kcount = nbuckets;
    ctx->shard_bst = bst;
    ctx->live_n = n;
    ctx->live_bst = bst;
    ctx->ds_ready = false;
    ctx->stage_done = MUMS_STAGE_SEEDS;
    HIPCHK(hipStreamSynchronize(st));
    shard_merge_stats(ctx, n);
    if (ctx->merge_chunked) {
        ctx->P = P_total;
        ctx->st.probes = P_total;
        ctx->st.groups = groups;
    }
    return MUMS_OK;
}

int mums_shard_restart_pending(mums_ctx* ctx, uint64_t* pending) {
    if (check_ctx(ctx) || !pending) return MUMS_E_INVALID;
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded merge run");
    *pending = ctx->shard_restart_pending ? std::max<uint64_t>(ctx->hc.repeat_limit, 1) : 0;
    return MUMS_OK;
}

int mums_shard_stream(mums_ctx* ctx, const void** d_records, uint64_t* n) {
    if (check_ctx(ctx) || !d_records || !n) return MUMS_E_INVALID;
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS || ctx->merge_chunked)
        return fail(ctx, MUMS_E_INVALID, "no sharded (one-pass) merge run");
    *d_records = ctx->sorted_rec;
    *n = ctx->shard_n;
    return MUMS_OK;
}

// The planner (one rank) on the ranks' merged streams gathered in rank order (= key order):
// MSD digit starts from the keys stage's per-rank bucket counts, one segment per rank, then
// stream_restart; every rank's block {n_live, nbst, nbst bucket starts, live records}.
int mums_shard_restart_plan(mums_ctx* ctx, uint64_t* d_stream, uint32_t nranks, const uint64_t* counts,
                            const uint32_t* first_bucket, const uint32_t* nbuckets, void* d_out,
                            uint64_t capacity_bytes, uint64_t* block_bytes) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded merge run");
    if (nranks == 0 || !counts || !first_bucket || !nbuckets || !block_bytes || !d_out)
        return fail(ctx, MUMS_E_INVALID, "bad restart plan arguments");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int B = ctx->msd_bits;
    const uint64_t nb = 1ull << B;
    std::vector<uint64_t> dstart(nb + 1, 0);
    for (uint64_t b = 0; b < nb; ++b) {
        uint64_t t = 0;
        for (uint32_t r = 0; r < nranks; ++r) t += counts[(uint64_t)r * nb + b];
        dstart[b + 1] = dstart[b] + t;
    }
    const uint64_t N = dstart[nb];
    std::vector<RestartSeg> segs(nranks);
    std::vector<int> mbs(nranks);
    uint64_t need = 0, expect = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
        if ((uint64_t)first_bucket[r] + nbuckets[r] > nb || first_bucket[r] != expect)
            return fail(ctx, MUMS_E_INVALID, "restart plan: key ranges must tile the buckets in rank order");
        expect = first_bucket[r] + nbuckets[r];
        mbs[r] = ceil_log2(nbuckets[r]);
        segs[r] = RestartSeg{dstart[first_bucket[r]], dstart[expect], 1u << mbs[r]};
        if (segs[r].hi - segs[r].lo >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 records per shard");
        need += 8 * (2 + (uint64_t)segs[r].nb + 1 + (segs[r].hi - segs[r].lo));
    }
    if (expect != nb) return fail(ctx, MUMS_E_INVALID, "restart plan: key ranges must cover every bucket");
    if (need > capacity_bytes) return fail(ctx, MUMS_E_INVALID, "restart plan: output buffer too small");
    if (N && !d_stream) return fail(ctx, MUMS_E_INVALID, "null stream");
    const uint64_t n_own = ctx->N;
    HIPCHK(ctx->crall.ensure((N + 64) * 8));
    uint64_t nbst = 0;
    for (const RestartSeg& g : segs) nbst += g.nb + 1;
    HIPCHK(ctx->rsbst.ensure(nbst * 4 + 64));
    ctx->N = N;   // stream_restart's stream: the whole merged stream (restored below)
    std::vector<uint64_t> n_live;
    bool live = false;
    std::vector<uint32_t> hb;
    const int kb = 2 * ctx->w + 1 - B;
    int rc = stream_restart(ctx, d_stream, ctx->crall.as<uint64_t>(), dstart, (uint32_t)kb, (uint32_t)ctx->rec_ib, segs,
                            [&](uint32_t r, uint32_t* d) -> int {
        hb.assign(segs[r].nb + 1, (uint32_t)(segs[r].hi - segs[r].lo));
        for (uint32_t b = 0; b < nbuckets[r]; ++b) hb[b] = (uint32_t)(dstart[first_bucket[r] + b] - segs[r].lo);
        HIPCHK(h2d_sync(d, hb.data(), hb.size() * 4, ctx->stream));
        return MUMS_OK;
    }, ctx->rsbst.as<uint32_t>(), n_live, &live, st);
    ctx->N = n_own;
    if (rc) return rc;
    // blocks: header words, bucket starts widened to 64 bits, records
    const uint64_t* src = live ? ctx->crall.as<uint64_t>() : d_stream;
    std::vector<uint32_t> all_bst(nbst);
    if (live) HIPCHK(hipMemcpy(all_bst.data(), ctx->rsbst.p, nbst * 4, hipMemcpyDeviceToHost));
    uint64_t o = 0, bo = 0;
    char* out = (char*)d_out;
    for (uint32_t r = 0; r < nranks; ++r) {
        const uint64_t nl = live ? n_live[r] : segs[r].hi - segs[r].lo;
        std::vector<uint64_t> head(2 + segs[r].nb + 1);
        head[0] = nl;
        head[1] = segs[r].nb + 1;
        for (uint64_t b = 0; b <= segs[r].nb; ++b) {
            uint64_t v;
            if (live) v = all_bst[bo + b];
            else v = b < nbuckets[r] ? dstart[first_bucket[r] + b] - segs[r].lo : segs[r].hi - segs[r].lo;
            head[2 + b] = v;
        }
        bo += segs[r].nb + 1;
        HIPCHK(h2d_sync(out + o, head.data(), head.size() * 8, ctx->stream));
        o += head.size() * 8;
        if (nl) HIPCHK(hipMemcpyAsync(out + o, src + segs[r].lo, nl * 8, hipMemcpyDeviceToDevice, st));
        o += nl * 8;
        block_bytes[r] = 8 * (head.size() + nl);
    }
    HIPCHK(hipStreamSynchronize(st));
    note_rs_bytes(ctx);
    ctx->crall.release();
    return MUMS_OK;
}

// Every rank: its block from the planner -> the live records replace the merged stream,
// the groups stage runs again (as restart_stage does on one context).
int mums_shard_restart_apply(mums_ctx* ctx, const void* d_block, uint64_t restarts, const uint64_t* offset_log) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS || ctx->merge_chunked)
        return fail(ctx, MUMS_E_INVALID, "no sharded (one-pass) merge run");
    if (!d_block || (restarts && !offset_log)) return fail(ctx, MUMS_E_INVALID, "bad restart block");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int mb = ctx->shard_mb;
    uint64_t head[2] = {0, 0};
    HIPCHK(hipMemcpy(head, d_block, 16, hipMemcpyDeviceToHost));
    const uint64_t nl = head[0];
    if (head[1] != (1ull << mb) + 1 || nl > ctx->shard_n)
        return fail(ctx, MUMS_E_INVALID, "restart block does not match this rank's merge");
    std::vector<uint64_t> b64(head[1]);
    HIPCHK(hipMemcpy(b64.data(), (const uint64_t*)d_block + 2, head[1] * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> bst(head[1]);
    for (uint64_t b = 0; b < head[1]; ++b) bst[b] = (uint32_t)b64[b];
    const int B = ctx->msd_bits;
    const int kb = 2 * ctx->w + 1 - B;
    ProbeSpace ps{};
    int rc = ensure_merge_space(ctx, ctx->shard_n, mb, kb, &ps);
    if (rc) return rc;
    uint64_t* dst = ctx->sorted_buf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>();
    if (nl) HIPCHK(hipMemcpyAsync(dst, (const uint64_t*)d_block + 2 + head[1], nl * 8, hipMemcpyDeviceToDevice, st));
    ctx->rs_info[0] = 2;
    ctx->rs_info[2] = restarts;
    return shard_regroup(ctx, dst, nl, bst, ps, restarts, offset_log, st);
}

// ---- the restart planned where the records are (mums_shard_restart_counts .. _finish) ----
// Rank r's merged stream holds every genome's SML indices [off_r[g], off_r[g] + n_r[g]) (the
// key ranges ascend with the rank), so its part of genome g's SortedMerList is its records
// of genome g in stream order.  Those parts answer the plan's reads (PlanData's distributed
// form); the restarts of lower ranks arrive as the running start points.

int mums_shard_restart_counts(mums_ctx* ctx, uint64_t* info) {
    if (check_ctx(ctx) || !info) return MUMS_E_INVALID;
    if (!have_device()) return fail(ctx, MUMS_E_NODEVICE, "no HIP device");
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded merge run");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G, n = ctx->shard_n;
    const int B = ctx->msd_bits;
    const uint32_t kb = (uint32_t)(2 * ctx->w + 1 - B);
    std::fill(info, info + 3 * Gu + 1, 0ull);
    ctx->ds_ready = false;
    ctx->rs_info[0] = ctx->rs_info[1] = ctx->rs_info[2] = ctx->rs_info[3] = 0;
    if (ctx->parity_masked || seg_onesweep_launches(kb) < (int)((kb + 7) / 8))
        return fail(ctx, MUMS_E_UNSUPPORTED, "restart with the segment fix-up sort (MUMS_DEV_SEGFIX)");
    const char* force = getenv("MUMS_DEV_SHARD_RESTART");
    if (ctx->progress_on || (force && !strcmp(force, "gather"))) {   // LogProgress needs the whole stream
        if (wants_tie_order(ctx))
            return fail(ctx, MUMS_E_UNSUPPORTED, "sharded repeat / enumeration tolerance: the gathered plan (LogProgress) "
                                                 "does not order every run of equal keys");
        if (ctx->merge_chunked)
            return fail(ctx, MUMS_E_UNSUPPORTED, "sharded restart after a chunked merge: the gathered plan (LogProgress) "
                                                 "needs one merge per rank");
        info[3 * Gu] = 1;
        return MUMS_OK;
    }
    // the local stream: 2^B global digit starts around this rank's buckets
    const uint64_t nd = 1ull << B;
    std::vector<uint64_t> dstart(nd + 1, 0);
    for (uint64_t d = 0; d <= nd; ++d) {
        if (d < ctx->shard_kfirst) dstart[d] = 0;
        else if (d - ctx->shard_kfirst <= ctx->shard_kcount) dstart[d] = ctx->shard_bst[d - ctx->shard_kfirst];
        else dstart[d] = n;
    }
    const uint64_t ccap = n / (restart::kRepeatLimit + 1) + 16;
    HIPCHK(ctx->crbuf.ensure((nd + 1) * 8 + 64 + ccap * 8 + 4096));
    uint64_t* d_dstart = ctx->crbuf.as<uint64_t>();
    unsigned long long* d_cnt = (unsigned long long*)(d_dstart + nd + 1);
    uint64_t* d_list = (uint64_t*)(d_cnt + 8);
    HIPCHK(hipMemcpyAsync(d_dstart, dstart.data(), (nd + 1) * 8, hipMemcpyHostToDevice, st));
    CrStream s{ctx->sorted_rec, d_dstart, (uint32_t)nd, n};
    s.kb = kb;
    s.ib = (uint32_t)ctx->rec_ib;
    HIPCHK(launch_cr_cands(s, d_list, d_cnt, ccap, st));
    unsigned long long C = 0;
    HIPCHK(hipMemcpyAsync(&C, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (C > ccap) return fail(ctx, MUMS_E_HIP, "restart: candidate list overflow (internal error)");
    if (C) {
        std::vector<uint64_t> cand(C);
        HIPCHK(hipMemcpy(cand.data(), d_list, C * 8, hipMemcpyDeviceToHost));
        std::sort(cand.begin(), cand.end());
        HIPCHK(h2d_sync(d_list, cand.data(), C * 8, ctx->stream));
    }
    ctx->ds_C = C;
    // per-genome block counts, this rank's part of every SML (full keys, genome-major)
    const uint64_t nblk = cr_blocks(n);
    HIPCHK(ctx->crcnt.ensure(Gu * (nblk + 1) * 4 + 256));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nblk + 2))));
    uint32_t* gscan = ctx->crcnt.as<uint32_t>();
    HIPCHK(launch_cr_counts(s, gt, gscan, ctx->tmp.p, st));
    std::vector<uint32_t> tot(Gu, 0);
    for (int g = 0; g < G; ++g)
        HIPCHK(hipMemcpyAsync(&tot[g], gscan + (uint64_t)g * (nblk + 1) + nblk, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->ds_n.assign(Gu, 0);
    std::vector<uint64_t> lbase(Gu + 1, 0);
    for (int g = 0; g < G; ++g) {
        ctx->ds_n[g] = tot[g];
        lbase[g + 1] = lbase[g] + tot[g];
    }
    if (lbase[G] != n) return fail(ctx, MUMS_E_HIP, "restart: genome counts differ from the stream (internal error)");
    HIPCHK(ctx->dsarr.ensure(8 * (10 * (Gu + 1) + 64)));
    ctx->ds_ties = false;
    uint64_t* d_lbase = ctx->dsarr.as<uint64_t>() + (Gu + 1);
    HIPCHK(hipMemcpyAsync(d_lbase, lbase.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(ctx->crall.ensure((n + 64) * 8));
    uint64_t* ck = ctx->crall.as<uint64_t>();
    HIPCHK(launch_cr_ck(s, gt, gscan, ck, st, d_lbase));
    for (int g = 0; g < G; ++g) {
        info[g] = tot[g];
        info[Gu + g] = ~0ull;
        if (!tot[g]) continue;
        HIPCHK(hipMemcpyAsync(&info[Gu + g], ck + lbase[g], 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&info[2 * Gu + g], ck + lbase[g + 1] - 1, 8, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    ctx->rs_info[1] = C;
    return MUMS_OK;
}

}  // extern "C"

namespace {
// device arrays of the distributed plan in ctx->dsarr (G + 1 words each)
struct DsArrays {
    uint64_t *dm, *lbase, *off, *n, *prv, *nxt, *S0;
    unsigned* bad;
};
DsArrays ds_arrays(mums_ctx* ctx) {
    const uint64_t W = (uint64_t)ctx->gt.G + 1;
    uint64_t* b = ctx->dsarr.as<uint64_t>();
    return DsArrays{b, b + W, b + 2 * W, b + 3 * W, b + 4 * W, b + 5 * W, b + 6 * W, (unsigned*)(b + 7 * W)};
}
restart::PlanData ds_plan_data(mums_ctx* ctx, const DsArrays& a) {
    restart::PlanData d{ctx->gt.G, a.dm, a.lbase, ctx->crall.as<uint64_t>()};
    d.off = a.off;
    d.n = a.n;
    d.prv = a.prv;
    d.nxt = a.nxt;
    const int sh = 2 * ctx->w + 1 - ctx->msd_bits;
    const uint64_t end = (uint64_t)ctx->shard_kfirst + ctx->shard_kcount;
    d.key_lo = (uint64_t)ctx->shard_kfirst << sh;
    d.key_hi = end >= (1ull << ctx->msd_bits) ? ~0ull : end << sh;
    d.bad = a.bad;
    return d;
}
// plan workspace in ctx->rsplan: [pre 3 C G + C/2][cbad C/2 + 1][S G][PlanOut][rkey C][rS C G]
struct DsPlan {
    uint64_t* pre;
    unsigned* cbad;
    uint64_t* S;
    restart::PlanOut* out;
    uint64_t *rkey, *rS;
};
DsPlan ds_plan(mums_ctx* ctx, uint64_t cap) {
    const uint64_t Gu = (uint64_t)ctx->gt.G;
    uint64_t* p = ctx->rsplan.as<uint64_t>();
    DsPlan w{};
    w.pre = p;
    p += 3 * cap * Gu + (cap + 1) / 2 + 1;
    w.cbad = (unsigned*)p;
    p += (cap + 1) / 2 + 1;
    w.S = p;
    p += Gu + 1;
    w.out = (restart::PlanOut*)p;
    p += (sizeof(restart::PlanOut) + 7) / 8 + 1;
    w.rkey = p;
    p += cap;
    w.rS = p;
    return w;
}
size_t ds_plan_bytes(uint64_t cap, uint64_t Gu) {
    return 8 * (3 * cap * Gu + (cap + 1) + 4 + Gu + 1 + (sizeof(restart::PlanOut) + 7) / 8 + 1 + cap + cap * Gu) + 4096;
}
// word offset of genome g in the all-gathered packed genomes (layout_packed over every genome;
// the context's own packed array holds only its genomes)
uint64_t all_woff(const GenomeTable& gt, int g) {
    GenomeTable t = gt;
    uint64_t words = 0;
    (void)layout_packed(t, &words);
    return t.woff[g];
}

// the restart's own device buffers (mums_shard_restart_info; the tie replay's workspace, O(the
// genome) on the rank replaying it, is not counted)
void note_rs_bytes(mums_ctx* ctx) {
    uint64_t b = 0;
    for (const DevBuf* x : {&ctx->crall, &ctx->crcnt, &ctx->crlive, &ctx->crruns, &ctx->rsplan, &ctx->crbuf,
                            &ctx->rsbst, &ctx->dsarr})
        b += x->cap;
    ctx->rs_info[3] = std::max<uint64_t>(ctx->rs_info[3], b);
}
}  // namespace

extern "C" {

int mums_shard_restart_prepare(mums_ctx* ctx, uint32_t nranks, uint32_t rank, const uint64_t* all_info, uint64_t* S0) {
    if (check_ctx(ctx) || !all_info || !S0 || rank >= nranks) return MUMS_E_INVALID;
    if (ctx->ds_n.size() != (size_t)ctx->gt.G || !ctx->crall.p)
        return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_counts first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G, rowlen = 3 * Gu + 1;
    std::vector<uint64_t> hm(Gu + 1, 0), off(Gu + 1, 0), hn(Gu + 1, 0), prv(Gu + 1, 0), nxt(Gu + 1, ~0ull),
        s0(Gu + 1, 0);
    for (int g = 0; g < G; ++g) {
        hm[g] = gt.m[g];
        uint64_t t = 0;
        for (uint32_t r = 0; r < nranks; ++r) {
            const uint64_t* row = all_info + (uint64_t)r * rowlen;
            if (r < rank) off[g] += row[g];
            t += row[g];
            if (r < rank && row[g]) prv[g] = row[2 * Gu + g];
        }
        for (uint32_t r = nranks; r-- > rank + 1;) {
            const uint64_t* row = all_info + (uint64_t)r * rowlen;
            if (row[g]) nxt[g] = row[Gu + g];
        }
        if (t != gt.m[g] || all_info[(uint64_t)rank * rowlen + g] != ctx->ds_n[g])
            return fail(ctx, MUMS_E_INVALID, "restart: the ranks' SML counts do not add up to the genome");
        hn[g] = ctx->ds_n[g];
        s0[g] = g < (int)ctx->start_points.size() ? ctx->start_points[g] : 0;
        S0[g] = s0[g];
    }
    ctx->ds_off.assign(off.begin(), off.begin() + Gu);
    const DsArrays a = ds_arrays(ctx);
    HIPCHK(hipMemcpyAsync(a.dm, hm.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.off, off.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.n, hn.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.prv, prv.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.nxt, nxt.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.S0, s0.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    const uint64_t C = ctx->ds_C, cap = C + 16;
    HIPCHK(ctx->rsplan.ensure(ds_plan_bytes(cap, Gu)));
    const DsPlan w = ds_plan(ctx, cap);
    const uint64_t nd = 1ull << ctx->msd_bits;
    const uint64_t* d_list = (const uint64_t*)((unsigned long long*)(ctx->crbuf.as<uint64_t>() + nd + 1) + 8);
    HIPCHK(launch_restart_dpre(ds_plan_data(ctx, a), d_list, C, w.pre, w.cbad, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->ds_ready = true;
    note_rs_bytes(ctx);
    return MUMS_OK;
}

int mums_shard_restart_step(mums_ctx* ctx, uint64_t* S, uint64_t* restarts, uint64_t* undecidable) {
    if (check_ctx(ctx) || !S || !restarts || !undecidable) return MUMS_E_INVALID;
    if (!ctx->ds_ready) return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_prepare first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const uint64_t Gu = (uint64_t)ctx->gt.G, C = ctx->ds_C, cap = C + 16;
    *restarts = 0;
    *undecidable = 0;
    ctx->ds_rkey.clear();
    ctx->ds_rS.clear();
    if (C == 0) return MUMS_OK;   // the start points pass through
    const DsArrays a = ds_arrays(ctx);
    const DsPlan w = ds_plan(ctx, cap);
    restart::PlanOut po{};
    po.cap = C;
    po.rkey = w.rkey;
    po.rS = w.rS;
    po.status = restart::kPlanOk;
    const unsigned zero = 0;
    HIPCHK(hipMemcpyAsync(w.S, S, Gu * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(w.out, &po, sizeof(po), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(a.bad, &zero, 4, hipMemcpyHostToDevice, st));
    const uint64_t nd = 1ull << ctx->msd_bits;
    const uint64_t* d_list = (const uint64_t*)((unsigned long long*)(ctx->crbuf.as<uint64_t>() + nd + 1) + 8);
    HIPCHK(launch_restart_dplan(ds_plan_data(ctx, a), d_list, C, w.pre, w.cbad, w.S, w.out, st));
    unsigned bad = 0;
    HIPCHK(hipMemcpyAsync(&po, w.out, sizeof(po), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&bad, a.bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(S, w.S, Gu * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (po.status != restart::kPlanOk) return fail(ctx, MUMS_E_HIP, "restart plan table full (internal error)");
    const uint64_t R = po.nrestarts;
    ctx->ds_rkey.assign(R, 0);
    ctx->ds_rS.assign(R * Gu, 0);
    if (R) {
        HIPCHK(hipMemcpy(ctx->ds_rkey.data(), w.rkey, R * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(ctx->ds_rS.data(), w.rS, R * Gu * 8, hipMemcpyDeviceToHost));
    }
    *restarts = R;
    *undecidable = bad ? 1 : 0;
    // test hook: the step reports an undecidable plan (a read beyond the rank's neighbours)
    const char* force = getenv("MUMS_DEV_SHARD_RESTART");
    if (force && !strcmp(force, "undecidable")) *undecidable = 1;
    return MUMS_OK;
}

int mums_shard_restart_log(mums_ctx* ctx, uint64_t* rkey, uint64_t* rS) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!ctx->ds_rkey.empty() && (!rkey || !rS)) return MUMS_E_INVALID;
    std::copy(ctx->ds_rkey.begin(), ctx->ds_rkey.end(), rkey);
    std::copy(ctx->ds_rS.begin(), ctx->ds_rS.end(), rS);
    return MUMS_OK;
}

int mums_shard_restart_runs(mums_ctx* ctx, uint64_t R, const uint64_t* rkey, const uint64_t* rS, uint64_t* runs,
                            uint64_t capacity, uint64_t* nruns) {
    if (check_ctx(ctx) || !nruns || (R && (!rkey || !rS)) || (capacity && !runs)) return MUMS_E_INVALID;
    if (!ctx->ds_ready) return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_prepare first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const uint64_t Gu = (uint64_t)ctx->gt.G, rows = R + 1, rcap = rows * Gu + 16;
    HIPCHK(ctx->crruns.ensure(rcap * 24 + rows * Gu * 8 + 256));
    uint64_t* d_runs = ctx->crruns.as<uint64_t>();
    uint64_t* d_sp = d_runs + 3 * rcap;
    unsigned long long* d_cnt = (unsigned long long*)(d_sp + rows * Gu);
    const DsArrays a = ds_arrays(ctx);
    HIPCHK(hipMemcpyAsync(d_sp, a.S0, Gu * 8, hipMemcpyDeviceToDevice, st));
    if (R) HIPCHK(hipMemcpyAsync(d_sp + Gu, rS, R * Gu * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(d_cnt, 0, 8, st));
    HIPCHK(launch_cr_druns(ctx->crall.as<uint64_t>(), ctx->gt.G, a.lbase, a.off, a.n, d_sp, rows, d_runs, d_cnt, rcap,
                           st));
    unsigned long long nr = 0;
    HIPCHK(hipMemcpyAsync(&nr, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));   // (rS is the caller's host array)
    if (nr > rcap) return fail(ctx, MUMS_E_HIP, "restart: run list overflow (internal error)");
    std::vector<std::array<uint64_t, 3>> v(nr);
    if (nr) HIPCHK(hipMemcpy(v.data(), d_runs, nr * 24, hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    *nruns = v.size();
    for (uint64_t q = 0; q < v.size() && q < capacity / 3; ++q)
        for (int k = 0; k < 3; ++k) runs[3 * q + k] = v[q][k];
    return v.size() * 3 > capacity ? fail(ctx, MUMS_E_INVALID, "run buffer too small") : MUMS_OK;
}

int mums_shard_restart_ties(mums_ctx* ctx, const uint32_t* d_packed_all, const uint64_t* runs, uint64_t nruns,
                            const uint64_t* vofs, uint32_t* d_out) {
    if (check_ctx(ctx) || (nruns && (!d_packed_all || !runs || !vofs || !d_out))) return MUMS_E_INVALID;
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded merge run");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const GenomeTable& gt = ctx->gt;
    for (int g = 0; g < gt.G; ++g) {
        bool any = false;
        for (uint64_t q = 0; q < nruns; ++q) any = any || (int)runs[3 * q] == g;
        if (!any) continue;
        const uint64_t m = gt.m[g];
        if (m >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList of more than 2^32 seed-mers");
        for (uint64_t q = 0; q < nruns; ++q)
            if ((int)runs[3 * q] == g && (runs[3 * q + 1] >= runs[3 * q + 2] || runs[3 * q + 2] > m))
                return fail(ctx, MUMS_E_INVALID, "restart: bad run");
        if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess) {
            (void)hipGetLastError();
            HIPCHK(hipStreamSynchronize(st));
            release_find_buffers(ctx);   // the previous FindMatches' tail buffers are dead here
            if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess)
                return fail(ctx, MUMS_E_NOMEM, "restart: no device memory for the SortedMerList tie order of a genome");
        }
        note_rs_bytes(ctx);
        const TieWs tw = tie_ws_layout(ctx->tiebuf.p, m, 1);
        const uint64_t b0 = 0;
        HIPCHK(tie_set_genomes(tw, &b0, &m, st));
        HIPCHK(tie_clear_flags(tw, st));
        for (uint64_t q = 0; q < nruns; ++q) {   // pair flags of every run: slots [lo, hi - 1)
            if ((int)runs[3 * q] != g) continue;
            const uint64_t lo = runs[3 * q + 1], hi = runs[3 * q + 2];
            if (hi - lo >= 2) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(tw.pf + lo), 1u, hi - 1 - lo, st));
        }
        uint64_t flagged = 0;
        HIPCHK(tie_prepare(tw, &flagged, st));
        if (flagged) {
            HIPCHK(launch_keys_of_genome(ctx->ss, d_packed_all + all_woff(gt, g), m, tw.K, st, false));
            HIPCHK(tie_replay(tw, st));
            ctx->tie_slots += flagged;
        }
        for (uint64_t q = 0; q < nruns; ++q) {
            if ((int)runs[3 * q] != g) continue;
            const uint64_t lo = runs[3 * q + 1], hi = runs[3 * q + 2];
            HIPCHK(hipMemcpyAsync(d_out + vofs[q], tw.V + lo, (hi - lo) * 4, hipMemcpyDeviceToDevice, st));
        }
        HIPCHK(hipStreamSynchronize(st));
    }
    if (nruns) {
        HIPCHK(hipStreamSynchronize(st));
        release_tiebuf(ctx);
    }
    return MUMS_OK;
}

int mums_shard_restart_finish(mums_ctx* ctx, uint64_t R, const uint64_t* rkey, const uint64_t* rS,
                              const uint64_t* runs, uint64_t nruns, const uint32_t* d_pos, const uint64_t* vofs) {
    if (check_ctx(ctx) || (R && (!rkey || !rS)) || (nruns && (!runs || !d_pos || !vofs))) return MUMS_E_INVALID;
    if (!ctx->ds_ready) return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_prepare first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const GenomeTable& gt = ctx->gt;
    const uint64_t Gu = (uint64_t)gt.G, n = ctx->shard_n;
    const int B = ctx->msd_bits, mb = ctx->shard_mb;
    const int kb = 2 * ctx->w + 1 - B;
    ctx->rs_info[0] = 1;
    ctx->rs_info[2] = R;
    auto done = [&]() {
        for (DevBuf* b : {&ctx->crall, &ctx->crcnt, &ctx->crlive, &ctx->crruns, &ctx->rsplan, &ctx->crbuf})
            b->release();
        ctx->ds_ready = false;
    };
    if (R == 0 && !have_start_points(ctx) && !ctx->ds_ties) {   // nothing moves: the stream and its groups stand
        note_rs_bytes(ctx);
        done();
        ctx->restarts = 0;
        ctx->offset_log.clear();
        ctx->shard_restart_pending = false;
        return MUMS_OK;
    }
    const uint64_t nd = 1ull << B;
    CrStream s{ctx->sorted_rec, ctx->crbuf.as<uint64_t>(), (uint32_t)nd, n};
    s.kb = (uint32_t)kb;
    s.ib = (uint32_t)ctx->rec_ib;
    const DsArrays a = ds_arrays(ctx);
    // device copies: runs + offsets, restart keys, start points of every phase
    const uint64_t words = 3 * nruns + nruns + R + R * Gu + 64;
    HIPCHK(ctx->crruns.ensure(words * 8 + 256));
    uint64_t* d_runs = ctx->crruns.as<uint64_t>();
    uint64_t* d_vofs = d_runs + 3 * nruns;
    uint64_t* d_rkey = d_vofs + nruns;
    uint64_t* d_rS = d_rkey + R;
    if (nruns) {
        HIPCHK(hipMemcpyAsync(d_runs, runs, 3 * nruns * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_vofs, vofs, nruns * 8, hipMemcpyHostToDevice, st));
    }
    if (R) {
        HIPCHK(hipMemcpyAsync(d_rkey, rkey, R * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_rS, rS, R * Gu * 8, hipMemcpyHostToDevice, st));
    }
    HIPCHK(launch_cr_dtie_write(s, gt, d_runs, nruns, ctx->crall.as<uint64_t>(), a.lbase, a.off, d_pos, d_vofs,
                                const_cast<uint64_t*>(ctx->sorted_rec), st));
    ProbeSpace ps{};
    int rc = ensure_merge_space(ctx, n, mb, kb, &ps);
    if (rc) return rc;
    uint64_t* dst = ctx->sorted_buf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>();
    const uint32_t nb = 1u << mb;
    HIPCHK(ctx->crlive.ensure(2 * (n + 64) * 4 + 2 * (nb + 64) * 4 + 64));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(n + 2))));
    uint32_t* live = ctx->crlive.as<uint32_t>();
    uint32_t* pos = live + n + 64;
    uint32_t* bst_in = pos + n + 64;
    uint32_t* bst_out = bst_in + nb + 64;
    uint32_t* d_total = bst_out + nb + 64;
    HIPCHK(hipMemcpyAsync(bst_in, ctx->shard_bst.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(launch_cr_live_compact(s, gt, ctx->crcnt.as<uint32_t>(), 0, n, d_rkey, R, d_rS, a.S0, live, pos,
                                  ctx->tmp.p, dst, bst_in, nb, bst_out, d_total, st, a.off));
    uint32_t nl = 0;
    std::vector<uint32_t> bst(nb + 1);
    HIPCHK(hipMemcpyAsync(&nl, d_total, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(bst.data(), bst_out, (nb + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    note_rs_bytes(ctx);
    done();
    std::vector<uint64_t> log(rS, rS + R * Gu);
    return shard_regroup(ctx, dst, nl, bst, ps, R, log.data(), st);
}

// ---- sharded repeat tolerance (MemHash.cpp:139-162): the first copies of a genome in its
// SortedMerList order need every run of equal keys in std::sort order (MemorySML.cpp:54).
// The runs lie inside the ranks' SML parts; rank g % world replays genome g's sort from the
// pair flags of every rank (rank order = SML order) and returns each rank its slots' ids.
int mums_shard_tie_flags(mums_ctx* ctx, const uint64_t* gofs, uint32_t* d_out) {
    if (check_ctx(ctx) || !gofs || (ctx->shard_n && !d_out)) return MUMS_E_INVALID;
    if (!ctx->ds_ready) return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_prepare first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const uint64_t W = (uint64_t)ctx->gt.G + 1;
    uint64_t* d_gofs = ctx->dsarr.as<uint64_t>() + 8 * W;
    HIPCHK(hipMemcpyAsync(d_gofs, gofs, (W - 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(launch_cr_pair_flags(ctx->crall.as<uint64_t>(), ctx->gt.G, ds_arrays(ctx).lbase, d_gofs, ctx->shard_n, d_out,
                                st));
    HIPCHK(hipStreamSynchronize(st));   // (gofs is the caller's host array)
    return MUMS_OK;
}

int mums_shard_tie_replay(mums_ctx* ctx, const uint32_t* d_packed_all, uint32_t genome, uint32_t nparts,
                          const uint32_t* d_flags, const uint64_t* flag_off, const uint64_t* lens, uint32_t* d_out,
                          const uint64_t* out_off) {
    if (check_ctx(ctx) || !d_packed_all || !flag_off || !lens || !out_off || !d_flags || !d_out) return MUMS_E_INVALID;
    if (!ctx->shard || ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded merge run");
    const GenomeTable& gt = ctx->gt;
    if (genome >= (uint32_t)gt.G) return fail(ctx, MUMS_E_INVALID, "bad genome");
    const uint64_t m = gt.m[genome];
    uint64_t tot = 0;
    for (uint32_t r = 0; r < nparts; ++r) tot += lens[r];
    if (tot != m) return fail(ctx, MUMS_E_INVALID, "tie replay: the parts do not cover the SortedMerList");
    if (m >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList of more than 2^32 seed-mers");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (m == 0) return MUMS_OK;
    if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess) {
        (void)hipGetLastError();
        HIPCHK(hipStreamSynchronize(st));
        release_find_buffers(ctx);
        if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess)
            return fail(ctx, MUMS_E_NOMEM, "repeat tolerance: no device memory for the SortedMerList tie order");
    }
    const TieWs tw = tie_ws_layout(ctx->tiebuf.p, m, 1);
    const uint64_t b0 = 0;
    HIPCHK(tie_set_genomes(tw, &b0, &m, st));
    HIPCHK(tie_clear_flags(tw, st));
    uint64_t o = 0;
    for (uint32_t r = 0; r < nparts; ++r) {   // the ranks' pair flags in SML order
        if (lens[r]) HIPCHK(hipMemcpyAsync(tw.pf + o, d_flags + flag_off[r], lens[r] * 4, hipMemcpyDeviceToDevice, st));
        o += lens[r];
    }
    uint64_t flagged = 0;
    HIPCHK(tie_prepare(tw, &flagged, st));
    uint32_t* ids = tw.Lpos;   // (free once the replay is done) ids at the flagged slots, ~0 elsewhere
    if (flagged) {
        HIPCHK(launch_keys_of_genome(ctx->ss, d_packed_all + all_woff(gt, (int)genome), m, tw.K, st, false));
        HIPCHK(tie_replay(tw, st));
        HIPCHK(hipMemsetAsync(ids, 0xFF, m * 4, st));
        HIPCHK(tie_slots_out(tw, ids, st));
        ctx->tie_slots += flagged;
    } else {
        HIPCHK(hipMemsetAsync(ids, 0xFF, m * 4, st));
    }
    o = 0;
    for (uint32_t r = 0; r < nparts; ++r) {
        if (lens[r]) HIPCHK(hipMemcpyAsync(d_out + out_off[r], ids + o, lens[r] * 4, hipMemcpyDeviceToDevice, st));
        o += lens[r];
    }
    HIPCHK(hipStreamSynchronize(st));
    return MUMS_OK;
}

int mums_shard_tie_apply(mums_ctx* ctx, const uint32_t* d_ids, const uint64_t* vofs) {
    if (check_ctx(ctx) || !vofs || (ctx->shard_n && !d_ids)) return MUMS_E_INVALID;
    if (!ctx->ds_ready) return fail(ctx, MUMS_E_INVALID, "mums_shard_restart_prepare first");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const uint64_t W = (uint64_t)ctx->gt.G + 1;
    uint64_t* d_vofs = ctx->dsarr.as<uint64_t>() + 9 * W;
    HIPCHK(hipMemcpyAsync(d_vofs, vofs, (W - 1) * 8, hipMemcpyHostToDevice, st));
    CrStream s{ctx->sorted_rec, ctx->crbuf.as<uint64_t>(), 1u << ctx->msd_bits, ctx->shard_n};
    s.kb = (uint32_t)(2 * ctx->w + 1 - ctx->msd_bits);
    s.ib = (uint32_t)ctx->rec_ib;
    HIPCHK(launch_cr_tie_vals(s, ctx->gt, ctx->crcnt.as<uint32_t>(), d_vofs, d_ids,
                              const_cast<uint64_t*>(ctx->sorted_rec), st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->ds_ties = true;
    ctx->ties_fixed = true;
    return MUMS_OK;
}

int mums_shard_restart_info(mums_ctx* ctx, uint64_t* info) {
    if (check_ctx(ctx) || !info) return MUMS_E_INVALID;
    std::copy(ctx->rs_info, ctx->rs_info + 4, info);
    return MUMS_OK;
}

int mums_probe_count(mums_ctx* ctx, uint64_t* count) {
    if (check_ctx(ctx) || !count) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no seed stage run");
    if (ctx->shard && ctx->shard_restart_pending)
        return fail(ctx, MUMS_E_INVALID, "sharded restart pending (mums_shard_restart_plan / _apply)");
    *count = ctx->P;
    return MUMS_OK;
}

int mums_probe_copy(mums_ctx* ctx, uint32_t* buckets, uint64_t* ref_index, uint64_t capacity) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no seed stage run");
    if (ctx->shard && ctx->merge_chunked)
        return fail(ctx, MUMS_E_UNSUPPORTED, "probe export after a chunked shard merge");
    if (ctx->shard && ctx->shard_restart_pending)
        return fail(ctx, MUMS_E_INVALID, "sharded restart pending (mums_shard_restart_plan / _apply)");
    if (capacity < ctx->P) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    if (!ctx->packed_path) return fail(ctx, MUMS_E_UNSUPPORTED, "probe export needs the packed-record path");
    if (ctx->P && (!ctx->probe_info || !ctx->sorted_rec))
        return fail(ctx, MUMS_E_UNSUPPORTED, "probe export after a chunked run (> 2^32 seed-mers)");
    const uint64_t P = ctx->P, N = ctx->N;
    if (P == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    std::vector<uint64_t> info(P), rec(N);
    std::vector<uint32_t> bkt(P), ids(P);
    HIPCHK(hipMemcpy(info.data(), ctx->probe_info, P * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(rec.data(), ctx->sorted_rec, N * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(bkt.data(), ctx->sorted_buckets, P * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ids.data(), ctx->sorted_ids, P * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> bucket_of_probe(P);
    for (uint64_t i = 0; i < P; ++i) bucket_of_probe[ids[i]] = bkt[i];
    for (uint64_t k = 0; k < P; ++k) {
        const uint64_t h = (uint32_t)info[k], gs = info[k] >> 32;
        uint64_t mn = ~0ull;
        const uint64_t imask = (1ull << ctx->rec_ib) - 1;
        for (uint64_t i = h; i < h + gs && i < N; ++i) mn = std::min<uint64_t>(mn, rec[i] & imask);
        if (buckets) buckets[k] = bucket_of_probe[k];
        if (ref_index) ref_index[k] = mn;
    }
    return MUMS_OK;
}


// ---- sharded FindMatches -------------------------------------------

namespace {

// (pending_ok: the packed genomes, which the restart's tie replay reads too)
int shard_seeds_done(mums_ctx* ctx, bool pending_ok = false) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!ctx->shard) return fail(ctx, MUMS_E_INVALID, "not a sharded context (mums_shard_layout)");
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "no sharded seed stage run");
    if (ctx->shard_restart_pending && !pending_ok)
        return fail(ctx, MUMS_E_INVALID, "sharded restart pending (mums_shard_restart_plan / _apply)");
    return MUMS_OK;
}

// stable sort of P u32 keys (< 2^bits) -> ctx->sorted_ids / sorted_buckets (rowtmp)
int sort_row_keys(mums_ctx* ctx, uint32_t* keys, uint64_t P, int bits, hipStream_t st) {
    uint32_t* kB = (uint32_t*)ctx->rowtmp.p + (P + 64);
    uint32_t* iA = kB + (P + 64);
    uint32_t* iB = iA + (P + 64);
    HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(P + 1)));
    int out = 0;
    HIPCHK(radix_sort<uint32_t>(keys, nullptr, P, bits, kB, iA, keys, iB, ctx->radix_tmp.p, &out, st));
    ctx->sorted_buckets = out ? keys : kB;
    ctx->sorted_ids = out ? iB : iA;
    return MUMS_OK;
}

// after an enumeration count (pairwise.hip en_rows32): a group with more than 2^31
// AddHashEntry calls (enum_tol^genomes) does not fit the row stream
int enum_count_check(mums_ctx* ctx, hipStream_t st) {
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, &ctx->counters.as<DevCounters>()->err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (err & 64u)
        return fail(ctx, MUMS_E_UNSUPPORTED, "enumeration tolerance: a seed group with more than 2^31 AddHashEntry calls");
    return MUMS_OK;
}

// PairwiseMatchFinder::FindMatches (PairwiseMatchFinder.cpp:37-73 over MemHash): pair
// path keys + sort, one probe row per single-copy genome pair of every group
// (pairwise.hip), then the rows' buckets and the FindMatches tail.
extern "C++" {
template <typename K>
int pairwise_rows(mums_ctx* ctx, uint64_t N, hipStream_t st) {
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const PairView<K> v{(const K*)ctx->sorted_key, ctx->sorted_idx};
    uint32_t* npairs = ctx->cval.as<uint32_t>();
    uint32_t* off = npairs + N + 64;
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    if (ctx->pairwise) HIPCHK(launch_pairwise_count<PairView<K>>(v, N, ctx->gt, npairs, dc, st));
    else HIPCHK(launch_enum_count<PairView<K>>(v, N, ctx->gt, mp, npairs, dc, st));
    HIPCHK(hipMemcpyAsync(off, npairs, N * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(exclusive_scan_u32(off, N, ctx->tmp.p, &dc->nprobes, st));
    uint32_t P = 0;
    HIPCHK(hipMemcpyAsync(&P, &dc->nprobes, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (int rc = enum_count_check(ctx, st)) return rc;
    ctx->P = P;
    HIPCHK(ctx->mprobe.ensure(((uint64_t)P + 1) * (size_t)(ctx->gt.G + 1) * 8));
    if (ctx->pairwise)
        HIPCHK(launch_pairwise_emit<PairView<K>>(v, N, ctx->gt, ctx->L, npairs, off, ctx->mprobe.as<int64_t>(), st));
    else
        HIPCHK(launch_enum_emit<PairView<K>>(v, N, ctx->gt, mp, ctx->L, npairs, off, ctx->mprobe.as<int64_t>(), st));
    return MUMS_OK;
}
}  // extern "C++"

// Also MemHash with enumeration tolerance > 1 (MemHash.cpp:139-162 -> the odometer of
// MatchFinder::EnumerateMatches, MatchFinder.cpp:342-393): one row per AddHashEntry call.
int run_pipeline_pairwise(mums_ctx* ctx, int stage) {
    hipStream_t st = ctx->stream;
    const int G = (int)ctx->genomes.size();
    const uint64_t N = ctx->N;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->pairwise ? 0 : ctx->masked,
                   ctx->pairwise ? 0 : ctx->seq_mask};
    GenomeTable& gt = ctx->gt;
    const int kbits = 2 * ctx->w + 1;
    ctx->packed_path = false;
    ctx->msd_bits = 0;
    const size_t kb = ctx->key64 ? 8 : 4;
    uint64_t words = 0;
    const uint32_t T = layout_packed(gt, &words);
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK(ctx->ckey.ensure(N * kb + 64));
    HIPCHK(ctx->kA.ensure(N * kb + 64));
    HIPCHK(ctx->kB.ensure(N * kb + 64));
    HIPCHK(ctx->vA.ensure(N * 4 + 64));
    HIPCHK(ctx->vB.ensure(N * 4 + 64));
    HIPCHK(ctx->cval.ensure(2 * (N + 64) * 4));
    HIPCHK(ctx->tmp.ensure(std::max(std::max(scan_tmp_bytes(N + 1), radix_tmp_bytes(N + 1)),
                                    scan_tmp_bytes((uint64_t)ctx->table_size))));
    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    std::vector<const char*> ptrs(G);
    for (int g = 0; g < G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
    HIPCHK(launch_seed_pack(ctx->ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 0, ctx->key64, ctx->ckey.p, 0,
                            nullptr, T, &dc->err, st));
    HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
    int buf = 0;
    if (ctx->key64)
        HIPCHK(radix_sort<uint64_t>(ctx->ckey.as<uint64_t>(), nullptr, N, kbits, ctx->kA.as<uint64_t>(),
                                    ctx->vA.as<uint32_t>(), ctx->kB.as<uint64_t>(), ctx->vB.as<uint32_t>(),
                                    ctx->tmp.p, &buf, st));
    else
        HIPCHK(radix_sort<uint32_t>(ctx->ckey.as<uint32_t>(), nullptr, N, kbits, ctx->kA.as<uint32_t>(),
                                    ctx->vA.as<uint32_t>(), ctx->kB.as<uint32_t>(), ctx->vB.as<uint32_t>(),
                                    ctx->tmp.p, &buf, st));
    ctx->sorted_buf = buf;
    ctx->sorted_key = buf ? ctx->kB.p : ctx->kA.p;
    ctx->sorted_idx = buf ? ctx->vB.as<uint32_t>() : ctx->vA.as<uint32_t>();
    ctx->sort_passes = (kbits + 7) / 8;
    HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
    if (wants_tie_order(ctx)) {   // the odometer runs over the copies in SML order
        RsStream s{};
        s.kind = ctx->key64 ? 2 : 1;
        s.key = ctx->sorted_key;
        s.idx = ctx->sorted_idx;
        const int r0 = tie_fix_stream(ctx, s, N, st);
        if (r0) return r0;
    }
    int rc = ctx->key64 ? pairwise_rows<uint64_t>(ctx, N, st) : pairwise_rows<uint32_t>(ctx, N, st);
    if (rc) return rc;
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
    if (ctx->hc.err & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
    if (ctx->hc.repeat_limit || have_start_points(ctx)) {   // MER_REPEAT_LIMIT restart (restart.hip)
        const uint64_t rep = ctx->hc.repeat_limit;
        RsStream s{};
        s.kind = ctx->key64 ? 2 : 1;
        s.key = ctx->sorted_key;
        s.idx = ctx->sorted_idx;
        void* dk = ctx->sorted_buf ? ctx->kA.p : ctx->kB.p;
        uint32_t* dv = ctx->sorted_buf ? ctx->vA.as<uint32_t>() : ctx->vB.as<uint32_t>();
        uint64_t nl = N;
        bool changed = false;
        rc = restart_fixup(ctx, s, N, dk, dv, nullptr, &nl, &changed, st);
        if (rc) return rc;
        if (changed) {
            ctx->sorted_buf ^= 1;
            ctx->sorted_key = dk;
            ctx->sorted_idx = dv;
            rc = ctx->key64 ? pairwise_rows<uint64_t>(ctx, nl, st) : pairwise_rows<uint32_t>(ctx, nl, st);
            if (rc) return rc;
            HIPCHK(h2d_sync(&dc->repeat_limit, &rep, 8, ctx->stream));
            HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
        }
    } else if (ctx->progress_on) {   // LogProgress without a restart (MatchFinder.cpp:296-309)
        RsStream s{};
        s.kind = ctx->key64 ? 2 : 1;
        s.key = ctx->sorted_key;
        s.idx = ctx->sorted_idx;
        rc = progress_pair_stream(ctx, s, N, st);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_GROUPS], st));
    const uint64_t P = ctx->P;
    if (P >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes in one FindMatches");
    ctx->probe_info = nullptr;
    int tbits = 1;
    while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)ctx->table_size) ++tbits;
    if (P) {
        HIPCHK(ctx->rowtmp.ensure((P + 64) * 16 + 8192));
        uint32_t* bkt = (uint32_t*)ctx->rowtmp.p;
        HIPCHK(launch_row_buckets(ctx->mprobe.as<int64_t>(), P, G, ctx->table_size, nullptr, 0, bkt, st));
        rc = sort_row_keys(ctx, bkt, P, tbits, st);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
    ctx->stage_done = MUMS_STAGE_SEEDS;
    if (stage >= MUMS_STAGE_ALL) {
        rc = find_tail(ctx, mp, ctx->packed.as<uint32_t>(), [&](MatProbes* v) {
            v->rows = ctx->mprobe.as<int64_t>();
            return MUMS_OK;
        }, st);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
    fill_stats(ctx, N);
    ctx->st.probes = P;
    return MUMS_OK;
}

// > 2^32 seed-mers per context (BASELINE config 5, chunked.hip): records with 33-bit
// global indices; the 2w+1-31 MSD digits are cut into power-of-two chunks of < 2^30
// records and every chunk runs scatter -> onesweep -> groups -> probe buckets [-> rows]
// on its own, in key order; the FindMatches tail then replays all chunks' rows.
// MER_REPEAT_LIMIT restarts / start points (MatchFinder.cpp:253-277, MemHash.cpp:117-127)
// over a whole merged stream srec of N records (N = ctx->N; key_low << ib | global index,
// 2^B MSD digits implicit, digit starts dstart), split into segments.  Candidates (groups
// above 1000 records) from the whole stream; if any (or start points): the G SortedMerLists
// as full keys in `other` (N + 64 slots), the restart plan (restart_plan.h), the std::sort
// order of the runs a start point falls into (smlsort.hip, one genome at a time; the ids of
// those records in srec are rewritten), then each segment's live records compacted into
// `other` at the segment's base: n_live[c], its bucket starts (bst_in(c, d) writes the
// original nb + 1 of them to device memory d) mapped into d_bst_out + sum of earlier (nb + 1).
// *live = false when every record lives (nothing written).
// the FindMatches tail's buffers (rows, chains, replay, MatchList) hold nothing the seed stage
// reads: freed when a seed-stage allocation does not fit beside them
void release_find_buffers(mums_ctx* ctx) {
    for (DevBuf* b : {&ctx->rowsall, &ctx->rowtmp, &ctx->sids, &ctx->summ, &ctx->chain_tmp, &ctx->chain_of, &ctx->pool,
                      &ctx->pool_loc, &ctx->cbuf, &ctx->spill, &ctx->tbl, &ctx->fk, &ctx->fkloc, &ctx->mprobe,
                      &ctx->out_len, &ctx->out_s})
        b->release();
    ctx->emit_tbl = nullptr;
    ctx->emit_base = nullptr;
    ctx->M = 0;
}

// the tie workspace, and the views the chunked FindMatches keeps inside it (rows, chain scratch)
void release_tiebuf(mums_ctx* ctx) {
    auto inside = [&](const DevBuf& b) {
        return b.borrowed && ctx->tiebuf.p && (const char*)b.p >= (const char*)ctx->tiebuf.p &&
               (const char*)b.p < (const char*)ctx->tiebuf.p + ctx->tiebuf.cap;
    };
    for (DevBuf* b : {&ctx->rowsall, &ctx->chain_tmp})
        if (inside(*b)) b->release();
    ctx->tiebuf.release();
    ctx->tiebuf_kept = false;
}

// tiebuf.ensure that first drops the views inside the workspace when it must reallocate
hipError_t tiebuf_ensure(mums_ctx* ctx, size_t bytes) {
    if (bytes > ctx->tiebuf.cap) release_tiebuf(ctx);
    return ctx->tiebuf.ensure(bytes);
}

// free device memory left beside a kept tie workspace (the chunk loop's buffers)
constexpr size_t kKeepTieFree = 24ull << 30;

// development: MUMS_DEV_RESTART_TIMING prints the wall time of every restart phase
struct PhaseClock {
    bool on;
    hipStream_t st;
    std::chrono::steady_clock::time_point t0;
    PhaseClock(hipStream_t s) : on(getenv("MUMS_DEV_RESTART_TIMING") != nullptr), st(s), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "restart phase %-28s %9.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};

// MatchFinder::LogProgress (MatchFinder.cpp:55-56, 137-164, 296-309): the text the reference
// writes while its merge runs.  Every MER_BUFFER_SIZE (10 000) mers read per genome from the
// phase's start point form a buffer; exhausting one adds its size to mers_processed and prints
// the whole percent when it changed ("N%.."), a newline when the tens digit changed.  A buffer
// is exhausted when the merge consumes its last mer, i.e. at that mer's masked key; in a phase
// that ends in a restart only the buffers ending at or before the plan's consumed positions
// were exhausted (restart_plan.h).  Events are ordered by masked key; inside one seed group
// holding buffer ends of several genomes with unequal sizes, the genomes' runs go in the
// merge's head order (restart_plan.h head_order over the genome-major SML keys: pw->ck, else
// built into ck_build, N slots).  s = the whole merged stream.
struct ProgressEv { uint64_t phase, g, size; };

// the text of buffer-refill events ev (query q[i] = g << 56 | SML index of the buffer's last
// mer) in nph phases whose start points are Sall (nph x G); base[p] = mers_processed when
// phase p starts (MatchFinder.cpp:147 / :150-158), or empty: the count carries across phases
// (ParallelMemHash.cpp:57-61 sets it once for all chunks)
int progress_text(mums_ctx* ctx, const std::vector<ProgressEv>& ev, const std::vector<uint64_t>& q, uint64_t nph,
                  const std::vector<uint64_t>& Sall, const std::vector<uint64_t>& base, const CrStream& s,
                  const uint32_t* gscan, hipStream_t st, const RestartWs* pw, uint64_t* ck_build);

int progress_log(mums_ctx* ctx, const CrStream& s, const uint32_t* gscan, hipStream_t st,
                 const RestartWs* pw = nullptr, uint64_t* ck_build = nullptr) {
    ctx->progress.clear();
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G;
    constexpr uint64_t kBuf = restart::kMerBuffer;
    const uint64_t R = ctx->restarts;
    if (R && ctx->consumed_log.size() != R * Gu) return fail(ctx, MUMS_E_HIP, "progress: restart plan without consumed positions");
    std::vector<ProgressEv> ev;
    std::vector<uint64_t> q;
    std::vector<uint64_t> S(Gu, 0), total_sp(R + 1, 0), Sall((R + 1) * Gu, 0);
    for (uint64_t p = 0; p <= R; ++p) {
        for (int g = 0; g < G; ++g) {
            S[g] = p == 0 ? (g < (int)ctx->start_points.size() ? ctx->start_points[g] : 0) : ctx->offset_log[(p - 1) * Gu + g];
            Sall[p * Gu + g] = S[g];
            total_sp[p] += S[g];
            const uint64_t m = gt.m[g];
            const uint64_t cons = p < R ? ctx->consumed_log[p * Gu + g] : m;
            for (uint64_t a = S[g]; a < m; a += kBuf) {
                const uint64_t e = std::min(a + kBuf, m);
                if (e > cons) break;
                ev.push_back(ProgressEv{p, (uint64_t)g, e - a});
                q.push_back(((uint64_t)g << 56) | (e - 1));
            }
        }
    }
    return progress_text(ctx, ev, q, R + 1, Sall, total_sp, s, gscan, st, pw, ck_build);
}

int progress_text(mums_ctx* ctx, const std::vector<ProgressEv>& ev, const std::vector<uint64_t>& q, uint64_t nph,
                  const std::vector<uint64_t>& Sall, const std::vector<uint64_t>& base, const CrStream& s,
                  const uint32_t* gscan, hipStream_t st, const RestartWs* pw, uint64_t* ck_build) {
    ctx->progress.clear();
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G;
    uint64_t total = 0;
    for (int g = 0; g < G; ++g) total += gt.n[g];   // MatchFinder.cpp:146: SortedMerList::Length() = seq_len
    std::vector<uint64_t> key(q.size(), 0);
    if (!q.empty() && !s.rec) {   // no packed stream (the pair path): the SMLs of pw answer
        if (!pw) return fail(ctx, MUMS_E_HIP, "progress: neither a stream nor SMLs (internal error)");
        DevBuf qb;
        HIPCHK(qb.ensure(q.size() * 16 + 64));
        uint64_t* d_q = qb.as<uint64_t>();
        HIPCHK(hipMemcpyAsync(d_q, q.data(), q.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(launch_cr_ck_query(pw->ck, gt, d_q, q.size(), d_q + q.size(), st));
        HIPCHK(hipMemcpyAsync(key.data(), d_q + q.size(), q.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    } else if (!q.empty()) {
        const uint64_t nblk = cr_blocks(s.N);
        if (!gscan) {
            HIPCHK(ctx->crcnt.ensure(Gu * (nblk + 1) * 4 + 256));
            HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nblk + 2))));
            HIPCHK(launch_cr_counts(s, gt, ctx->crcnt.as<uint32_t>(), ctx->tmp.p, st));
            gscan = ctx->crcnt.as<uint32_t>();
        }
        DevBuf qb;
        HIPCHK(qb.ensure(q.size() * 16 + 64));
        uint64_t* d_q = qb.as<uint64_t>();
        HIPCHK(hipMemcpyAsync(d_q, q.data(), q.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(launch_cr_query(s, gt, gscan, d_q, q.size(), d_q + q.size(), st));
        HIPCHK(hipMemcpyAsync(key.data(), d_q + q.size(), q.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    std::vector<uint64_t> ord(ev.size());
    for (uint64_t i = 0; i < ord.size(); ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
        if (ev[a].phase != ev[b].phase) return ev[a].phase < ev[b].phase;
        return key[a] < key[b];
    });
    std::vector<std::pair<uint64_t, uint64_t>> groups;   // [begin, end) in ord
    std::vector<uint64_t> gk, gu;
    std::vector<uint32_t> gp;
    for (uint64_t i = 0; i < ord.size();) {
        uint64_t j = i + 1;
        while (j < ord.size() && ev[ord[j]].phase == ev[ord[i]].phase && key[ord[j]] == key[ord[i]]) ++j;
        uint64_t U = 0;
        bool uneq = false;
        for (uint64_t k = i; k < j; ++k) {
            U |= 1ull << ev[ord[k]].g;
            uneq = uneq || ev[ord[k]].size != ev[ord[i]].size;
        }
        if ((U & (U - 1)) && uneq) {
            groups.push_back({i, j});
            gk.push_back(key[ord[i]]);
            gu.push_back(U);
            gp.push_back((uint32_t)ev[ord[i]].phase);
        }
        i = j;
    }
    if (!groups.empty() && (pw || ck_build)) {
        const uint64_t ng = groups.size();
        DevBuf aux;
        HIPCHK(aux.ensure((nph * Gu + 2 * ng + 2 * (Gu + 1)) * 8 + ng * 4 + ng * Gu * 4 + 1024));
        uint64_t* d_S = aux.as<uint64_t>();
        uint64_t* d_gk = d_S + nph * Gu;
        uint64_t* d_gu = d_gk + ng;
        uint64_t* d_dm = d_gu + ng;
        uint64_t* d_db = d_dm + Gu + 1;
        uint32_t* d_gp = (uint32_t*)(d_db + Gu + 1);
        int* d_ord = (int*)(d_gp + ng);
        RestartWs w{};
        if (pw) {
            w = *pw;
        } else {   // gscan was built above (the queries are nonempty when groups exist)
            HIPCHK(launch_cr_ck(s, gt, gscan, ck_build, st));
            std::vector<uint64_t> hm(Gu + 1, 0), hb(Gu + 1, 0);
            for (int g = 0; g < G; ++g) {
                hm[g] = gt.m[g];
                hb[g] = gt.base[g];
            }
            HIPCHK(hipMemcpyAsync(d_dm, hm.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(d_db, hb.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
            w.ck = ck_build;
            w.dm = d_dm;
            w.dbase = d_db;
        }
        HIPCHK(hipMemcpyAsync(d_S, Sall.data(), Sall.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_gk, gk.data(), ng * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_gu, gu.data(), ng * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(d_gp, gp.data(), ng * 4, hipMemcpyHostToDevice, st));
        HIPCHK(launch_tie_heads(w, G, d_gk, d_gu, d_gp, d_S, ng, d_ord, st));
        std::vector<int> ho(ng * Gu);
        HIPCHK(hipMemcpyAsync(ho.data(), d_ord, ho.size() * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::vector<int> rank(Gu);
        for (uint64_t x = 0; x < ng; ++x) {
            std::fill(rank.begin(), rank.end(), G);
            for (int k = 0; k < G && ho[x * Gu + k] >= 0; ++k) rank[ho[x * Gu + k]] = k;
            std::stable_sort(ord.begin() + groups[x].first, ord.begin() + groups[x].second,
                             [&](uint64_t a, uint64_t b) { return rank[ev[a].g] < rank[ev[b].g]; });
        }
    }
    double m_progress = -1;   // MatchFinder.cpp:143; kept across restarts
    uint64_t processed = 0;
    uint64_t phase = ~0ull;
    char b[32];
    for (uint64_t i : ord) {
        if (ev[i].phase != phase) {
            phase = ev[i].phase;
            if (!base.empty()) processed = base[phase];   // :147 / :150-158
        }
        processed += ev[i].size;
        const double old = m_progress;
        m_progress = ((double)processed / (double)total) * 100.0;   // PROGRESS_GRANULARITY 100
        if ((int)old != (int)m_progress) {
            snprintf(b, sizeof b, "%d%%..", (int)((m_progress / 100.0) * 100));
            ctx->progress += b;
        }
        if (((int)old / 10) != ((int)m_progress / 10)) ctx->progress += "\n";
    }
    return MUMS_OK;
}

// ParallelMemHash LogProgress (ParallelMemHash.cpp:56-61, 86-101) in the schedule of one
// OpenMP thread: the chunks' SearchRange calls in chunk order, genome g of chunk c read in
// MER_BUFFER_SIZE buffers from S = hcs[c][g] up to the chunk's search_len (the next chunk's
// start; the last chunk: the SML end), mers_processed set to 0 once and carried across the
// chunks.  A chunk cut by MER_REPEAT_LIMIT (compat_truncate) refills only the buffers its
// merge consumed.  The SML keys are the genome-major ckeys in ctx->crall.
int progress_compat(mums_ctx* ctx, uint32_t nch, const std::vector<uint64_t>& hcs, hipStream_t st) {
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G;
    constexpr uint64_t kBuf = restart::kMerBuffer;
    if (hcs.size() < (uint64_t)nch * Gu) return fail(ctx, MUMS_E_HIP, "progress: chunk starts missing (internal error)");
    if (int rc0 = compat_ck_ready(ctx, st)) return rc0;
    std::vector<ProgressEv> ev;
    std::vector<uint64_t> q, Sall((uint64_t)nch * Gu, 0);
    for (uint32_t c = 0; c < nch; ++c) {
        for (int g = 0; g < G; ++g) {
            const uint64_t m = gt.m[g];
            const uint64_t S = std::min(hcs[(uint64_t)c * Gu + g], m);
            uint64_t E = c + 1 < nch ? std::min(hcs[(uint64_t)(c + 1) * Gu + g], m) : m;
            if (E < S) E = S;
            const uint64_t cz = ctx->compat_cons.empty() ? ~0ull : ctx->compat_cons[(uint64_t)c * Gu + g];
            const uint64_t cons = cz == ~0ull ? E : cz;
            Sall[(uint64_t)c * Gu + g] = S;
            for (uint64_t a = S; a < E; a += kBuf) {
                const uint64_t e = std::min(a + kBuf, E);
                if (e > cons) break;
                ev.push_back(ProgressEv{c, (uint64_t)g, e - a});
                q.push_back(((uint64_t)g << 56) | (e - 1));
            }
        }
    }
    DevBuf aux;
    HIPCHK(aux.ensure(2 * (Gu + 1) * 8 + 64));
    std::vector<uint64_t> hm(2 * (Gu + 1), 0);
    for (int g = 0; g < G; ++g) {
        hm[g] = gt.m[g];
        hm[Gu + 1 + g] = gt.base[g];
    }
    HIPCHK(hipMemcpyAsync(aux.p, hm.data(), hm.size() * 8, hipMemcpyHostToDevice, st));
    RestartWs w{};
    w.ck = ctx->crall.as<uint64_t>();
    w.dm = aux.as<uint64_t>();
    w.dbase = aux.as<uint64_t>() + Gu + 1;
    const CrStream none{nullptr, nullptr, 0, 0};
    const int rc = progress_text(ctx, ev, q, nch, Sall, {}, none, nullptr, st, &w, nullptr);
    HIPCHK(hipStreamSynchronize(st));   // aux is freed on return
    return rc;
}

// the single-context packed stream (records key_low << 32 | index, 2^B MSD buckets starting at
// the device u32 bucket starts bstart) as a CrStream for progress_log
int progress_packed(mums_ctx* ctx, const uint64_t* rec, const uint32_t* bstart, int B, uint64_t n, hipStream_t st,
                    const RestartWs* pw, uint64_t* ck_build) {
    const uint64_t nd = 1ull << B;
    std::vector<uint32_t> h32(nd + 1);
    HIPCHK(hipMemcpyAsync(h32.data(), bstart, (nd + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<uint64_t> h64(nd + 1);
    for (uint64_t d = 0; d <= nd; ++d) h64[d] = B ? h32[d] : (d ? n : 0);
    DevBuf db;
    HIPCHK(db.ensure((nd + 1) * 8 + 64));
    HIPCHK(hipMemcpyAsync(db.p, h64.data(), (nd + 1) * 8, hipMemcpyHostToDevice, st));
    CrStream s{rec, db.as<uint64_t>(), (uint32_t)nd, n};
    s.kb = (uint32_t)(2 * ctx->w + 1 - B);
    s.ib = 32;
    const int rc = progress_log(ctx, s, nullptr, st, pw, ck_build);
    HIPCHK(hipStreamSynchronize(st));   // db and the query buffer are freed on return
    return rc;
}

// the pair path (keys + indices, no packed stream): the SMLs of the restart workspace
int progress_pairs(mums_ctx* ctx, const RestartWs* pw, hipStream_t st) {
    CrStream none{nullptr, nullptr, 0, 0};
    return progress_log(ctx, none, nullptr, st, pw);
}

int progress_pair_stream(mums_ctx* ctx, const RsStream& s, uint64_t n, hipStream_t st) {
    HIPCHK(ctx->rsbuf.ensure(restart_ws_bytes(n, ctx->gt.G)));
    const RestartWs w = restart_ws_layout(ctx->rsbuf.p, n, ctx->gt.G);
    HIPCHK(launch_restart_smls(s, n, ctx->gt, w, st));
    ctx->restarts = 0;
    ctx->offset_log.clear();
    ctx->consumed_log.clear();
    const int rc = progress_pairs(ctx, &w, st);
    HIPCHK(hipStreamSynchronize(st));
    return rc;
}

int stream_restart(mums_ctx* ctx, uint64_t* srec, uint64_t* other, const std::vector<uint64_t>& dstart, uint32_t kb,
                   uint32_t ib, const std::vector<RestartSeg>& segs,
                   const std::function<int(uint32_t, uint32_t*)>& bst_in, uint32_t* d_bst_out,
                   std::vector<uint64_t>& n_live, bool* live_out, hipStream_t st) {
    PhaseClock pc(st);
    const GenomeTable& gt = ctx->gt;
    const int G = gt.G;
    const uint64_t Gu = (uint64_t)G;
    const uint64_t N = ctx->N;
    const uint32_t nd = (uint32_t)dstart.size() - 1;
    *live_out = false;
    n_live.assign(segs.size(), 0);
    ctx->restarts = 0;
    ctx->offset_log.clear();
    const uint64_t ccap = N / (restart::kRepeatLimit + 1) + 16;   // candidates: runs of > 1000 records
    HIPCHK(ctx->crbuf.ensure((nd + 1) * 8 + 64 + ccap * 8 + 4096));
    uint64_t* d_dstart = ctx->crbuf.as<uint64_t>();
    unsigned long long* d_cnt = (unsigned long long*)(d_dstart + nd + 1);
    uint64_t* d_list = (uint64_t*)(d_cnt + 8);
    HIPCHK(hipMemcpyAsync(d_dstart, dstart.data(), (nd + 1) * 8, hipMemcpyHostToDevice, st));
    CrStream s{srec, d_dstart, nd, N};
    s.kb = kb;
    s.ib = ib;
    HIPCHK(launch_cr_cands(s, d_list, d_cnt, ccap, st));
    unsigned long long C = 0;
    HIPCHK(hipMemcpyAsync(&C, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->cr_cands = C;
    pc.mark("candidates");
    ctx->consumed_log.clear();
    if (C == 0 && !have_start_points(ctx)) return ctx->progress_on ? progress_log(ctx, s, nullptr, st, nullptr, other) : MUMS_OK;
    if (C > ccap) return fail(ctx, MUMS_E_HIP, "restart: candidate list overflow (internal error)");
    if (ctx->parity_masked || seg_onesweep_launches(kb) < (int)((kb + 7) / 8))
        return fail(ctx, MUMS_E_UNSUPPORTED, "restart with the segment fix-up sort (MUMS_DEV_SEGFIX)");
    std::vector<uint64_t> cand(C);
    if (C) {
        HIPCHK(hipMemcpy(cand.data(), d_list, C * 8, hipMemcpyDeviceToHost));
        std::sort(cand.begin(), cand.end());
        HIPCHK(hipMemcpyAsync(d_list, cand.data(), C * 8, hipMemcpyHostToDevice, st));
    }
    // per-genome block counts and the SMLs (full keys) in the other buffer
    const uint64_t nblk = cr_blocks(N);
    HIPCHK(ctx->crcnt.ensure(Gu * (nblk + 1) * 4 + 256));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nblk + 2))));
    uint32_t* gscan = ctx->crcnt.as<uint32_t>();
    HIPCHK(launch_cr_counts(s, gt, gscan, ctx->tmp.p, st));
    uint64_t* ck = other;
    HIPCHK(launch_cr_ck(s, gt, gscan, ck, st));
    pc.mark("SMLs (counts, keys)");
    // the plan (restart.hip's kernels over the SMLs)
    std::vector<uint64_t> S0(G, 0), hm(G + 1, 0), hb(G + 1, 0);
    for (int g = 0; g < G && g < (int)ctx->start_points.size(); ++g) S0[g] = ctx->start_points[g];
    for (int g = 0; g < G; ++g) {
        hm[g] = gt.m[g];
        hb[g] = gt.base[g];
    }
    const uint64_t cap = C + 16;
    const size_t plan_words = cap + 1 + 3 * cap * Gu + (cap + 1) / 2 + 2 * Gu + 16 + cap + 2 * cap * Gu + 2 * (Gu + 1);
    HIPCHK(ctx->rsplan.ensure(plan_words * 8 + sizeof(restart::PlanOut) + 4096));
    uint64_t* p_list = ctx->rsplan.as<uint64_t>();
    uint64_t* d_pre = p_list + cap + 1;
    uint64_t* d_S = d_pre + 3 * cap * Gu + (cap + 1) / 2;
    uint64_t* d_S0 = d_S + Gu;
    restart::PlanOut* d_out = (restart::PlanOut*)(d_S0 + Gu);
    uint64_t* d_rkey = d_S0 + Gu + 16;
    uint64_t* d_rS = d_rkey + cap;
    uint64_t* d_dm = d_rS + cap * Gu;
    uint64_t* d_db = d_dm + Gu + 1;
    uint64_t* d_rC = d_db + Gu + 1;
    if (C) HIPCHK(hipMemcpyAsync(p_list, d_list, C * 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(d_dm, hm.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_db, hb.data(), (Gu + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_S, S0.data(), Gu * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_S0, S0.data(), Gu * 8, hipMemcpyHostToDevice, st));
    restart::PlanOut po{};
    po.cap = C;
    po.rkey = d_rkey;
    po.rS = d_rS;
    po.rC = d_rC;
    po.status = restart::kPlanOk;
    HIPCHK(hipMemcpyAsync(d_out, &po, sizeof(po), hipMemcpyHostToDevice, st));
    RestartWs w{};
    w.dm = d_dm;
    w.dbase = d_db;
    w.ck = ck;
    HIPCHK(launch_restart_plan(w, G, p_list, C, d_pre, d_S, d_out, st));
    HIPCHK(hipMemcpyAsync(&po, d_out, sizeof(po), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (po.status != restart::kPlanOk) return fail(ctx, MUMS_E_HIP, "restart plan table full (internal error)");
    const uint64_t R = po.nrestarts;
    ctx->restarts = R;
    ctx->offset_log.assign(R * Gu, 0);
    if (R) HIPCHK(hipMemcpy(ctx->offset_log.data(), d_rS, R * Gu * 8, hipMemcpyDeviceToHost));
    ctx->consumed_log.assign(R * Gu, 0);
    if (R) HIPCHK(hipMemcpy(ctx->consumed_log.data(), d_rC, R * Gu * 8, hipMemcpyDeviceToHost));
    pc.mark("plan");
    if (ctx->progress_on) {   // the stream is still whole here (compaction below)
        const int rc = progress_log(ctx, s, gscan, st, &w);
        if (rc) return rc;
    }
    if (R == 0 && !have_start_points(ctx)) return MUMS_OK;
    // start points inside runs of equal keys: those runs in std::sort order (MemorySML.cpp:54)
    const uint64_t rcap = (R + 1) * Gu + 16;
    HIPCHK(ctx->crruns.ensure(rcap * 24 + (R + 1) * 8 + 256));
    uint64_t* d_runs = ctx->crruns.as<uint64_t>();
    uint64_t* d_sp = d_runs + 3 * rcap;   // genome g's start points, one per row
    HIPCHK(hipMemsetAsync(d_cnt, 0, 8, st));
    HIPCHK(launch_cr_runs(ck, gt, d_S0, 1, d_runs, d_cnt, rcap, st));
    HIPCHK(launch_cr_runs(ck, gt, d_rS, R, d_runs, d_cnt, rcap, st));
    unsigned long long nruns = 0;
    HIPCHK(hipMemcpyAsync(&nruns, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (nruns > rcap) return fail(ctx, MUMS_E_HIP, "restart: run list overflow (internal error)");
    if (nruns) {
        std::vector<uint64_t> hr(3 * nruns);
        HIPCHK(hipMemcpy(hr.data(), d_runs, 3 * nruns * 8, hipMemcpyDeviceToHost));
        for (int g = 0; g < G; ++g) {
            bool any = false;
            for (uint64_t q = 0; q < nruns; ++q) any = any || (int)hr[3 * q] == g;
            if (!any) continue;
            const uint64_t m = gt.m[g];
            if (m >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList of more than 2^32 seed-mers");
            if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess) {
                // the previous FindMatches' tail buffers are dead during the seed stage: free them
                // and try again (2 x 3 Gbp: ~135 GB of tie workspace beside 96 GB of records)
                (void)hipGetLastError();
                HIPCHK(hipStreamSynchronize(st));
                pc.mark("tie workspace (first try)");
                release_find_buffers(ctx);
                pc.mark("FindMatches buffers freed");
                if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess)
                    return fail(ctx, MUMS_E_NOMEM, "restart: no device memory for the SortedMerList tie order of a "
                                                   "genome");
            }
            pc.mark("tie workspace");
            const TieWs tw = tie_ws_layout(ctx->tiebuf.p, m, 1);
            const uint64_t b0 = 0;
            HIPCHK(tie_set_genomes(tw, &b0, &m, st));
            HIPCHK(tie_clear_flags(tw, st));
            std::vector<uint64_t> sp(R + 1);
            sp[0] = S0[g];
            for (uint64_t r = 0; r < R; ++r) sp[r + 1] = ctx->offset_log[r * Gu + g];
            HIPCHK(hipMemcpyAsync(d_sp, sp.data(), (R + 1) * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));   // (sp is a host temporary)
            HIPCHK(tie_mark_starts(tw, ck + gt.base[g], d_sp, R + 1, st));
            uint64_t flagged = 0;
            HIPCHK(tie_prepare(tw, &flagged, st));
            pc.mark("tie flags");
            if (!flagged) continue;
            HIPCHK(launch_cr_kpos(s, gt, g, tw.K, st));
            pc.mark("tie keys in position order");
            HIPCHK(tie_replay(tw, st));
            pc.mark("tie replay");
            HIPCHK(launch_cr_tie_write(s, gt, g, d_runs, nruns, ck, tw.V, srec, st));
            ctx->tie_slots += flagged;
            if (pc.on) fprintf(stderr, "restart genome %d: %lu flagged slots, %lu runs\n", g, (unsigned long)flagged,
                               (unsigned long)nruns);
            pc.mark("tie order of one genome");
        }
        HIPCHK(hipStreamSynchronize(st));
        size_t free_b = 0, total_b = 0;
        if (!(ctx->keep_tiebuf == 2 ||
              (ctx->keep_tiebuf == 1 && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b >= kKeepTieFree)))
            release_tiebuf(ctx);
        else
            ctx->tiebuf_kept = true;
        pc.mark("tie workspace freed");
    }
    // every segment's live records (SML index >= the start point of its key's phase),
    // compacted into `other` at the segment's base (the SMLs there are dead now)
    uint64_t nmax = 0, nbmax = 0;
    for (const RestartSeg& g : segs) {
        nmax = std::max(nmax, g.hi - g.lo);
        nbmax = std::max<uint64_t>(nbmax, g.nb);
    }
    HIPCHK(ctx->crlive.ensure(2 * (nmax + 64) * 4 + (nbmax + 64) * 4));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nmax + 2))));
    uint32_t* live = ctx->crlive.as<uint32_t>();
    uint32_t* pos = live + nmax + 64;
    uint32_t* bst = pos + nmax + 64;
    uint32_t* d_total = (uint32_t*)d_cnt;
    uint64_t bo = 0;
    for (uint32_t c = 0; c < (uint32_t)segs.size(); ++c) {
        const uint64_t lo = segs[c].lo, hi = segs[c].hi;
        const int rc = bst_in(c, bst);
        if (rc) return rc;
        HIPCHK(launch_cr_live_compact(s, gt, gscan, lo, hi, d_rkey, R, d_rS, d_S0, live, pos, ctx->tmp.p, other + lo,
                                      bst, segs[c].nb, d_bst_out + bo, d_total, st));
        bo += segs[c].nb + 1;
        uint32_t t = 0;
        HIPCHK(hipMemcpyAsync(&t, d_total, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        n_live[c] = t;
    }
    pc.mark("live compaction");
    for (DevBuf* b : {&ctx->crcnt, &ctx->crlive, &ctx->crruns}) b->release();
    *live_out = true;
    return MUMS_OK;
}

// Repeat tolerance in the chunked mode (MemHash.cpp:139-162: the first copies of a genome
// in SML order): every run of equal keys of the resident stream (buffer sbuf) takes the
// std::sort order (smlsort.hip, all runs flagged), one genome after the other; the SMLs
// (full keys, genome-major) are built in the other buffer.
int chunked_tie_fix(mums_ctx* ctx, int sbuf, const std::vector<uint64_t>& dstart, hipStream_t st) {
    uint64_t* srec = sbuf ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>();
    uint64_t* ck = sbuf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>();
    const GenomeTable& gt = ctx->gt;
    const uint64_t N = ctx->N, Gu = (uint64_t)gt.G;
    const uint32_t nd = (uint32_t)dstart.size() - 1;
    PhaseClock pc(st);
    HIPCHK(ctx->crbuf.ensure((nd + 1) * 8 + 4096));
    uint64_t* d_dstart = ctx->crbuf.as<uint64_t>();
    HIPCHK(hipMemcpyAsync(d_dstart, dstart.data(), (nd + 1) * 8, hipMemcpyHostToDevice, st));
    CrStream s{srec, d_dstart, nd, N};
    s.kb = 31;
    s.ib = 33;
    const uint64_t nblk = cr_blocks(N);
    HIPCHK(ctx->crcnt.ensure(Gu * (nblk + 1) * 4 + 256));
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nblk + 2))));
    uint32_t* gscan = ctx->crcnt.as<uint32_t>();
    HIPCHK(launch_cr_counts(s, gt, gscan, ctx->tmp.p, st));
    HIPCHK(launch_cr_ck(s, gt, gscan, ck, st));
    pc.mark("tie order: SMLs");
    for (int g = 0; g < gt.G; ++g) {
        const uint64_t m = gt.m[g];
        if (m < 2) continue;
        if (m >= 0xFFFFFFF0ull) return fail(ctx, MUMS_E_UNSUPPORTED, "SortedMerList of more than 2^32 seed-mers");
        if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess) {
            (void)hipGetLastError();
            HIPCHK(hipStreamSynchronize(st));
            release_find_buffers(ctx);
            if (tiebuf_ensure(ctx, tie_ws_bytes(m, 1)) != hipSuccess)
                return fail(ctx, MUMS_E_NOMEM, "repeat tolerance: no device memory for the SortedMerList tie order");
        }
        const TieWs tw = tie_ws_layout(ctx->tiebuf.p, m, 1);
        const uint64_t b0 = 0;
        HIPCHK(tie_set_genomes(tw, &b0, &m, st));
        HIPCHK(tie_clear_flags(tw, st));
        HIPCHK(tie_mark_all(tw, ck + gt.base[g], st));
        uint64_t flagged = 0;
        HIPCHK(tie_prepare(tw, &flagged, st));
        if (!flagged) continue;
        HIPCHK(launch_cr_kpos(s, gt, g, tw.K, st));
        HIPCHK(tie_replay(tw, st));
        HIPCHK(launch_cr_tie_all(s, gt, gscan, g, tw.ts, tw.V, srec, st));
        ctx->tie_slots += flagged;
        pc.mark("tie order of one genome (all runs)");
    }
    HIPCHK(hipStreamSynchronize(st));
    ctx->ties_fixed = true;
    return MUMS_OK;
}

// The chunked mode's restart (all chunks resident and sorted in buffer sbuf): live chunks
// into the other buffer (*live_rec), n_live[c], the chunks' bucket starts in ctx->rsbst.
int chunked_restart(mums_ctx* ctx, int sbuf, const std::vector<uint64_t>& dstart, const std::vector<uint64_t>& cbase,
                    uint32_t nbc, uint32_t nch, std::vector<uint64_t>& n_live, uint64_t** live_rec,
                    const std::function<int(uint32_t, uint64_t, uint32_t*)>& chunk_starts, hipStream_t st) {
    uint64_t* srec = sbuf ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>();
    uint64_t* other = sbuf ? ctx->recA.as<uint64_t>() : ctx->recB.as<uint64_t>();
    *live_rec = nullptr;
    std::vector<RestartSeg> segs(nch);
    for (uint32_t c = 0; c < nch; ++c) segs[c] = RestartSeg{cbase[c], cbase[c + 1], nbc};
    HIPCHK(ctx->rsbst.ensure((uint64_t)nch * (nbc + 1) * 4 + 64));
    bool live = false;
    const int rc = stream_restart(ctx, srec, other, dstart, 31, 33, segs, [&](uint32_t c, uint32_t* d) -> int {
        return chunk_starts(c, cbase[c + 1] - cbase[c], d);
    }, ctx->rsbst.as<uint32_t>(), n_live, &live, st);
    if (rc) return rc;
    if (live) *live_rec = other;
    return MUMS_OK;
}

int run_pipeline_chunked(mums_ctx* ctx, int stage) {
    hipStream_t st = ctx->stream;
    const int G = (int)ctx->genomes.size();
    const uint64_t N = ctx->N;
    // PairwiseMatchFinder / enumeration tolerance > 1: every chunk's groups enumerated into
    // rows (pairwise.hip over launch_chunk_pairs' 64-bit-index pairs) instead of the probe
    // stage; the rows' order is the AddHashEntry call order as in run_pipeline_pairwise
    const bool enum_rows = ctx->pairwise || ctx->enum_tol > 1;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->pairwise ? 0 : ctx->masked,
                   ctx->pairwise ? 0 : ctx->seq_mask};
    GenomeTable& gt = ctx->gt;
    const int kbits = 2 * ctx->w + 1;
    // implicit digit bits: the record keeps 31 key bits + 33 index bits.  Above 8 of them
    // (w20-21, the default seed of genomes above ~1.07 Gbp) the scatter splits by the top 8
    // and keeps the next S in side bytes; msd_split refines every chunk (msdsplit.hip).
    const int Bt = kbits - 31;
    const int S = Bt > 8 ? Bt - 8 : 0;
    const int B = Bt - S;       // scatter (MSD) digit bits
    if (Bt < 1 || Bt > 12)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed-mers (chunked mode) needs seed weight 16-21");
    if (N >= (1ull << 33)) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^33 seed-mers per context");
    // repeat tolerance: the first copies of a genome follow its SML's std::sort order, replayed
    // over the resident stream (chunked_tie_fix)
    if (wants_tie_order(ctx) && getenv("MUMS_DEV_CHUNK_STREAM"))
        return fail(ctx, MUMS_E_UNSUPPORTED, "repeat tolerance in the chunked mode needs the resident layout");
    ctx->packed_path = true;
    ctx->key64 = true;
    ctx->msd_bits = Bt;
    ctx->parity_masked = false;
    uint64_t words = 0;
    const uint32_t T = layout_packed(gt, &words);
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    HIPCHK(ctx->hist.ensure(((uint64_t)T << B) * 4 + 64));
    HIPCHK(ctx->ctab.ensure((1u << B) * 8 + 64));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    const bool prof = ctx->profiling;
    if (prof && !ctx->ev_ds[0])
        for (int i = 0; i < 16; ++i) HIPCHK(hipEventCreate(&ctx->ev_ds[i]));
    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    std::vector<const char*> ptrs(G);
    for (int g = 0; g < G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
    uint32_t* hist = ctx->hist.as<uint32_t>();
    HIPCHK(launch_seed_pack(ctx->ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 1, true, nullptr, B, hist, T,
                            &dc->err, st));
    HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
    const uint32_t nd = 1u << B;
    HIPCHK(launch_digit_totals(hist, nd, T, ctx->ctab.as<unsigned long long>(), st));
    std::vector<unsigned long long> tot(nd);
    HIPCHK(hipMemcpyAsync(tot.data(), ctx->ctab.p, nd * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->hc.err & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
    // chunk bits: the fewest power-of-two digit groups each holding < cap records
    uint64_t cap = (1ull << 30) - 4096;
    if (const char* e = getenv("MUMS_DEV_CHUNK_RECORDS")) cap = std::min<uint64_t>(cap, strtoull(e, nullptr, 10));
    int cb = 0;
    for (; cb <= B; ++cb) {
        const uint32_t per = 1u << (B - cb);
        bool ok = true;
        for (uint32_t d0 = 0; d0 < nd && ok; d0 += per) {
            uint64_t sum = 0;
            for (uint32_t d = d0; d < d0 + per; ++d) sum += tot[d];
            ok = sum < cap;
        }
        if (ok) break;
    }
    if (cb > B) return fail(ctx, MUMS_E_UNSUPPORTED, "chunked mode: one MSD digit holds more seed-mers than a chunk (2^30)");
    const int mb8 = B - cb;                               // scatter digits per chunk: 2^mb8
    const uint32_t nbc8 = 1u << mb8, nch = 1u << cb;
    const int mb = mb8 + S;                               // sort buckets per chunk (after the split)
    const uint32_t nbc = 1u << mb;
    uint64_t nmax = 0;
    for (uint32_t c = 0; c < nch; ++c) {
        uint64_t sum = 0;
        for (uint32_t d = c * nbc8; d < (c + 1) * nbc8; ++d) sum += tot[d];
        nmax = std::max(nmax, sum);
    }
    ProbeSpace ps{};
    int rc = ensure_merge_space(ctx, nmax + 1, mb, 31, &ps);
    if (rc) return rc;
    HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes((uint64_t)nbc8 * T + 1))));
    if (S) HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, msd_split_tmp_bytes(nmax + 1, mb8))));
    // resident layout (the 288 GB of HBM hold all 2 x N records): every chunk's slice of
    // the MSD histogram scanned on its own, ONE scatter of all records to their chunk
    // (64-bit chunk bases), then each chunk sorted / grouped in place.  Otherwise (or
    // with MUMS_DEV_CHUNK_STREAM set) the scatter runs once per chunk into a chunk-sized
    // buffer, recomputing the keys every time.
    std::vector<uint64_t> cbase(nch + 1, 0);
    for (uint32_t c = 0; c < nch; ++c) {
        uint64_t sum = 0;
        for (uint32_t d = c * nbc8; d < (c + 1) * nbc8; ++d) sum += tot[d];
        cbase[c + 1] = cbase[c] + sum;
    }
    bool resident = getenv("MUMS_DEV_CHUNK_STREAM") == nullptr;
    if (S && !resident)
        return fail(ctx, MUMS_E_UNSUPPORTED, "seed weight 20-21 in the chunked mode needs the resident layout");
    if (resident) {
        size_t fr = 0, total_mem = 0;
        HIPCHK(hipMemGetInfo(&fr, &total_mem));
        const uint64_t need = 2 * (N + 64) * 8 + (S ? N + 64 : 0);
        resident = need + (uint64_t)(1ull << 30) < (uint64_t)fr + ctx->recA.cap + ctx->recB.cap + ctx->side.cap;
        if (S && !resident)
            return fail(ctx, MUMS_E_NOMEM, "seed weight 20-21 in the chunked mode: records and side bytes do not fit");
        if (wants_tie_order(ctx) && !resident)
            return fail(ctx, MUMS_E_NOMEM, "repeat tolerance in the chunked mode: the records do not fit resident");
    }
    if (enum_rows && !resident)
        return fail(ctx, MUMS_E_UNSUPPORTED, "PairwiseMatchFinder / enumeration tolerance > 1 in the chunked mode "
                                             "needs the resident layout");
    DevBuf epair;   // enum_rows: one chunk's (full ckey, index) pairs + per-head call counts and offsets
    if (enum_rows) {
        HIPCHK(epair.ensure((nmax + 64) * 24 + 256));
        HIPCHK(ctx->tmp.ensure(std::max(ctx->tmp.cap, scan_tmp_bytes(nmax + 1))));
    }
    if (resident) {
        HIPCHK(ctx->recA.ensure((N + 64) * 8));
        HIPCHK(ctx->recB.ensure((N + 64) * 8));
        HIPCHK(ctx->ctab.ensure((nd + nch + 8) * 8 + 64));
        uint64_t* d_cbase = ctx->ctab.as<uint64_t>() + nd;
        HIPCHK(hipMemcpyAsync(d_cbase, cbase.data(), nch * 8, hipMemcpyHostToDevice, st));
        for (uint32_t c = 0; c < nch; ++c)
            HIPCHK(exclusive_scan_u32(hist + (uint64_t)c * nbc8 * T, (uint64_t)nbc8 * T, ctx->tmp.p, nullptr, st));
        if (S) {
            HIPCHK(ctx->side.ensure(N + 64));
            HIPCHK(ctx->cbst.ensure((uint64_t)nch * (nbc + 1) * 4 + (nbc8 + 64) * 4 + 64));
        }
        HIPCHK(launch_seed_scatter_chunk(ctx->ss, gt, ctx->packed.as<uint32_t>(), B, hist, T, 0, 0,
                                         ctx->recA.as<uint64_t>(), st, d_cbase, mb8, S ? ctx->side.as<uint8_t>() : nullptr,
                                         S));
    }
    // the sort buckets of chunk c: from its slice of the MSD histogram, or (S > 0) the split's
    // starts kept in ctx->cbst
    uint32_t* cbst = S ? ctx->cbst.as<uint32_t>() : nullptr;
    auto chunk_starts = [&](uint32_t c, uint64_t n_c, uint32_t* d) -> int {
        if (S) HIPCHK(hipMemcpyAsync(d, cbst + (uint64_t)c * (nbc + 1), (nbc + 1) * 4ull, hipMemcpyDeviceToDevice, st));
        else HIPCHK(seg_bucket_starts(mb > 0 ? hist + (uint64_t)c * nbc * T : nullptr, T, mb, n_c, d, st));
        return MUMS_OK;
    };
    uint64_t P_total = 0, groups = 0;
    double ms_sort = 0, ms_groups = 0, ms_buckets = 0, ms_dom = 0;
    uint64_t dom_bytes = 0, dom_launches = 0;
    auto el = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
        return (double)ms;
    };
    const int npass = seg_onesweep_launches(31);
    // resident layout: every chunk is sorted first (pass 1), so that a MER_REPEAT_LIMIT
    // restart or start points (chunked_restart) see the whole merged stream; then groups /
    // probes / rows per chunk in key order (pass 2), on the live records after a restart.
    // Streaming layout: sort + groups per chunk in one pass (restarts refused).
    int sbuf = 0;
    uint64_t* live_rec = nullptr;            // after a restart: compacted chunks (cbase offsets)
    std::vector<uint64_t> n_live(nch, 0);
    DevBuf& lbst = ctx->rsbst;               // per chunk: compacted bucket starts (nbc + 1)
    for (uint32_t c = 0; c < nch && resident; ++c) {
        const uint32_t dlo = c * nbc8;
        uint64_t n_c = 0;
        for (uint32_t d = dlo; d < dlo + nbc8; ++d) n_c += tot[d];
        uint64_t* rA = ctx->recA.as<uint64_t>() + cbase[c];
        uint64_t* rB = ctx->recB.as<uint64_t>() + cbase[c];
        uint32_t* bstart = ctx->mstart.as<uint32_t>();
        if (S) {   // chunk c's 2^mb8 scatter buckets split by the side digits: rA -> rB
            uint32_t* bst8 = ctx->cbst.as<uint32_t>() + (uint64_t)nch * (nbc + 1);
            uint32_t* out = cbst + (uint64_t)c * (nbc + 1);
            HIPCHK(seg_bucket_starts(mb8 > 0 ? hist + (uint64_t)dlo * T : nullptr, T, mb8, n_c, bst8, st));
            if (n_c) HIPCHK(msd_split(rA, ctx->side.as<uint8_t>() + cbase[c], rB, n_c, mb8, S, bst8, out, ctx->tmp.p, st));
            else HIPCHK(hipMemsetAsync(out, 0, (nbc + 1) * 4ull, st));
        }
        if (n_c == 0) continue;
        HIPCHK(hipEventRecord(ctx->ev[EV_CHAINS], st));
        rc = chunk_starts(c, n_c, bstart);
        if (rc) return rc;
        SegTile* tiles = ctx->tiles.as<SegTile>();
        HIPCHK(build_seg_tiles_from_starts(bstart, mb, n_c, tiles, &dc->ntiles, ctx->tmp.p, st));
        // the sort reads the split's output (rB) when S > 0; sbuf names the buffer holding
        // the sorted chunk (0: recA, 1: recB) either way
        int sb = 0;
        HIPCHK(seg_onesweep_sort(S ? rB : rA, S ? rA : rB, n_c, 31, mb, bstart, ctx->tmp.p, &dc->err, &sb, st,
                                 prof ? ctx->ev_ds : nullptr, 33, mp.repeat_tol == 0 && mp.enum_tol == 1));
        sbuf = S ? 1 - sb : sb;
        HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
        HIPCHK(hipEventSynchronize(ctx->ev[EV_SORT]));
        ms_sort += el(EV_CHAINS, EV_SORT);
        if (prof)
            for (int p = 0; p < npass; ++p) {
                float ms = 0.f;
                (void)hipEventElapsedTime(&ms, ctx->ev_ds[2 * p], ctx->ev_ds[2 * p + 1]);
                ms_dom += ms;
            }
        dom_bytes += n_c * 16 * (uint64_t)npass;
        dom_launches += (uint64_t)npass;
    }
    if (!resident && have_start_points(ctx))
        return fail(ctx, MUMS_E_UNSUPPORTED, "start points in the chunked mode without resident records");
    if (resident) {
        // global starts of the 2^Bt implicit digits (the restart's full keys)
        std::vector<uint64_t> dstart((1ull << Bt) + 1, 0);
        if (S) {
            std::vector<uint32_t> hb((uint64_t)nch * (nbc + 1));
            HIPCHK(hipMemcpyAsync(hb.data(), cbst, hb.size() * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (uint32_t c = 0; c < nch; ++c)
                for (uint32_t j = 0; j < nbc; ++j) dstart[(uint64_t)c * nbc + j] = cbase[c] + hb[(uint64_t)c * (nbc + 1) + j];
            dstart[1ull << Bt] = N;
        } else {
            for (uint32_t d = 0; d < nd; ++d) dstart[d + 1] = dstart[d] + tot[d];
        }
        // the tie workspace (135 GB at 2 x 3 Gbp; its hipMalloc alone is 3-4 s) stays allocated
        // between calls: a FindMatches call's rows and chain scratch live inside it (below)
        ctx->keep_tiebuf = stage < MUMS_STAGE_ALL ? 1 : 2;
        ctx->ties_fixed = false;
        if (wants_tie_order(ctx)) {
            rc = chunked_tie_fix(ctx, sbuf, dstart, st);
            if (rc) return rc;
        }
        rc = chunked_restart(ctx, sbuf, dstart, cbase, nbc, nch, n_live, &live_rec, chunk_starts, st);
        ctx->keep_tiebuf = 0;
        if (rc) return rc;
    }
    // FindMatches: a kept tie workspace is the arena of the probe rows and the sliced chain
    // scratch when both fit in it; else it is released so the tail can allocate them
    const size_t Wrow = (size_t)(G + 1) * 8;
    const size_t chain_need = chain_tmp_bytes(find_chunk() + 1, ctx->table_size, G) + 4096;
    if (stage == MUMS_STAGE_ALL && ctx->tiebuf.p && ctx->tiebuf.cap < chain_need + (N / 4) * Wrow) release_tiebuf(ctx);
    // rows of chunk c's Pc probes / calls appended behind the P_total so far (grown, kept)
    auto grow_rows = [&](uint64_t Pc, uint32_t c) -> int {
        if (P_total + Pc >= (1ull << 32) - 64)   // probe ids are 32-bit (bucket order, chains)
            return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes in one FindMatches");
        const size_t W = Wrow;
        if (ctx->rowsall.cap < (P_total + Pc + 1) * W) {   // grow, keeping the rows so far
            // sized for the chunks to come at this chunk's rate (+10 %): one growth
            // at 2 x 3 Gbp instead of a doubling that would not fit next to the records
            const uint64_t est = (uint64_t)((double)(P_total + Pc) * nch / (c + 1) * 1.1) + 1;
            const size_t want = std::max(P_total + Pc + 1, est) * W;
            DevBuf nb;
            // (inside the kept workspace: all the room the chain scratch leaves, whatever the
            // skewed first-chunk estimate says; outgrowing it moves the rows out below)
            const bool in_tie = !ctx->rowsall.borrowed && ctx->tiebuf.p &&
                                ctx->tiebuf.cap > chain_need + (P_total + Pc + 1) * W &&
                                nb.borrow(ctx->tiebuf, 0, ctx->tiebuf.cap - chain_need);
            if (!in_tie && ctx->tiebuf.p) {   // the rows outgrow the kept workspace: give it up
                HIPCHK(hipStreamSynchronize(st));
                if (ctx->rowsall.borrowed) {   // (rows so far inside it: moved out first)
                    DevBuf keep;
                    HIPCHK(keep.ensure(P_total * W + 64));
                    if (P_total) HIPCHK(hipMemcpyAsync(keep.p, ctx->rowsall.p, P_total * W, hipMemcpyDeviceToDevice, st));
                    HIPCHK(hipStreamSynchronize(st));
                    ctx->rowsall.release();
                    ctx->rowsall = keep;
                }
                release_tiebuf(ctx);
            }
            if (!in_tie) HIPCHK(nb.ensure(want));
            if (P_total) HIPCHK(hipMemcpyAsync(nb.p, ctx->rowsall.p, P_total * W, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
            ctx->rowsall.release();
            ctx->rowsall = nb;
        }
        return MUMS_OK;
    };
    for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t dlo = c * nbc8;
        uint64_t n_c = 0;
        for (uint32_t d = dlo; d < dlo + nbc8; ++d) n_c += tot[d];
        if (n_c == 0) continue;
        uint32_t* slice = hist + (uint64_t)dlo * T;
        const uint64_t o = resident ? cbase[c] : 0;
        uint64_t* rA = ctx->recA.as<uint64_t>() + o;
        uint64_t* rB = ctx->recB.as<uint64_t>() + o;
        HIPCHK(hipEventRecord(ctx->ev[EV_CHAINS], st));   // chunk start (scatter counts as sort)
        uint32_t* bstart = ctx->mstart.as<uint32_t>();
        if (!resident) {
            HIPCHK(exclusive_scan_u32(slice, (uint64_t)nbc8 * T, ctx->tmp.p, nullptr, st));
            HIPCHK(launch_seed_scatter_chunk(ctx->ss, gt, ctx->packed.as<uint32_t>(), B, slice, T, dlo, nbc8, rA, st));
        }
        if (live_rec) {   // the chunk's live records after the restarts
            n_c = n_live[c];
            HIPCHK(hipMemcpyAsync(bstart, lbst.as<uint32_t>() + (uint64_t)c * (nbc + 1), (nbc + 1) * 4ull,
                                  hipMemcpyDeviceToDevice, st));
        } else {
            rc = chunk_starts(c, n_c, bstart);
            if (rc) return rc;
        }
        SegTile* tiles = ctx->tiles.as<SegTile>();
        const uint64_t ub = seg_tiles_upper(n_c, mb);
        HIPCHK(build_seg_tiles_from_starts(bstart, mb, n_c, tiles, &dc->ntiles, ctx->tmp.p, st));
        if (!resident) {
            int buf = 0;
            HIPCHK(seg_onesweep_sort(rA, rB, n_c, 31, mb, bstart, ctx->tmp.p, &dc->err, &buf, st,
                                     prof ? ctx->ev_ds : nullptr, 33, mp.repeat_tol == 0 && mp.enum_tol == 1));
            ctx->sorted_rec = buf ? rB : rA;
            if (prof)
                for (int p = 0; p < npass; ++p) {
                    float ms = 0.f;
                    (void)hipEventElapsedTime(&ms, ctx->ev_ds[2 * p], ctx->ev_ds[2 * p + 1]);
                    ms_dom += ms;
                }
            dom_bytes += n_c * 16 * (uint64_t)npass;
            dom_launches += (uint64_t)npass;
        } else {
            ctx->sorted_rec = live_rec ? live_rec + o : (sbuf ? rB : rA);
        }
        HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
        if (enum_rows) {   // the chunk's AddHashEntry calls as rows (no probe stage)
            uint64_t* ek = epair.as<uint64_t>();
            uint64_t* ei = ek + (n_c + 32);
            uint32_t* ncalls = (uint32_t*)(ei + (n_c + 32));
            uint32_t* off = ncalls + (n_c + 32);
            const PairView<uint64_t, uint64_t> pv{ek, ei};
            uint32_t pc32 = 0;
            if (n_c) {
                HIPCHK(launch_chunk_pairs(ctx->sorted_rec, n_c, bstart, nbc + 1, (uint64_t)c * nbc, ek, ei, st));
                if (ctx->pairwise) HIPCHK(launch_pairwise_count(pv, n_c, gt, ncalls, dc, st));
                else HIPCHK(launch_enum_count(pv, n_c, gt, mp, ncalls, dc, st));
                HIPCHK(hipMemcpyAsync(off, ncalls, n_c * 4, hipMemcpyDeviceToDevice, st));
                HIPCHK(exclusive_scan_u32(off, n_c, ctx->tmp.p, &dc->nprobes, st));
                HIPCHK(hipMemcpyAsync(&pc32, &dc->nprobes, 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                if ((rc = enum_count_check(ctx, st))) return rc;
            }
            const uint64_t Pc = pc32;
            if (stage >= MUMS_STAGE_ALL && Pc) {
                rc = grow_rows(Pc, c);
                if (rc) return rc;
                int64_t* rows = (int64_t*)((char*)ctx->rowsall.p + P_total * Wrow);
                if (ctx->pairwise) HIPCHK(launch_pairwise_emit(pv, n_c, gt, ctx->L, ncalls, off, rows, st));
                else HIPCHK(launch_enum_emit(pv, n_c, gt, mp, ctx->L, ncalls, off, rows, st));
            }
            HIPCHK(hipEventRecord(ctx->ev[EV_GROUPS], st));
            HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
            HIPCHK(hipEventSynchronize(ctx->ev[EV_BUCKETS]));
            ms_groups += el(EV_SORT, EV_GROUPS);
            P_total += Pc;
            continue;
        }
        if (n_c) {
            rc = groups_dispatch<RecViewT<33>>(ctx, RecViewT<33>{ctx->sorted_rec}, tiles, ub, mp, ps.probe_info,
                                               ps.probe_bucket, ps.slot_info, ps.slot_bucket, st);
            if (rc) return rc;
        } else {
            HIPCHK(hipMemsetAsync(&dc->nprobes, 0, 4, st));
            HIPCHK(hipMemsetAsync(&dc->ngroups, 0, 4, st));
        }
        rc = finish_seeds(ctx, ps, st);
        if (rc) return rc;
        if (ctx->hc.repeat_limit && !resident)
            return fail(ctx, MUMS_E_UNSUPPORTED, "chunked mode without resident records: a seed group above "
                                                 "MER_REPEAT_LIMIT (the SearchRange restart needs all chunks resident)");
        HIPCHK(hipEventSynchronize(ctx->ev[EV_BUCKETS]));
        if (!resident) ms_sort += el(EV_CHAINS, EV_SORT);
        ms_groups += el(EV_SORT, EV_GROUPS);
        ms_buckets += el(EV_GROUPS, EV_BUCKETS);
        groups += ctx->hc.ngroups;
        const uint64_t Pc = ctx->P;
        if (stage >= MUMS_STAGE_ALL && Pc) {
            rc = grow_rows(Pc, c);
            if (rc) return rc;
            rc = materialize_dispatch<RecViewT<33>>(ctx, RecViewT<33>{ctx->sorted_rec}, mp, st,
                                                    (int64_t*)((char*)ctx->rowsall.p + P_total * Wrow));
            if (rc) return rc;
        }
        P_total += Pc;
    }
    ctx->P = P_total;
    ctx->stage_done = MUMS_STAGE_SEEDS;
    if (live_rec) {   // the report counts the groups above MER_REPEAT_LIMIT of the whole stream
        ctx->hc.repeat_limit = ctx->cr_cands;
        HIPCHK(h2d_sync(&dc->repeat_limit, &ctx->cr_cands, 8, ctx->stream));
    }
    if (stage >= MUMS_STAGE_ALL) {
        int tbits = 1;
        while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)ctx->table_size) ++tbits;
        ctx->probe_info = nullptr;
        if (P_total > find_chunk()) {   // the rows hold everything FindMatches reads: the records are dead
            HIPCHK(hipStreamSynchronize(st));
            for (DevBuf* b : {&ctx->pbuf, &ctx->mprobe, &ctx->tiles}) b->release();
            ctx->sorted_rec = nullptr;
            ctx->probe_info = nullptr;
            (void)ctx->rowtmp.borrow(ctx->recB, 0, (P_total + 64) * 16 + 8192);   // sliced FindMatches arena
        }
        if (P_total) {
            HIPCHK(ctx->rowtmp.ensure((P_total + 64) * 16 + 8192));
            uint32_t* bkt = (uint32_t*)ctx->rowtmp.p;
            HIPCHK(launch_row_buckets(ctx->rowsall.as<int64_t>(), P_total, G, ctx->table_size, nullptr, 0, bkt, st));
            rc = sort_row_keys(ctx, bkt, P_total, tbits, st);
            if (rc) return rc;
        }
        HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
        rc = find_tail(ctx, mp, ctx->packed.as<uint32_t>(), [&](MatProbes* v) {
            v->rows = ctx->rowsall.as<int64_t>();
            return MUMS_OK;
        }, st);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
    fill_stats(ctx, N);
    mums_stats& s = ctx->st;
    s.probes = P_total;
    s.groups = groups;
    s.ms_sort = ms_sort;
    s.ms_groups = ms_groups;
    s.ms_buckets = ms_buckets;
    s.chunks = nch;
    s.sort_passes = (uint64_t)npass;
    s.key_bytes = 8;
    s.ms_dominant = prof ? ms_dom : 0.0;
    s.dominant_bytes = prof ? dom_bytes : 0;
    s.dominant_launches = prof ? dom_launches : 0;
    return MUMS_OK;
}

}  // namespace

int mums_shard_bucket_counts(mums_ctx* ctx, uint64_t* counts) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (!counts) return fail(ctx, MUMS_E_INVALID, "null counts");
    HIPCHK(hipSetDevice(ctx->device));
    const uint32_t Tb = ctx->table_size;
    std::fill(counts, counts + Tb, 0ull);
    hipStream_t st = ctx->stream;
    rc = shard_chunk_rows(ctx, st);
    if (rc) return rc;
    if (ctx->P == 0) return MUMS_OK;
    DevCounters* dc = ctx->counters.as<DevCounters>();
    if (shard_rows_from_all(ctx)) {   // the buckets of every chunk's rows (key order kept per bucket)
        int tbits = 1;
        while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)Tb) ++tbits;
        HIPCHK(ctx->rowtmp.ensure((ctx->P + 64) * 16 + 8192));
        uint32_t* bkt = (uint32_t*)ctx->rowtmp.p;
        HIPCHK(launch_row_buckets(ctx->rowsall.as<int64_t>(), ctx->P, ctx->gt.G, Tb, nullptr, 0, bkt, st));
        rc = sort_row_keys(ctx, bkt, ctx->P, tbits, st);
        if (rc) return rc;
    }
    HIPCHK(ctx->bstart.ensure((size_t)Tb * 4));
    HIPCHK(ctx->bend.ensure((size_t)Tb * 4));
    HIPCHK(hipMemsetAsync(ctx->bstart.p, 0, (size_t)Tb * 4, st));
    HIPCHK(hipMemsetAsync(ctx->bend.p, 0, (size_t)Tb * 4, st));
    HIPCHK(launch_bucket_ranges(ctx->sorted_buckets, ctx->P, ctx->bstart.as<uint32_t>(), ctx->bend.as<uint32_t>(),
                                &dc->max_bucket, st));
    std::vector<uint32_t> b0(Tb), b1(Tb);
    HIPCHK(hipMemcpyAsync(b0.data(), ctx->bstart.p, (size_t)Tb * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(b1.data(), ctx->bend.p, (size_t)Tb * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint32_t b = 0; b < Tb; ++b) counts[b] = b1[b] - b0[b];
    return MUMS_OK;
}

int mums_shard_probe_rows(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_rows,
                          uint64_t capacity_rows, uint64_t* counts) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (nranks == 0 || nranks > 1024 || !bounds || !counts) return fail(ctx, MUMS_E_INVALID, "bad rank bounds");
    if (bounds[0] != 0 || bounds[nranks] != ctx->table_size)
        return fail(ctx, MUMS_E_INVALID, "bucket bounds must cover [0, table_size)");
    for (uint32_t r = 0; r < nranks; ++r)
        if (bounds[r] > bounds[r + 1]) return fail(ctx, MUMS_E_INVALID, "bucket bounds must not decrease");
    const uint64_t P = ctx->P;
    if (capacity_rows < P) return fail(ctx, MUMS_E_INVALID, "row buffer too small");
    std::fill(counts, counts + nranks, 0ull);
    if (P == 0) return MUMS_OK;
    if (!d_rows) return fail(ctx, MUMS_E_INVALID, "null row buffer");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    const int64_t* src = ctx->rowsall.as<int64_t>();   // a chunked merge: every chunk's rows
    if (!shard_rows_from_all(ctx)) {
        rc = materialize_seeds(ctx, mp, st);
        if (rc) return rc;
        src = ctx->mprobe.as<int64_t>();
    } else if (!ctx->shard_rows_built) {
        return fail(ctx, MUMS_E_INVALID, "mums_shard_bucket_counts first (a chunked merge's rows)");
    }
    const int G = ctx->gt.G;
    HIPCHK(ctx->rowtmp.ensure((P + 64) * 16 + 8192));
    HIPCHK(ctx->keybuf.ensure((size_t)(nranks + 1) * 8 + 64));
    HIPCHK(hipMemcpyAsync(ctx->keybuf.p, bounds, (size_t)(nranks + 1) * 4, hipMemcpyHostToDevice, st));
    uint32_t* dest = (uint32_t*)ctx->rowtmp.p;
    HIPCHK(launch_row_buckets(src, P, G, ctx->table_size, ctx->keybuf.as<uint32_t>(), nranks, dest, st));
    rc = sort_row_keys(ctx, dest, P, std::max(1, ceil_log2(nranks)), st);   // stable: key order per rank
    if (rc) return rc;
    const uint32_t* perm = ctx->sorted_ids;
    HIPCHK(launch_gather_rows(src, perm, P, G, d_rows, st));
    // rows per destination rank = run lengths of the sorted destinations
    std::vector<uint32_t> sd(P);
    HIPCHK(hipMemcpyAsync(sd.data(), ctx->sorted_buckets, P * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint64_t i = 0; i < P; ++i) ++counts[sd[i]];
    return MUMS_OK;
}

// ---- sharded FindMatches with the chains labelled where the probes are -----
// On related genomes ~95 % of the probes share one hash bucket (the main diagonal's offset,
// MemHash.cpp:213), so labelling chains on the bucket owner left one rank with the chain
// stage.  Instead every rank labels the chains of ITS probes (its seed-stage key range, key
// order) against the all-gathered packed genomes -- the line sort, links and walks divide
// like the seed stage -- and ships each chain's entry with the rows to the bucket owner
// (all probes of a chain share its bucket).  The owner merges equal entries (a chain whose
// probes sit on several ranks is labelled by each of them) and replays its buckets.
int mums_shard_chain_label(mums_ctx* ctx, const uint32_t* d_packed_all, uint64_t* nchains) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (ctx->P && !d_packed_all) return fail(ctx, MUMS_E_INVALID, "null packed genomes");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    rc = shard_chunk_rows(ctx, st);   // a chunked merge / enumeration: every row
    if (rc) return rc;
    const uint64_t P = ctx->P;
    const int G = ctx->gt.G;
    const int64_t* src = ctx->rowsall.as<int64_t>();
    if (!shard_rows_from_all(ctx)) {
        rc = materialize_seeds(ctx, mp, st);
        if (rc) return rc;
        src = ctx->mprobe.as<int64_t>();
    }
    ctx->lab_rows = src;
    ctx->lab_nch = 0;
    ctx->lab_p = P;
    ctx->lab_ms = 0;
    if (nchains) *nchains = 0;
    if (P == 0) return MUMS_OK;
    if (P >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes on one rank");
    uint64_t words = 0;
    (void)layout_packed(ctx->gt, &words);   // the walks read every genome at its global word offset
    const uint64_t C = std::min<uint64_t>(P, find_chunk());
    HIPCHK(ctx->chain_of.ensure((P + 1) * 4));
    HIPCHK(ctx->chain_tmp.ensure(chain_tmp_bytes(C + 1, ctx->table_size, G)));
    HIPCHK(ctx->radix_tmp.ensure(chain_radix_tmp_bytes(C + 1)));
    HIPCHK(ctx->tmp.ensure(scan_tmp_bytes(C + 1)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    MatProbes v{};
    v.rows = src;
    uint64_t nloc = 0;
    if (G <= 4) rc = label_slices<4>(ctx, v, d_packed_all, mp, st, &nloc);
    else if (G <= 8) rc = label_slices<8>(ctx, v, d_packed_all, mp, st, &nloc);
    else if (G <= 16) rc = label_slices<16>(ctx, v, d_packed_all, mp, st, &nloc);
    else if (G <= 32) rc = label_slices<32>(ctx, v, d_packed_all, mp, st, &nloc);
    else rc = label_slices<64>(ctx, v, d_packed_all, mp, st, &nloc);
    if (rc == MUMS_OK && P > C) {   // several slices: their equal entries merged here already
        DevCounters* dc = ctx->counters.as<DevCounters>();
        const size_t W = (size_t)(G + 2) * 8;
        HIPCHK(ctx->chain_tmp.ensure(chain_merge_tmp_bytes(nloc)));
        HIPCHK(ctx->pool.ensure((nloc + 1) * W));
        HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(nloc + 1)));
        HIPCHK(ctx->fk.ensure((nloc + 1) * 4));
        HIPCHK(launch_chain_merge(ctx->pool_loc.as<int64_t>(), nloc, G, ctx->chain_of.as<uint32_t>(), P,
                                  ctx->pool.as<int64_t>(), ctx->chain_tmp.p, ctx->radix_tmp.p, ctx->tmp.p, &dc->nchains,
                                  st, ctx->fkloc.as<uint32_t>(), ctx->fk.as<uint32_t>()));
        uint32_t nc = 0;
        HIPCHK(hipMemcpyAsync(&nc, &dc->nchains, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::swap(ctx->pool, ctx->pool_loc);
        std::swap(ctx->fk, ctx->fkloc);
        nloc = nc;
    }
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    ctx->lab_nch = nloc;
    ctx->lab_ms = ms;
    if (nchains) *nchains = nloc;
    return MUMS_OK;
}

// The rank's probes' and chains' destination ranks (bucket ranges bounds[0..nranks]) in
// ctx->labx: pdest per probe, the chains stably sorted by destination (cperm, scdest, cinv) and
// the per-destination entry counts.  Layout of labx: pdest, pinv [P + 64]; cdest, ckB, ciA, ciB,
// cinv, ckA2 [nch + 64]; rstart [nranks + 1]; cstart [nranks + 1]; scratch [2 nranks + 64].
struct ChainDests {
    uint32_t *pdest, *pinv, *cdest, *ckB, *ciA, *ciB, *cinv, *ckA2, *rstart, *cstart, *scratch;
    const uint32_t* scdest = nullptr;
    const uint32_t* cperm = nullptr;
};
static int chain_dests(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, ChainDests* cd,
                       uint64_t* entry_counts, hipStream_t st) {
    if (nranks == 0 || nranks > 1024 || !bounds || !entry_counts) return fail(ctx, MUMS_E_INVALID, "bad rank bounds");
    if (bounds[0] != 0 || bounds[nranks] != ctx->table_size)
        return fail(ctx, MUMS_E_INVALID, "bucket bounds must cover [0, table_size)");
    for (uint32_t r = 0; r < nranks; ++r)
        if (bounds[r] > bounds[r + 1]) return fail(ctx, MUMS_E_INVALID, "bucket bounds must not decrease");
    const uint64_t P = ctx->P, nch = ctx->lab_nch;
    const int G = ctx->gt.G;
    const int bits = std::max(1, ceil_log2(nranks));
    HIPCHK(ctx->labx.ensure((P + 64) * 8 + (nch + 64) * 24 + (size_t)(nranks + 1) * 8 + (size_t)(2 * nranks + 64) * 4 +
                            4096));
    cd->pdest = ctx->labx.as<uint32_t>();
    cd->pinv = cd->pdest + (P + 64);
    cd->cdest = cd->pinv + (P + 64);
    cd->ckB = cd->cdest + (nch + 64);
    cd->ciA = cd->ckB + (nch + 64);
    cd->ciB = cd->ciA + (nch + 64);
    cd->cinv = cd->ciB + (nch + 64);
    cd->ckA2 = cd->cinv + (nch + 64);
    cd->rstart = cd->ckA2 + (nch + 64);
    cd->cstart = cd->rstart + (nranks + 1);
    cd->scratch = cd->cstart + (nranks + 1);
    HIPCHK(ctx->keybuf.ensure((size_t)(nranks + 1) * 8 + 64));
    HIPCHK(hipMemcpyAsync(ctx->keybuf.p, bounds, (size_t)(nranks + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(launch_row_buckets(ctx->lab_rows, P, G, ctx->table_size, ctx->keybuf.as<uint32_t>(), nranks, cd->pdest, st));
    std::fill(entry_counts, entry_counts + nranks, 0ull);
    if (nch) {   // chains: destination of the first probe (all probes of a chain share its bucket), stable
        HIPCHK(launch_chain_dest(ctx->fkloc.as<uint32_t>(), nch, cd->pdest, cd->cdest, st));
        HIPCHK(hipMemcpyAsync(cd->ckA2, cd->cdest, nch * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(std::max(P, nch) + 1)));
        int out = 0;
        HIPCHK(radix_sort<uint32_t>(cd->ckA2, nullptr, nch, bits, cd->ckB, cd->ciA, cd->ckA2, cd->ciB,
                                    ctx->radix_tmp.p, &out, st));
        cd->scdest = out ? cd->ckA2 : cd->ckB;
        cd->cperm = out ? cd->ciB : cd->ciA;
        HIPCHK(launch_inverse_perm(cd->cperm, nch, cd->cinv, st));
        std::vector<uint32_t> scd(nch);
        HIPCHK(hipMemcpyAsync(scd.data(), cd->scdest, nch * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (uint64_t i = 0; i < nch; ++i) ++entry_counts[scd[i]];
    }
    return MUMS_OK;
}

int mums_shard_chain_export(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_rows, uint32_t* d_tags,
                            uint64_t capacity_rows, int64_t* d_entries, uint32_t* d_first, uint64_t capacity_entries,
                            uint64_t* row_counts, uint64_t* entry_counts) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (!row_counts || !entry_counts) return fail(ctx, MUMS_E_INVALID, "bad rank bounds");
    const uint64_t P = ctx->P, nch = ctx->lab_nch;
    if (nranks == 0 || nranks > 1024) return fail(ctx, MUMS_E_INVALID, "bad rank bounds");
    std::fill(row_counts, row_counts + nranks, 0ull);
    std::fill(entry_counts, entry_counts + nranks, 0ull);
    if (P == 0) return MUMS_OK;
    if (!ctx->lab_rows) return fail(ctx, MUMS_E_INVALID, "mums_shard_chain_label first");
    if (capacity_rows < P || capacity_entries < nch) return fail(ctx, MUMS_E_INVALID, "export buffer too small");
    if (!d_rows || !d_tags || (nch && (!d_entries || !d_first))) return fail(ctx, MUMS_E_INVALID, "null export buffer");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int G = ctx->gt.G;
    const int bits = std::max(1, ceil_log2(nranks));
    HIPCHK(ctx->rowtmp.ensure((P + 64) * 16 + 8192));
    ChainDests cd{};
    if ((rc = chain_dests(ctx, nranks, bounds, &cd, entry_counts, st))) return rc;
    // rows: stable by destination (key order per destination)
    uint32_t* dest = (uint32_t*)ctx->rowtmp.p;
    HIPCHK(hipMemcpyAsync(dest, cd.pdest, P * 4, hipMemcpyDeviceToDevice, st));
    rc = sort_row_keys(ctx, dest, P, bits, st);
    if (rc) return rc;
    const uint32_t* perm = ctx->sorted_ids;
    const uint32_t* sdest = ctx->sorted_buckets;
    HIPCHK(launch_inverse_perm(perm, P, cd.pinv, st));
    HIPCHK(launch_gather_rows(ctx->lab_rows, perm, P, G, d_rows, st));
    std::vector<uint32_t> sd(P);
    HIPCHK(hipMemcpyAsync(sd.data(), sdest, P * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint64_t i = 0; i < P; ++i) ++row_counts[sd[i]];
    std::vector<uint32_t> starts(2 * (nranks + 1), 0);
    for (uint32_t r = 0; r < nranks; ++r) {
        starts[r + 1] = starts[r] + (uint32_t)row_counts[r];
        starts[nranks + 1 + r + 1] = starts[nranks + 1 + r] + (uint32_t)entry_counts[r];
    }
    HIPCHK(hipMemcpyAsync(cd.rstart, starts.data(), starts.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(launch_chain_tags(ctx->chain_of.as<uint32_t>(), perm, sdest, P, cd.cinv, cd.cstart, d_tags, st));
    HIPCHK(launch_chain_entries_out(ctx->pool_loc.as<int64_t>(), ctx->fkloc.as<uint32_t>(), cd.cperm, cd.scdest, nch, G,
                                    cd.pinv, cd.rstart, d_entries, d_first, st));
    HIPCHK(hipStreamSynchronize(st));   // (starts is a host vector)
    return MUMS_OK;
}

// ---- sharded FindMatches, kept-probe export (default in mums_shard_run) ----------------
// Only two kinds of AddHashEntry call can touch a bucket vector (the replay from kept probes,
// replay.hip): a chain's first call, and a suspicious one (its first-genome start at or past
// the chain's next_s).  Whether a probe is either depends on the chains of the whole bucket,
// which only its owner sees: so the entries go first (mums_shard_chain_entries), the owner
// answers per entry {next_s, first} (mums_shard_entry_thresholds), and the ranks then send only
// those probes (mums_shard_kept_export; on related genomes ~5 % of them) -- every other one
// collides with its chain entry and is counted (dropped_counts) instead of sent.
int mums_shard_chain_entries(mums_ctx* ctx, uint32_t nranks, const uint32_t* bounds, int64_t* d_entries,
                             uint64_t capacity_entries, uint64_t* entry_counts) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    ctx->kx_nranks = 0;
    if (nranks == 0 || nranks > 1024 || !entry_counts) return fail(ctx, MUMS_E_INVALID, "bad rank bounds");
    std::fill(entry_counts, entry_counts + nranks, 0ull);
    const uint64_t P = ctx->P, nch = ctx->lab_nch;
    if (P && !ctx->lab_rows) return fail(ctx, MUMS_E_INVALID, "mums_shard_chain_label first");
    if (capacity_entries < nch) return fail(ctx, MUMS_E_INVALID, "export buffer too small");
    if (nch && !d_entries) return fail(ctx, MUMS_E_INVALID, "null export buffer");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    ChainDests cd{};
    if (P && (rc = chain_dests(ctx, nranks, bounds, &cd, entry_counts, st))) return rc;
    ctx->kx_estart.assign(nranks + 1, 0);
    for (uint32_t r = 0; r < nranks; ++r) ctx->kx_estart[r + 1] = ctx->kx_estart[r] + (uint32_t)entry_counts[r];
    if (nch)
        HIPCHK(launch_chain_entries_out(ctx->pool_loc.as<int64_t>(), ctx->fkloc.as<uint32_t>(), cd.cperm, cd.scdest,
                                        nch, ctx->gt.G, nullptr, nullptr, d_entries, nullptr, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->kx_nranks = nranks;
    return MUMS_OK;
}

int mums_shard_entry_thresholds(mums_ctx* ctx, const int64_t* d_entries, uint64_t nentries, uint32_t* d_thr) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (nentries == 0) return MUMS_OK;
    if (!d_entries || !d_thr) return fail(ctx, MUMS_E_INVALID, "null entries / thresholds");
    if (nentries >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 chain entries on one rank");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK(ctx->pool.ensure((nentries + 1) * (size_t)(ctx->gt.G + 2) * 8));
    HIPCHK(ctx->chain_tmp.ensure(chain_thr_tmp_bytes(nentries + 1)));
    HIPCHK(ctx->radix_tmp.ensure(radix_tmp_bytes(nentries + 1)));
    HIPCHK(ctx->tmp.ensure(scan_tmp_bytes(nentries + 1)));
    uint32_t nm = 0;
    HIPCHK(launch_chain_thresholds(d_entries, nentries, ctx->gt, mp, ctx->pool.as<int64_t>(), ctx->chain_tmp.p,
                                   ctx->radix_tmp.p, ctx->tmp.p, &dc->nchains, &nm, (uint2*)d_thr, st));
    HIPCHK(hipStreamSynchronize(st));
    if (getenv("MUMS_DEV_SHARD_DEBUG")) {   // development: what the owner answers
        std::vector<uint32_t> h(2 * nentries);
        HIPCHK(hipMemcpy(h.data(), d_thr, nentries * 8, hipMemcpyDeviceToHost));
        uint64_t nfirst = 0, nnone = 0;
        for (uint64_t e = 0; e < nentries; ++e) {
            nfirst += h[2 * e + 1];
            nnone += h[2 * e] == 0xFFFFFFFFu;
        }
        fprintf(stderr, "entry_thresholds: %llu entries -> %u chains, first %llu, next_s none %llu, e0 {%u,%u} e1 {%u,%u}\n",
                (unsigned long long)nentries, nm, (unsigned long long)nfirst, (unsigned long long)nnone, h[0], h[1],
                nentries > 1 ? h[2] : 0u, nentries > 1 ? h[3] : 0u);
    }
    return MUMS_OK;
}

int mums_shard_kept_export(mums_ctx* ctx, uint32_t nranks, const uint32_t* d_thr, int64_t* d_rows, uint32_t* d_tags,
                           uint64_t capacity_rows, uint32_t* d_first, uint64_t* row_counts, uint64_t* dropped_counts) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (!row_counts || !dropped_counts || nranks == 0 || nranks > 1024)
        return fail(ctx, MUMS_E_INVALID, "bad rank count");
    if (ctx->kx_nranks != nranks) return fail(ctx, MUMS_E_INVALID, "mums_shard_chain_entries first (same ranks)");
    std::fill(row_counts, row_counts + nranks, 0ull);
    std::fill(dropped_counts, dropped_counts + nranks, 0ull);
    const uint64_t P = ctx->P, nch = ctx->lab_nch;
    if (P == 0) return MUMS_OK;
    if (nch && (!d_thr || !d_first)) return fail(ctx, MUMS_E_INVALID, "null thresholds / first rows");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int G = ctx->gt.G;
    ChainDests cd{};   // the layout chain_dests left in labx
    cd.pdest = ctx->labx.as<uint32_t>();
    cd.pinv = cd.pdest + (P + 64);
    cd.cdest = cd.pinv + (P + 64);
    cd.ckB = cd.cdest + (nch + 64);
    cd.ciA = cd.ckB + (nch + 64);
    cd.ciB = cd.ciA + (nch + 64);
    cd.cinv = cd.ciB + (nch + 64);
    cd.ckA2 = cd.cinv + (nch + 64);
    cd.rstart = cd.ckA2 + (nch + 64);
    cd.cstart = cd.rstart + (nranks + 1);
    cd.scratch = cd.cstart + (nranks + 1);
    HIPCHK(ctx->rowtmp.ensure((P + 64) * 16 + 8192));
    uint32_t* dest = (uint32_t*)ctx->rowtmp.p;
    HIPCHK(launch_kept_dest(ctx->lab_rows, P, G, ctx->chain_of.as<uint32_t>(), cd.cinv, (const uint2*)d_thr,
                            ctx->fkloc.as<uint32_t>(), cd.pdest, nranks, dest, st));
    rc = sort_row_keys(ctx, dest, P, std::max(1, ceil_log2(2ull * nranks)), st);   // stable: key order per destination
    if (rc) return rc;
    const uint32_t* perm = ctx->sorted_ids;
    const uint32_t* sdest = ctx->sorted_buckets;
    std::vector<uint32_t> first(2 * nranks, (uint32_t)P);
    HIPCHK(hipMemcpyAsync(cd.scratch, first.data(), first.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(launch_dest_first(sdest, P, cd.scratch, st));
    HIPCHK(hipMemcpyAsync(first.data(), cd.scratch, first.size() * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint64_t end = P;
    for (int64_t d = 2 * (int64_t)nranks - 1; d >= 0; --d) {
        const uint64_t c = first[d] == (uint32_t)P ? 0 : end - first[d];
        if (c) end = first[d];
        if (d < (int64_t)nranks) row_counts[d] = c;
        else dropped_counts[d - nranks] = c;
    }
    uint64_t K = 0;
    std::vector<uint32_t> starts(2 * (nranks + 1), 0);
    for (uint32_t r = 0; r < nranks; ++r) {
        starts[r + 1] = starts[r] + (uint32_t)row_counts[r];
        starts[nranks + 1 + r + 1] = ctx->kx_estart[r + 1];
        K += row_counts[r];
    }
    if (capacity_rows < K) return fail(ctx, MUMS_E_INVALID, "export buffer too small");
    if (K && (!d_rows || !d_tags)) return fail(ctx, MUMS_E_INVALID, "null export buffer");
    std::vector<uint32_t> rcount(nranks);
    for (uint32_t r = 0; r < nranks; ++r) rcount[r] = (uint32_t)row_counts[r];
    HIPCHK(hipMemcpyAsync(cd.rstart, starts.data(), starts.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(cd.scratch, rcount.data(), nranks * 4, hipMemcpyHostToDevice, st));
    HIPCHK(launch_gather_rows(ctx->lab_rows, perm, K, G, d_rows, st));
    HIPCHK(launch_chain_tags(ctx->chain_of.as<uint32_t>(), perm, sdest, K, cd.cinv, cd.cstart, d_tags, st));
    // the chains in export order: their destinations are kx_estart's blocks
    if (nch) {
        std::vector<uint32_t> xd(nch);
        for (uint32_t r = 0; r < nranks; ++r)
            for (uint32_t x = ctx->kx_estart[r]; x < ctx->kx_estart[r + 1]; ++x) xd[x] = r;
        HIPCHK(hipMemcpyAsync(cd.ckB, xd.data(), nch * 4, hipMemcpyHostToDevice, st));
        HIPCHK(launch_entry_first(cd.ckB, nch, cd.scratch, perm, sdest, K, ctx->chain_of.as<uint32_t>(), cd.cinv,
                                  cd.rstart, d_first, st));
        HIPCHK(hipStreamSynchronize(st));   // (xd is a host vector)
    }
    HIPCHK(hipStreamSynchronize(st));   // (starts / rcount are host vectors)
    if (getenv("MUMS_DEV_SHARD_DEBUG")) {
        uint64_t dr = 0;
        for (uint32_t r = 0; r < nranks; ++r) dr += dropped_counts[r];
        fprintf(stderr, "kept_export: P %llu chains %llu kept %llu dropped %llu\n", (unsigned long long)P,
                (unsigned long long)nch, (unsigned long long)K, (unsigned long long)dr);
    }
    return MUMS_OK;
}

int mums_shard_find_kept(mums_ctx* ctx, const int64_t* d_rows, const uint32_t* d_tags, uint64_t nrows,
                         const int64_t* d_entries, const uint32_t* d_first, uint64_t nentries, uint32_t nsrc,
                         const uint64_t* src_rows, const uint64_t* src_entries, uint64_t dropped,
                         const uint32_t* d_packed_all) {
    ctx->kept_rows = true;
    const int rc = mums_shard_find_labelled(ctx, d_rows, d_tags, nrows, d_entries, d_first, nentries, nsrc, src_rows,
                                            src_entries, d_packed_all);
    ctx->kept_rows = false;
    if (rc) return rc;
    ctx->own_dropped = dropped;
    ctx->st.collision_count += dropped;   // every probe not sent collides with its chain entry
    ctx->st.probes = nrows + dropped;     // the AddHashEntry calls of the owned buckets
    return MUMS_OK;
}

int mums_shard_chain_info(mums_ctx* ctx, uint64_t* info) {
    if (check_ctx(ctx) || !info) return MUMS_E_INVALID;
    info[0] = ctx->lab_p;
    info[1] = ctx->lab_nch;
    info[2] = (uint64_t)(ctx->lab_ms * 1000.0 + 0.5);
    info[3] = ctx->own_rows;   // rows this rank replayed as bucket owner (kept or all)
    return MUMS_OK;
}

int mums_shard_packed_info(mums_ctx* ctx, uint64_t* word_offset, uint64_t* nwords, uint64_t* total_words) {
    int rc = shard_seeds_done(ctx, true);
    if (rc) return rc;
    GenomeTable g = ctx->gt;
    uint64_t total = 0;
    (void)layout_packed(g, &total);
    if (total_words) *total_words = total;
    if (ctx->slice) {
        // a position slice's packed words are those of bases [begin, end) of its genome
        // (16 bases a word; the genome's last slice also holds the tail and pad words):
        // word-exact only for slices starting on a 64-base boundary (shard.genome_slices)
        const uint32_t gi = ctx->slice_genome;
        const uint64_t b0 = ctx->slice_begin, b1 = ctx->slice_end;
        const bool last = b1 >= ctx->gt.m[gi];
        if (b0 % 64 || (!last && b1 % 64))
            return fail(ctx, MUMS_E_UNSUPPORTED, "sharded FindMatches on position slices needs 64-base slice bounds");
        const uint64_t w0 = g.woff[gi] + b0 / 16;
        const uint64_t w1 = last ? g.woff[gi + 1] : g.woff[gi] + b1 / 16;
        GenomeTable lt = ctx->lgt;
        uint64_t local = 0;
        (void)layout_packed(lt, &local);
        if (w1 - w0 > local) return fail(ctx, MUMS_E_INVALID, "slice ASCII shorter than its packed words");
        if (word_offset) *word_offset = w0;
        if (nwords) *nwords = w1 - w0;
        return MUMS_OK;
    }
    const uint32_t nl = (uint32_t)ctx->genomes.size();
    if (word_offset) *word_offset = g.woff[ctx->shard_first];
    if (nwords) *nwords = g.woff[ctx->shard_first + nl] - g.woff[ctx->shard_first];
    return MUMS_OK;
}

int mums_shard_packed_copy(mums_ctx* ctx, uint32_t* d_dst) {
    uint64_t off = 0, n = 0, tot = 0;
    int rc = mums_shard_packed_info(ctx, &off, &n, &tot);
    if (rc) return rc;
    if (n == 0) return MUMS_OK;
    if (!d_dst) return fail(ctx, MUMS_E_INVALID, "null destination");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(d_dst, ctx->packed.p, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return MUMS_OK;
}

int mums_shard_find_labelled(mums_ctx* ctx, const int64_t* d_rows, const uint32_t* d_tags, uint64_t nrows,
                             const int64_t* d_entries, const uint32_t* d_first, uint64_t nentries, uint32_t nsrc,
                             const uint64_t* src_rows, const uint64_t* src_entries, const uint32_t* d_packed_all) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (nrows && (!d_rows || !d_tags || !d_packed_all || !d_entries || !d_first))
        return fail(ctx, MUMS_E_INVALID, "null rows / chain labels / packed genomes");
    if (nrows >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes on one rank");
    if (nsrc == 0 || !src_rows || !src_entries) return fail(ctx, MUMS_E_INVALID, "no source blocks");
    uint64_t sr = 0, se = 0;
    for (uint32_t s = 0; s < nsrc; ++s) {
        sr += src_rows[s];
        se += src_entries[s];
    }
    if (sr != nrows || se != nentries) return fail(ctx, MUMS_E_INVALID, "source blocks do not add up");
    if (nentries > nrows && !ctx->kept_rows) return fail(ctx, MUMS_E_INVALID, "more chains than probes");
    ctx->own_rows = nrows;
    ctx->own_dropped = 0;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int G = ctx->gt.G;
    // the labels, rebased: a row's entry index past the entry blocks of the sources before it,
    // an entry's first probe past their row blocks
    HIPCHK(ctx->chain_of.ensure((nrows + 1) * 4));
    HIPCHK(ctx->pool_loc.ensure((nentries + 1) * (size_t)(G + 2) * 8));
    HIPCHK(ctx->fkloc.ensure((nentries + 1) * 4));
    if (nrows) HIPCHK(hipMemcpyAsync(ctx->chain_of.p, d_tags, nrows * 4, hipMemcpyDeviceToDevice, st));
    if (nentries) {
        HIPCHK(hipMemcpyAsync(ctx->pool_loc.p, d_entries, nentries * (size_t)(G + 2) * 8, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(ctx->fkloc.p, d_first, nentries * 4, hipMemcpyDeviceToDevice, st));
    }
    uint64_t ro = 0, eo = 0;
    for (uint32_t s = 0; s < nsrc; ++s) {
        if (s) {
            HIPCHK(launch_add_offset(ctx->chain_of.as<uint32_t>() + ro, src_rows[s], (uint32_t)eo, st));
            HIPCHK(launch_add_offset(ctx->fkloc.as<uint32_t>() + eo, src_entries[s], (uint32_t)ro, st));
        }
        ro += src_rows[s];
        eo += src_entries[s];
    }
    ctx->prelabelled = true;
    ctx->prelab_n = nentries;
    rc = mums_shard_find(ctx, d_rows, nrows, d_packed_all);
    ctx->prelabelled = false;
    ctx->prelab_n = 0;
    return rc;
}

int mums_shard_find(mums_ctx* ctx, const int64_t* d_rows, uint64_t nrows, const uint32_t* d_packed_all) {
    int rc = shard_seeds_done(ctx);
    if (rc) return rc;
    if (nrows && (!d_rows || !d_packed_all)) return fail(ctx, MUMS_E_INVALID, "null rows / packed genomes");
    if (nrows >= (1ull << 32) - 64) return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed probes on one rank");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    uint64_t words = 0;
    (void)layout_packed(ctx->gt, &words);        // chain walks read every genome at its global offset
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    for (int e = EV_KEYS; e <= EV_GROUPS; ++e) HIPCHK(hipEventRecord(ctx->ev[e], st));
    ctx->P = nrows;
    ctx->probe_info = nullptr;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    int tbits = 1;
    while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)ctx->table_size) ++tbits;
    if (nrows) {
        HIPCHK(ctx->rowtmp.ensure((nrows + 64) * 16 + 8192));
        uint32_t* bkt = (uint32_t*)ctx->rowtmp.p;
        HIPCHK(launch_row_buckets(d_rows, nrows, ctx->gt.G, ctx->table_size, nullptr, 0, bkt, st));
        rc = sort_row_keys(ctx, bkt, nrows, tbits, st);   // stable: key order inside every bucket
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
    rc = find_tail(ctx, mp, d_packed_all, [&](MatProbes* v) {
        v->rows = d_rows;
        return MUMS_OK;
    }, st);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));
    fill_stats(ctx, 0);
    ctx->st.probes = nrows;
    return MUMS_OK;
}

}  // extern "C"
