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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mums.h"
#include "mums_internal.h"
#include "seed_device.h"

using namespace mums;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        size_t want = bytes + (bytes >> 4) + 4096;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        else p = nullptr;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T> T* as() const { return (T*)p; }
};

struct GenomeIn {
    const char* d_ptr;
    uint64_t n;
    bool owned;
};

enum { EV_START, EV_KEYS, EV_SORT, EV_GROUPS, EV_BUCKETS, EV_REPLAY, EV_OUTPUT, EV_COUNT };

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
    bool use_onesweep = true;
    hipEvent_t ev[EV_COUNT] = {};
    bool profiling = false;
    hipEvent_t ev_ds[16] = {};   // 2 per radix pass (<= 8 passes)

    // state of the last run
    int stage_done = 0;
    bool key64 = false;
    bool packed_path = false;
    int msd_bits = 0;
    int L = 0, w = 0;
    uint64_t pattern = 0, N = 0, P = 0, M = 0;
    int sorted_buf = 0;
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
    uint32_t* counts = ctx->partials.as<uint32_t>();          // [ntiles] probes, then [ntiles] groups
    uint32_t* gcounts = counts + ntiles + 32;
    uint32_t* offs = gcounts + ntiles + 32;
    DevCounters* dc = ctx->counters.as<DevCounters>();
    HIPCHK((launch_probe_tiles<MG, View>(v, tiles, ntiles, ctx->N, ctx->gt, mp, ctx->L, counts, slot_info, slot_bucket,
                                         dc, st)));
    HIPCHK(exclusive_scan_u32(gcounts, ntiles, ctx->tmp.p, &dc->ngroups, st));
    HIPCHK(hipMemcpyAsync(offs, counts, ntiles * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(exclusive_scan_u32(offs, ntiles, ctx->tmp.p, &dc->nprobes, st));
    HIPCHK(launch_probe_compact(ntiles, counts, offs, slot_info, slot_bucket, probe_info, probe_bucket, st));
    return MUMS_OK;
}

template <typename View>
int groups_dispatch(mums_ctx* ctx, View v, const SegTile* tiles, uint64_t ntiles, const MatchParams& mp,
                    uint64_t* pi, uint32_t* pb, uint64_t* si, uint32_t* sb, hipStream_t st) {
    const int G = (int)ctx->genomes.size();
    if (G <= 4) return run_groups<4, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    if (G <= 8) return run_groups<8, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    if (G <= 16) return run_groups<16, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
    return run_groups<32, View>(ctx, v, tiles, ntiles, mp, pi, pb, si, sb, st);
}

template <typename View>
int replay_dispatch(mums_ctx* ctx, View v, const MatchParams& mp, hipStream_t st) {
    const int G = (int)ctx->genomes.size();
#define MUMS_REPLAY_CALL(MG)                                                                                        \
    HIPCHK((launch_replay<MG, View>(v, ctx->N, ctx->gt, mp, ctx->ss, ctx->probe_info, ctx->sorted_ids,              \
                                    ctx->bstart.as<uint32_t>(), ctx->bend.as<uint32_t>(), ctx->tbl.as<uint32_t>(),  \
                                    ctx->pool.as<int64_t>(), ctx->packed.as<uint32_t>(), ctx->tsize.as<uint32_t>(), \
                                    ctx->counters.p, st)))
    if (G <= 4) MUMS_REPLAY_CALL(4);
    else if (G <= 8) MUMS_REPLAY_CALL(8);
    else if (G <= 16) MUMS_REPLAY_CALL(16);
    else MUMS_REPLAY_CALL(32);
#undef MUMS_REPLAY_CALL
    return MUMS_OK;
}

// keys -> sorted stream -> probes -> bucket-sorted probes [-> replay -> MatchList]
int run_pipeline(mums_ctx* ctx, int stage) {
    hipStream_t st = ctx->stream;
    const int G = (int)ctx->genomes.size();
    const uint64_t N = ctx->N;
    MatchParams mp{ctx->repeat_tol, ctx->enum_tol, ctx->table_size, ctx->masked, ctx->seq_mask};
    GenomeTable& gt = ctx->gt;

    // packed genomes + key-kernel tiles
    uint64_t words = 0;
    uint32_t T = 0;
    for (int g = 0; g < G; ++g) {
        gt.woff[g] = words;
        words += (packed_words(gt.n[g]) + 3) & ~3ull;
        gt.tfirst[g] = T;
        T += (uint32_t)((gt.n[g] + kSeedTile - 1) / kSeedTile);
    }
    gt.woff[G] = words;
    for (int g = G; g <= kMaxG; ++g) gt.tfirst[g] = T;
    HIPCHK(ctx->packed.ensure(words * 4 + 64));
    HIPCHK(ctx->counters.ensure(sizeof(DevCounters)));
    DevCounters* dc = ctx->counters.as<DevCounters>();
    std::vector<const char*> ptrs(G);
    for (int g = 0; g < G; ++g) ptrs[g] = ctx->genomes[g].d_ptr;
    const SeedSpec& ss = ctx->ss;

    const int kbits = 2 * ctx->w + 1;
    ctx->packed_path = kbits <= 32 + kMaxMsdBits;
    ctx->msd_bits = ctx->packed_path ? std::max(0, kbits - 32) : 0;
    if (const char* e = getenv("MUMS_DEV_MSD_BITS"))   // development knob (sort layout experiments)
        if (ctx->packed_path) ctx->msd_bits = std::min(kMaxMsdBits, std::max(ctx->msd_bits, atoi(e)));
    const int B = ctx->msd_bits;
    const int passes = ctx->packed_path ? (kbits - B + 7) / 8 : (kbits + 7) / 8;
    const size_t kb = ctx->key64 ? 8 : 4;
    const uint64_t ntiles_groups = ctx->packed_path ? seg_tiles_upper(N, B) : (N + kSegTile - 1) / kSegTile;
    const uint64_t pcap = N / 2 + 1;
    const uint64_t nslots = group_slot_count(ntiles_groups);

    // workspace (grow-only; no allocation in steady state)
    size_t tmpb = std::max(scan_tmp_bytes(N), radix_tmp_bytes(pcap));
    tmpb = std::max(tmpb, scan_tmp_bytes((uint64_t)ctx->table_size));
    if (ctx->packed_path) {
        HIPCHK(ctx->recA.ensure(N * 8 + 64));
        HIPCHK(ctx->recB.ensure(N * 8 + 64));
        HIPCHK(ctx->tiles.ensure(ntiles_groups * sizeof(SegTile) + 64));
        if (B > 0) HIPCHK(ctx->hist.ensure(((uint64_t)T << B) * 4 + 64));
        tmpb = std::max(tmpb, seg_tmp_bytes(N, B));
        tmpb = std::max(tmpb, onesweep_tmp_bytes(N, B, kbits - B));
        HIPCHK(ctx->mstart.ensure(((1ull << B) + 64) * 4));
        tmpb = std::max(tmpb, scan_tmp_bytes((uint64_t)T << B));
    } else {
        HIPCHK(ctx->ckey.ensure(N * kb + 64));
        HIPCHK(ctx->kA.ensure(N * kb + 64));
        HIPCHK(ctx->kB.ensure(N * kb + 64));
        HIPCHK(ctx->vA.ensure(N * 4 + 64));
        HIPCHK(ctx->vB.ensure(N * 4 + 64));
        HIPCHK(ctx->tiles.ensure(ntiles_groups * sizeof(SegTile) + 64));
        tmpb = std::max(tmpb, radix_tmp_bytes(N));
    }
    HIPCHK(ctx->tmp.ensure(tmpb));
    HIPCHK(ctx->partials.ensure((3 * ntiles_groups + 128) * 4));
    HIPCHK(ctx->pbuf.ensure(pcap * (8 + 4 * 4) + nslots * 12 + 256));
    char* pb = (char*)ctx->pbuf.p;
    uint64_t* probe_info = (uint64_t*)pb;
    uint64_t* slot_info = probe_info + pcap;
    uint32_t* probe_bucket = (uint32_t*)(slot_info + nslots);
    uint32_t* bucketB = probe_bucket + pcap;
    uint32_t* idsA = bucketB + pcap;
    uint32_t* idsB = idsA + pcap;
    uint32_t* slot_bucket = idsB + pcap;

    HIPCHK(hipEventRecord(ctx->ev[EV_START], st));
    HIPCHK(hipMemsetAsync(dc, 0, sizeof(DevCounters), st));
    const bool prof = ctx->profiling;
    if (prof && !ctx->ev_ds[0])
        for (int i = 0; i < 16; ++i) HIPCHK(hipEventCreate(&ctx->ev_ds[i]));

    int rc = MUMS_OK;
    if (ctx->packed_path) {
        SegTile* tiles = ctx->tiles.as<SegTile>();
        uint32_t* hist = ctx->hist.as<uint32_t>();
        HIPCHK(launch_seed_pack(ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 1, true, nullptr, B, hist, T,
                                &dc->err, st));
        if (B > 0) HIPCHK(exclusive_scan_u32(hist, (uint64_t)T << B, ctx->tmp.p, nullptr, st));
        HIPCHK(launch_seed_scatter(ss, gt, ctx->packed.as<uint32_t>(), B, hist, T, ctx->recA.as<uint64_t>(), st));
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        HIPCHK(build_seg_tiles(B > 0 ? hist : nullptr, T, B, N, tiles, &dc->ntiles, ctx->mstart.as<uint32_t>(),
                               ctx->tmp.p, st));
        int buf = 0;
        if (ctx->use_onesweep && N < (1ull << 30) && kbits - B <= 32)
            HIPCHK(seg_onesweep_sort(ctx->recA.as<uint64_t>(), ctx->recB.as<uint64_t>(), N, kbits - B, B, tiles,
                                     ntiles_groups, ctx->mstart.as<uint32_t>(), ctx->tmp.p, &dc->err, &buf, st,
                                     prof ? ctx->ev_ds : nullptr));
        else
            HIPCHK(seg_radix_sort(ctx->recA.as<uint64_t>(), ctx->recB.as<uint64_t>(), N, kbits - B, tiles,
                                  ntiles_groups, ctx->tmp.p, &buf, st, prof ? ctx->ev_ds : nullptr));
        ctx->sorted_buf = buf;
        ctx->sorted_rec = buf ? ctx->recB.as<uint64_t>() : ctx->recA.as<uint64_t>();
        HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
        rc = groups_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, tiles, ntiles_groups, mp, probe_info,
                                      probe_bucket, slot_info, slot_bucket, st);
    } else {
        HIPCHK(launch_seed_pack(ss, gt, ptrs.data(), ctx->packed.as<uint32_t>(), 0, ctx->key64, ctx->ckey.p, 0,
                                nullptr, T, &dc->err, st));
        HIPCHK(hipEventRecord(ctx->ev[EV_KEYS], st));
        int buf = 0;
        SegTile* tiles = ctx->tiles.as<SegTile>();
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
        HIPCHK(hipEventRecord(ctx->ev[EV_SORT], st));
        if (ctx->key64)
            rc = groups_dispatch<PairView<uint64_t>>(ctx, PairView<uint64_t>{(const uint64_t*)ctx->sorted_key,
                                                                             ctx->sorted_idx},
                                                     tiles, ntiles_groups, mp, probe_info, probe_bucket, slot_info,
                                                     slot_bucket, st);
        else
            rc = groups_dispatch<PairView<uint32_t>>(ctx, PairView<uint32_t>{(const uint32_t*)ctx->sorted_key,
                                                                             ctx->sorted_idx},
                                                     tiles, ntiles_groups, mp, probe_info, probe_bucket, slot_info,
                                                     slot_bucket, st);
    }
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->hc.err & 1u) return fail(ctx, MUMS_E_GAP, "Gap in genome sequence ('-' encountered)");
    if (ctx->hc.err & 2u) return fail(ctx, MUMS_E_HIP, "sort look-back timed out (internal error)");
    ctx->P = ctx->hc.nprobes;
    ctx->probe_info = probe_info;
    HIPCHK(hipEventRecord(ctx->ev[EV_GROUPS], st));

    // probes grouped by hash bucket, key order kept (stable); values = probe ids
    int tbits = 1;
    while (tbits < 32 && ((uint64_t)1 << tbits) < (uint64_t)ctx->table_size) ++tbits;
    int pout = 0;
    HIPCHK(radix_sort<uint32_t>(probe_bucket, nullptr, ctx->P, tbits, bucketB, idsA, probe_bucket, idsB, ctx->tmp.p,
                                &pout, st));
    ctx->sorted_buckets = pout ? probe_bucket : bucketB;
    ctx->sorted_ids = pout ? idsB : idsA;
    HIPCHK(hipEventRecord(ctx->ev[EV_BUCKETS], st));
    ctx->stage_done = MUMS_STAGE_SEEDS;

    if (stage >= MUMS_STAGE_ALL) {
        const uint32_t Tb = ctx->table_size;
        HIPCHK(ctx->bstart.ensure((size_t)Tb * 4));
        HIPCHK(ctx->bend.ensure((size_t)Tb * 4));
        HIPCHK(ctx->tsize.ensure((size_t)Tb * 4));
        HIPCHK(ctx->obase.ensure((size_t)Tb * 4 + 64));
        HIPCHK(ctx->pool.ensure((ctx->P + 1) * (size_t)(G + 2) * 8));
        HIPCHK(ctx->tbl.ensure((ctx->P + 1) * 4));
        HIPCHK(hipMemsetAsync(ctx->bstart.p, 0, (size_t)Tb * 4, st));
        HIPCHK(hipMemsetAsync(ctx->bend.p, 0, (size_t)Tb * 4, st));
        HIPCHK(hipMemsetAsync(ctx->tsize.p, 0, (size_t)Tb * 4, st));
        HIPCHK(launch_bucket_ranges(ctx->sorted_buckets, ctx->P, ctx->bstart.as<uint32_t>(), ctx->bend.as<uint32_t>(),
                                    st));
        if (ctx->P > 0) {
            if (ctx->packed_path) rc = replay_dispatch<RecView>(ctx, RecView{ctx->sorted_rec}, mp, st);
            else if (ctx->key64)
                rc = replay_dispatch<PairView<uint64_t>>(
                    ctx, PairView<uint64_t>{(const uint64_t*)ctx->sorted_key, ctx->sorted_idx}, mp, st);
            else
                rc = replay_dispatch<PairView<uint32_t>>(
                    ctx, PairView<uint32_t>{(const uint32_t*)ctx->sorted_key, ctx->sorted_idx}, mp, st);
            if (rc) return rc;
        }
        HIPCHK(hipEventRecord(ctx->ev[EV_REPLAY], st));
        HIPCHK(hipMemcpyAsync(ctx->obase.p, ctx->tsize.p, (size_t)Tb * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(exclusive_scan_u32(ctx->obase.as<uint32_t>(), Tb, ctx->tmp.p, &dc->nmatches, st));
        HIPCHK(hipMemcpyAsync(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        ctx->M = ctx->hc.nmatches;
        HIPCHK(ctx->out_len.ensure((ctx->M + 1) * 8));
        HIPCHK(ctx->out_s.ensure((ctx->M + 1) * (size_t)G * 8));
        HIPCHK(launch_emit(ctx->tsize.as<uint32_t>(), ctx->obase.as<uint32_t>(), ctx->bstart.as<uint32_t>(),
                           ctx->tbl.as<uint32_t>(), ctx->pool.as<int64_t>(), G, Tb, ctx->out_len.as<uint64_t>(),
                           ctx->out_s.as<int64_t>(), st));
        HIPCHK(hipEventRecord(ctx->ev[EV_OUTPUT], st));
        ctx->stage_done = MUMS_STAGE_ALL;
    }
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&ctx->hc, dc, sizeof(DevCounters), hipMemcpyDeviceToHost));

    // stats
    mums_stats& s = ctx->st;
    s = mums_stats{};
    s.seedmers = N;
    s.groups = ctx->hc.ngroups;
    s.probes = ctx->P;
    s.repeat_limit_groups = ctx->hc.repeat_limit;
    auto el = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
        return (double)ms;
    };
    s.ms_keys = el(EV_START, EV_KEYS);
    s.ms_sort = el(EV_KEYS, EV_SORT);
    s.ms_groups = el(EV_SORT, EV_GROUPS);
    s.ms_buckets = el(EV_GROUPS, EV_BUCKETS);
    s.key_bytes = ctx->packed_path ? 8 : kb;
    s.sort_passes = (uint64_t)passes;
    if (prof && N > 0) {
        for (int p = 0; p < passes; ++p) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ctx->ev_ds[2 * p], ctx->ev_ds[2 * p + 1]);
            s.ms_dominant += ms;
            // algorithmic bytes of one downsweep launch: packed records read + written
            // (8 + 8); pairs: read K (+4 after pass 0) and write K + 4
            s.dominant_bytes += ctx->packed_path ? N * 16 : N * (kb + (p ? 4 : 0) + kb + 4);
        }
        s.dominant_launches = (uint64_t)passes;
    }
    if (ctx->stage_done >= MUMS_STAGE_ALL) {
        s.mem_count = ctx->hc.entries;
        s.collision_count = ctx->hc.collisions;
        s.ms_replay = el(EV_BUCKETS, EV_REPLAY);
        s.ms_output = el(EV_REPLAY, EV_OUTPUT);
        s.ms_total = el(EV_START, EV_OUTPUT);
    } else {
        s.ms_total = el(EV_START, EV_BUCKETS);
    }
    return MUMS_OK;
}

int check_ctx(mums_ctx* ctx) {
    if (!ctx) return MUMS_E_INVALID;
    ctx->err.clear();
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
                      &ctx->pbuf, &ctx->keybuf, &ctx->mstart};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i < EV_COUNT; ++i)
        if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
    for (int i = 0; i < 16; ++i)
        if (ctx->ev_ds[i]) (void)hipEventDestroy(ctx->ev_ds[i]);
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
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 32 genomes per context");
    HIPCHK(hipSetDevice(ctx->device));
    char* d = nullptr;
    HIPCHK(hipMalloc(&d, n + 16));
    if (n) HIPCHK(hipMemcpy(d, ascii, n, hipMemcpyHostToDevice));
    ctx->genomes.push_back({d, n, true});
    ctx->stage_done = 0;
    return MUMS_OK;
}

int mums_add_genome_device(mums_ctx* ctx, const void* d_ascii, uint64_t n) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (!d_ascii && n) return fail(ctx, MUMS_E_INVALID, "Null gnSequence pointer");
    if (ctx->genomes.size() >= (size_t)kMaxG)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 32 genomes per context");
    ctx->genomes.push_back({(const char*)d_ascii, n, false});
    ctx->stage_done = 0;
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
    HIPCHK(hipSetDevice(ctx->device));
    ctx->stage_done = 0;
    ctx->M = ctx->P = 0;
    const int G = (int)ctx->genomes.size();
    if (ctx->enum_tol > 1)
        return fail(ctx, MUMS_E_UNSUPPORTED, "enumeration tolerance > 1 (MatchFinder::EnumerateMatches) not implemented");
    // seed (MatchList.h:351-357 default, SortedMerList::Create checks :788-798)
    uint64_t total = 0;
    for (auto& g : ctx->genomes) total += g.n;
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
        gt.n[g] = ctx->genomes[g].n;
        gt.m[g] = gt.n[g] < (uint64_t)L ? 0 : gt.n[g] - L + 1;
        gt.base[g] = N;
        N += gt.m[g];
    }
    gt.base[G] = N;
    for (int g = G + 1; g <= kMaxG; ++g) gt.base[g] = N;
    if (N >= 0xFFFFFFF0ull)
        return fail(ctx, MUMS_E_UNSUPPORTED, "more than 2^32 seed-mers per context (chunked mode not implemented)");
    ctx->N = N;
    if (G == 0) {
        ctx->stage_done = MUMS_STAGE_ALL;
        ctx->st = mums_stats{};
        return MUMS_OK;
    }
    ctx->ss = make_seed_spec(pat, L, w);
    int rc = run_pipeline(ctx, stage);
    return rc;
}

int mums_find(mums_ctx* ctx) { return mums_find_stage(ctx, MUMS_STAGE_ALL); }

int mums_result_count(mums_ctx* ctx, uint64_t* count, uint32_t* seq_count) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (count) *count = ctx->M;
    if (seq_count) *seq_count = (uint32_t)ctx->genomes.size();
    return MUMS_OK;
}

int mums_result_copy(mums_ctx* ctx, uint64_t* lengths, int64_t* starts) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_ALL) return fail(ctx, MUMS_E_INVALID, "no completed FindMatches on this context");
    if (ctx->M == 0) return MUMS_OK;
    HIPCHK(hipSetDevice(ctx->device));
    const size_t G = ctx->genomes.size();
    if (lengths) HIPCHK(hipMemcpy(lengths, ctx->out_len.p, ctx->M * 8, hipMemcpyDeviceToHost));
    if (starts) HIPCHK(hipMemcpy(starts, ctx->out_s.p, ctx->M * G * 8, hipMemcpyDeviceToHost));
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

int mums_build_sml(mums_ctx* ctx, uint32_t genome, uint32_t* positions, uint64_t cap) {
    if (check_ctx(ctx)) return MUMS_E_INVALID;
    if (ctx->stage_done < MUMS_STAGE_SEEDS) return fail(ctx, MUMS_E_INVALID, "keys not sorted yet");
    if (genome >= ctx->genomes.size()) return fail(ctx, MUMS_E_INVALID, "genome index out of range");
    const uint64_t m = ctx->gt.m[genome];
    if (cap < m) return fail(ctx, MUMS_E_INVALID, "output buffer too small");
    HIPCHK(hipSetDevice(ctx->device));
    // the merged sorted stream restricted to one genome is that genome's SML
    const uint64_t N = ctx->N;
    std::vector<uint32_t> idx(N);
    if (ctx->packed_path) {
        std::vector<uint64_t> rec(N);
        if (N) HIPCHK(hipMemcpy(rec.data(), ctx->sorted_rec, N * 8, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < N; ++i) idx[i] = (uint32_t)rec[i];
    } else if (N) {
        HIPCHK(hipMemcpy(idx.data(), ctx->sorted_idx, N * 4, hipMemcpyDeviceToHost));
    }
    const uint64_t lo = ctx->gt.base[genome], hi = ctx->gt.base[genome + 1];
    uint64_t o = 0;
    for (uint64_t i = 0; i < N; ++i)
        if (idx[i] >= lo && idx[i] < hi) positions[o++] = (uint32_t)(idx[i] - lo);
    return MUMS_OK;
}

}  // extern "C"
