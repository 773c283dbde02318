// shard_comm.hip -- multi-GPU MemHash behind the C ABI.
//
// One context per rank (mums_shard_layout / mums_shard_slice + its genomes), one
// communicator per rank.  mums_shard_run drives the sharded seed stage and FindMatches
// with the rank's collectives issued on the context's stream:
//   1. keys     : mums_shard_keys -> 8-B records bucketed by the top B key bits;
//   2. counts   : all-gather of the per-bucket record counts; the buckets are cut into
//                 world contiguous key ranges of balanced record counts (key_ranges);
//   3. exchange : one all-to-allv moves every key range to its owner rank, sources in
//                 rank order (= global seed-mer index order);
//   4. merge    : mums_shard_merge -> this key range's probes in AddHashEntry order;
//      (4b. a MER_REPEAT_LIMIT restart or start points: streams gathered on rank 0, which
//      plans and returns every rank's live records; mums_shard_restart_*)
//   5. buckets  : all-gather of per-hash-bucket probe counts, bucket ranges per rank;
//   6. rows     : mums_shard_probe_rows + all-to-allv of the probe rows;
//   7. genomes  : all-gather(v) of the 2-bit packed genomes (chain walks read any genome);
//   8. find     : mums_shard_find -> this rank's buckets of the bucket-major MatchList.
// Communicators: RCCL (ncclCommInitRank for one process per GPU, ncclCommInitAll for one
// process driving several GPUs from one thread per device; all-to-allv = grouped
// ncclSend/ncclRecv over xGMI), an in-process host-staged communicator for ranks that
// are threads of one process (tests of the orchestration on a single GPU), or the
// caller's own transport through two host callbacks (mums_comm_init_host: MPI, gloo, ...).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/mums.h"
#include "mums_internal.h"

struct mums_comm {
    int world = 1, rank = 0, device = 0;
    std::string err;
    virtual ~mums_comm() = default;
    // host arrays: recv[world][n] = every rank's send[n]
    virtual int allgather_u64(const uint64_t* send, size_t n, uint64_t* recv, hipStream_t st) = 0;
    // device buffers, byte counts per peer; send / recv blocks in rank order
    virtual int alltoallv(const void* d_send, const uint64_t* send_bytes, void* d_recv, const uint64_t* recv_bytes,
                          hipStream_t st) = 0;
    // device DevBufs for the run (kept across runs)
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
        int ensure(size_t bytes) {
            if (bytes <= cap) return 0;
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            const size_t want = bytes + (bytes >> 4) + 4096;
            if (hipMalloc(&p, want) != hipSuccess) return -1;
            cap = want;
            return 0;
        }
        ~Buf() {
            if (p) (void)hipFree(p);
        }
    } rec, recv, rows, rrows, packed, packed_all, tags, rtags, ents, rents, efk, refk, ascii, thr, rthr;
    uint64_t sent_rows = 0, sent_bytes = 0, recv_rows = 0, recv_bytes = 0;   // last FindMatches exchange
    bool packed_done = false;   // packed_all holds this run's genomes (gather_packed)
};

namespace {

int comm_fail(mums_comm* c, const std::string& m) {
    c->err = m;
    return MUMS_E_HIP;
}

// exclusive prefix sums of per-peer byte counts: the block offsets of an all-to-allv's send
// or receive buffer (blocks in rank order).  Shared by both communicators, so the in-process
// one (tested on one GPU) checks the same arithmetic the RCCL one runs.
std::vector<uint64_t> block_offsets(const uint64_t* bytes, int world) {
    std::vector<uint64_t> off(world + 1, 0);
    for (int r = 0; r < world; ++r) off[r + 1] = off[r] + bytes[r];
    return off;
}

// ---- RCCL ---------------------------------------------------------------------------
struct RcclComm : mums_comm {
    ncclComm_t nc = nullptr;
    Buf scratch;
    ~RcclComm() override {
        if (nc) (void)ncclCommDestroy(nc);
    }
    int allgather_u64(const uint64_t* send, size_t n, uint64_t* recv, hipStream_t st) override {
        if (scratch.ensure((world + 1) * n * 8 + 64)) return comm_fail(this, "allgather buffer");
        uint64_t* d = (uint64_t*)scratch.p;
        // on the collective's stream: a pageable host-to-device hipMemcpy may return before its
        // DMA is done, and the rank's stream is not ordered after the null stream
        if (hipMemcpyAsync(d + (size_t)world * n, send, n * 8, hipMemcpyHostToDevice, st) != hipSuccess)
            return comm_fail(this, "allgather H2D");
        ncclResult_t r = ncclAllGather(d + (size_t)world * n, d, n, ncclUint64, nc, st);
        if (r != ncclSuccess) return comm_fail(this, std::string("ncclAllGather: ") + ncclGetErrorString(r));
        if (hipStreamSynchronize(st) != hipSuccess ||
            hipMemcpy(recv, d, (size_t)world * n * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return comm_fail(this, "allgather D2H");
        if (getenv("MUMS_DEV_COMM_DEBUG")) {
            uint64_t a = 0, b = 0;
            for (size_t i = 0; i < n; ++i) a += send[i] * (i + 1);
            for (size_t i = 0; i < n; ++i) b += recv[(size_t)rank * n + i] * (i + 1);
            fprintf(stderr, "rank %d allgather n %zu send %lu recv-own %lu\n", rank, n, (unsigned long)a,
                    (unsigned long)b);
        }
        return MUMS_OK;
    }
    int alltoallv(const void* d_send, const uint64_t* sb, void* d_recv, const uint64_t* rb, hipStream_t st) override {
        const std::vector<uint64_t> soff = block_offsets(sb, world), roff = block_offsets(rb, world);
        if (sb[rank] != rb[rank]) return comm_fail(this, "alltoallv: self counts differ");
        if (sb[rank] && hipMemcpyAsync((char*)d_recv + roff[rank], (const char*)d_send + soff[rank], sb[rank],
                                       hipMemcpyDeviceToDevice, st) != hipSuccess)
            return comm_fail(this, "alltoallv self copy");
        ncclResult_t r = ncclGroupStart();
        for (int p = 0; p < world && r == ncclSuccess; ++p) {
            if (p == rank) continue;
            if (sb[p]) r = ncclSend((const char*)d_send + soff[p], sb[p], ncclChar, p, nc, st);
            if (r == ncclSuccess && rb[p]) r = ncclRecv((char*)d_recv + roff[p], rb[p], ncclChar, p, nc, st);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess)
            return comm_fail(this, std::string("RCCL all-to-allv: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
        return MUMS_OK;
    }
};

// ---- in-process ranks (threads), host-staged ----------------------------------------
struct LocalShared {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<std::vector<uint64_t>> host;          // per rank
    std::vector<const void*> dsend;
    std::vector<std::vector<uint64_t>> sbytes;
    explicit LocalShared(int w) : world(w), host(w), dsend(w), sbytes(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

struct LocalComm : mums_comm {
    std::shared_ptr<LocalShared> sh;
    int allgather_u64(const uint64_t* send, size_t n, uint64_t* recv, hipStream_t) override {
        sh->host[rank].assign(send, send + n);
        sh->barrier();
        for (int r = 0; r < world; ++r) std::memcpy(recv + (size_t)r * n, sh->host[r].data(), n * 8);
        sh->barrier();
        return MUMS_OK;
    }
    int alltoallv(const void* d_send, const uint64_t* sb, void* d_recv, const uint64_t* rb, hipStream_t st) override {
        if (hipStreamSynchronize(st) != hipSuccess) return comm_fail(this, "stream sync");
        sh->dsend[rank] = d_send;
        sh->sbytes[rank].assign(sb, sb + world);
        sh->barrier();
        const std::vector<uint64_t> roff = block_offsets(rb, world);
        int rc = MUMS_OK;
        for (int s = 0; s < world; ++s) {   // source s's block for this rank
            const uint64_t so = block_offsets(sh->sbytes[s].data(), world)[rank];
            const uint64_t nb = sh->sbytes[s][rank];
            if (nb != rb[s]) rc = comm_fail(this, "alltoallv: counts differ");
            else if (nb && hipMemcpyAsync((char*)d_recv + roff[s], (const char*)sh->dsend[s] + so, nb, hipMemcpyDefault,
                                          st) != hipSuccess)
                rc = comm_fail(this, "alltoallv copy");
        }
        // the copies complete before anything reads them: a device-to-device hipMemcpy may return
        // before its copy is done, and the rank's kernels run on its own (non-blocking) stream
        if (hipStreamSynchronize(st) != hipSuccess) rc = comm_fail(this, "alltoallv copy sync");
        sh->barrier();   // sources stay valid until every rank has copied
        return rc;
    }
};

// ---- the caller's transport (mums_comm_ops), host-staged ------------------------------
// Every collective of mums_shard_run goes through two host callbacks, so a caller whose
// ranks already talk over MPI, gloo or a job launcher's sockets runs the sharded pipeline
// without RCCL (and ranks that are processes sharing one GPU can run it: RCCL refuses two
// ranks on one device).
struct HostComm : mums_comm {
    mums_comm_ops ops{};
    void* user = nullptr;
    std::vector<char> hs, hr;   // host staging of the all-to-allv
    int allgather_u64(const uint64_t* send, size_t n, uint64_t* recv, hipStream_t) override {
        if (ops.allgather_u64(user, send, n, recv) != 0) return comm_fail(this, "host allgather callback failed");
        return MUMS_OK;
    }
    int alltoallv(const void* d_send, const uint64_t* sb, void* d_recv, const uint64_t* rb, hipStream_t st) override {
        const std::vector<uint64_t> soff = block_offsets(sb, world), roff = block_offsets(rb, world);
        if (sb[rank] != rb[rank]) return comm_fail(this, "alltoallv: self counts differ");
        try {
            hs.resize(soff[world] + 1);
            hr.resize(roff[world] + 1);
        } catch (const std::bad_alloc&) {
            return comm_fail(this, "alltoallv: host staging allocation");
        }
        if (hipStreamSynchronize(st) != hipSuccess ||
            (soff[world] && hipMemcpy(hs.data(), d_send, soff[world], hipMemcpyDeviceToHost) != hipSuccess))
            return comm_fail(this, "alltoallv D2H");
        if (ops.alltoallv(user, hs.data(), sb, hr.data(), rb) != 0) return comm_fail(this, "host alltoallv callback failed");
        // on the rank's stream, waited for: the kernels that read d_recv run there
        if (roff[world] && (hipMemcpyAsync(d_recv, hr.data(), roff[world], hipMemcpyHostToDevice, st) != hipSuccess ||
                            hipStreamSynchronize(st) != hipSuccess))
            return comm_fail(this, "alltoallv H2D");
        return MUMS_OK;
    }
};

// key_ranges (libmems_amd/shard.py): boundary r at the first bucket whose prefix sum
// reaches ceil(total * r / world)
void key_ranges(const std::vector<uint64_t>& tot, int world, std::vector<uint32_t>& first,
                std::vector<uint32_t>& count) {
    const uint32_t nb = (uint32_t)tot.size();
    std::vector<uint64_t> cum(nb + 1, 0);
    for (uint32_t b = 0; b < nb; ++b) cum[b + 1] = cum[b] + tot[b];
    const uint64_t total = cum[nb];
    std::vector<uint32_t> bounds{0};
    for (int r = 1; r < world; ++r) {
        const unsigned __int128 t = ((unsigned __int128)total * (unsigned)r + (unsigned)world - 1) / (unsigned)world;
        const uint64_t target = (uint64_t)t;
        const uint32_t b = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        bounds.push_back(std::min(std::max(b, bounds.back()), nb));
    }
    bounds.push_back(nb);
    first.assign(world, 0);
    count.assign(world, 0);
    for (int r = 0; r < world; ++r) {
        first[r] = bounds[r];
        count[r] = bounds[r + 1] - bounds[r];
    }
}

#define RC(x)                        \
    do {                             \
        const int rc_ = (x);         \
        if (rc_ != MUMS_OK) return rc_; \
    } while (0)

// Every rank's status after a local step, before the next collective: a failure on any rank
// (e.g. mums_shard_merge refusing an input on the rank owning that key range) ends every
// rank with the lowest failing rank's code instead of leaving the others blocked in the
// collective.  Ranks that did not fail name the failing rank in mums_comm_last_error.
int agree(mums_comm* c, int rc, hipStream_t st) {
    if (c->world == 1) return rc;
    const uint64_t mine = (uint64_t)(uint32_t)rc;
    std::vector<uint64_t> all(c->world, 0);
    const int r2 = c->allgather_u64(&mine, 1, all.data(), st);
    if (r2 != MUMS_OK) return rc != MUMS_OK ? rc : r2;
    for (int r = 0; r < c->world; ++r) {
        const int code = (int)(int32_t)(uint32_t)all[r];
        if (code == MUMS_OK) continue;
        if (r != c->rank) c->err = "rank " + std::to_string(r) + " failed (status " + std::to_string(code) + ")";
        return code;
    }
    return MUMS_OK;
}

// a local step's status: OK, or the step's code (allocation failures as MUMS_E_NOMEM)
#define AGREE(x) RC(agree(comm, (x), st))

// 7. all-gather(v) of the 2-bit packed genomes into comm->packed_all, genome g at its word
// offset (FindMatches' chain walks, the restart's tie replay read any genome); once per run
int gather_packed(mums_ctx* ctx, mums_comm* comm, hipStream_t st) {
    const int W = comm->world;
    int rc = MUMS_OK;
    uint64_t woff = 0, nw = 0, total = 0;
    rc = mums_shard_packed_info(ctx, &woff, &nw, &total);
    if (rc == MUMS_OK && (comm->packed_all.ensure((total + 1) * 4) || comm->packed.ensure((nw + 1) * 4)))
        rc = MUMS_E_NOMEM;
    if (rc == MUMS_OK && hipMemsetAsync(comm->packed_all.p, 0, (total + 1) * 4, st) != hipSuccess) rc = MUMS_E_HIP;
    if (rc == MUMS_OK)
        rc = mums_shard_packed_copy(ctx, W == 1 ? (uint32_t*)comm->packed_all.p + woff : (uint32_t*)comm->packed.p);
    if (rc == MUMS_OK && W > 1 && comm->rec.ensure((size_t)W * nw * 4 + 8)) rc = MUMS_E_NOMEM;
    AGREE(rc);
    if (W > 1) {   // all-gather(v) of the packed slices as an all-to-allv with one block per peer
        std::vector<uint64_t> meta{woff, nw}, M((size_t)2 * W);
        RC(comm->allgather_u64(meta.data(), 2, M.data(), st));
        // every rank sends its slice to every rank; received blocks land in rank order,
        // which is word-offset order (genome blocks / slices ascend with the rank)
        std::vector<uint64_t> sb(W, nw * 4), rb(W);
        uint64_t o = 0;
        bool ordered = true;
        for (int p = 0; p < W; ++p) {
            rb[p] = M[(size_t)2 * p + 1] * 4;
            ordered = ordered && M[(size_t)2 * p] == o;
            o += M[(size_t)2 * p + 1];
        }
        if (!ordered) return comm_fail(comm, "packed slices are not in rank order");   // the same on every rank
        // the send buffer is the slice repeated per peer (all-to-allv sends disjoint blocks)
        rc = MUMS_OK;
        for (int p = 0; p < W && rc == MUMS_OK; ++p)
            if (nw && hipMemcpyAsync((uint32_t*)comm->rec.p + (size_t)p * nw, comm->packed.p, nw * 4,
                                     hipMemcpyDeviceToDevice, st) != hipSuccess)
                rc = MUMS_E_HIP;
        AGREE(rc);
        RC(comm->alltoallv(comm->rec.p, sb.data(), comm->packed_all.p, rb.data(), st));
    }
    comm->packed_done = true;
    return MUMS_OK;
}

// ParallelMemHash compat over the ranks (compat_ranks.hip): every rank holds
// the whole input (an all-gather of the genomes' ASCII) and searches its contiguous range of
// the chunks with tables of its own (ParallelMemHash.cpp:42-103 on chunks [nch r / W,
// nch (r + 1) / W)); the tables' buckets go to their owners (balanced hash-bucket ranges, as
// in MemHash's sharded find), which re-add the ranks' tables rank after rank (MergeTable,
// :105-121).  The ranks' lists in rank order are the one-thread MatchList (the oracle's rank
// model, tests/test_compat_logs_cpu.py::test_chunk_range_ranks_model).
int compat_shard_run(mums_ctx* ctx, mums_comm* comm, int stage, hipStream_t st) {
    const int W = comm->world, R = comm->rank;
    uint32_t first = 0, nown = 0;
    std::vector<uint64_t> lens;
    AGREE(mums::ctx_compat_layout(ctx, &first, &nown, &lens));
    const int G = (int)lens.size();
    std::vector<uint64_t> gofs((size_t)G + 1, 0);
    for (int g = 0; g < G; ++g) gofs[g + 1] = gofs[g] + lens[g];
    std::vector<const char*> ptrs((size_t)G, nullptr), own(nown, nullptr);
    int rc = MUMS_OK;
    for (uint32_t i = 0; i < nown && rc == MUMS_OK; ++i) {
        const void* p = nullptr;
        uint64_t n = 0;
        rc = mums_genome_device(ctx, i, &p, &n);
        own[i] = (const char*)p;
    }
    AGREE(rc);
    if (W == 1) {
        if (first != 0 || nown != (uint32_t)G) return comm_fail(comm, "one rank must own every genome");
        for (int g = 0; g < G; ++g) ptrs[g] = own[g];
    } else {   // all-gather(v) of the owned genome blocks (blocks ascend with the rank)
        std::vector<uint64_t> meta{first, nown}, MT((size_t)2 * W);
        RC(comm->allgather_u64(meta.data(), 2, MT.data(), st));
        uint64_t next = 0;
        for (int p = 0; p < W; ++p) {
            if (MT[(size_t)2 * p] != next && MT[(size_t)2 * p + 1] != 0)
                return comm_fail(comm, "genome blocks are not in rank order");
            next = std::max<uint64_t>(next, MT[(size_t)2 * p] + MT[(size_t)2 * p + 1]);
        }
        if (next != (uint64_t)G) return comm_fail(comm, "the ranks' genome blocks do not cover the layout");
        const uint64_t mine = gofs[first + nown] - gofs[first];
        rc = (comm->rec.ensure((size_t)W * mine + 64) || comm->ascii.ensure(gofs[G] + 64)) ? MUMS_E_NOMEM : MUMS_OK;
        for (int p = 0; p < W && rc == MUMS_OK; ++p)
            for (uint32_t i = 0; i < nown && rc == MUMS_OK; ++i)
                if (lens[first + i] &&
                    hipMemcpyAsync((char*)comm->rec.p + (size_t)p * mine + (gofs[first + i] - gofs[first]), own[i],
                                   lens[first + i], hipMemcpyDeviceToDevice, st) != hipSuccess)
                    rc = MUMS_E_HIP;
        AGREE(rc);
        std::vector<uint64_t> sb(W, mine), rb(W, 0);
        for (int p = 0; p < W; ++p) {
            const uint64_t f = MT[(size_t)2 * p], n = MT[(size_t)2 * p + 1];
            rb[p] = n ? gofs[f + n] - gofs[f] : 0;
        }
        RC(comm->alltoallv(comm->rec.p, sb.data(), comm->ascii.p, rb.data(), st));
        for (int g = 0; g < G; ++g) ptrs[g] = (const char*)comm->ascii.p + gofs[g];
    }
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK) rc = mums::ctx_compat_rank_find(ctx, ptrs.data(), lens.data(), G, (uint32_t)R, (uint32_t)W, stage);
    AGREE(rc);
    if (stage != MUMS_STAGE_ALL) return MUMS_OK;
    uint32_t T = 0, Gt = 0;
    RC(mums::ctx_table_genomes(ctx, &T, &Gt));
    std::vector<uint64_t> bc(T, 0), BC((size_t)W * T);
    uint64_t M = 0;
    AGREE(mums::ctx_compat_rank_export(ctx, bc.data(), nullptr, &M));
    RC(comm->allgather_u64(bc.data(), T, BC.data(), st));
    std::vector<uint64_t> btot(T, 0);
    for (int r = 0; r < W; ++r)
        for (uint32_t b = 0; b < T; ++b) btot[b] += BC[(size_t)r * T + b];
    std::vector<uint32_t> bf, bn;
    key_ranges(btot, W, bf, bn);
    const uint64_t rowb = 8ull * (G + 2);
    rc = comm->ents.ensure((M + 1) * rowb) ? MUMS_E_NOMEM : MUMS_OK;
    if (rc == MUMS_OK) rc = mums::ctx_compat_rank_export(ctx, bc.data(), (int64_t*)comm->ents.p, &M);
    AGREE(rc);
    const uint32_t nb = bn[R];
    std::vector<uint64_t> cnt((size_t)W * nb), sb(W, 0), rb(W, 0);
    uint64_t nrecv = 0;
    for (int p = 0; p < W; ++p)
        for (uint32_t b = bf[p]; b < bf[p] + bn[p]; ++b) sb[p] += bc[b] * rowb;
    for (int s2 = 0; s2 < W; ++s2)
        for (uint32_t j = 0; j < nb; ++j) {
            cnt[(size_t)s2 * nb + j] = BC[(size_t)s2 * T + bf[R] + j];
            rb[s2] += cnt[(size_t)s2 * nb + j] * rowb;
            nrecv += cnt[(size_t)s2 * nb + j];
        }
    const void* rows = comm->ents.p;
    if (W > 1) {
        AGREE(comm->rents.ensure((nrecv + 1) * rowb) ? MUMS_E_NOMEM : MUMS_OK);
        RC(comm->alltoallv(comm->ents.p, sb.data(), comm->rents.p, rb.data(), st));
        rows = comm->rents.p;
    }
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK) rc = mums::ctx_compat_rank_merge(ctx, (const int64_t*)rows, (uint32_t)W, cnt.data(), nb);
    return agree(comm, rc, st);
}

// 4b (default). The restart planned where the records are (mums_shard_restart_counts ..
// _finish): rank r holds SML indices [off_r[g], off_r[g] + n_r[g]) of every genome, so the
// plan runs on the ranks' own SML parts -- candidate precompute everywhere at once, then the
// plan rank after rank with the running start points (G words per step).  Straddled runs
// get their std::sort order on rank g % world from the all-gathered packed genomes; every
// rank compacts its own live records.  Nothing is gathered: rank 0 holds O(its records).
// *done = false (nothing changed) when any rank's plan needs a key beyond its neighbours.
int shard_restart_local(mums_ctx* ctx, mums_comm* comm, hipStream_t st, bool* done) {
    *done = false;
    const int W = comm->world, R = comm->rank;
    const bool dbg = getenv("MUMS_DEV_SHARD_RESTART_DEBUG") != nullptr;
    uint32_t T = 0, G = 0;
    RC(mums::ctx_table_genomes(ctx, &T, &G));
    const uint64_t Gu = G, row = 3 * Gu + 2;   // mums_shard_restart_counts' info + candidates
    std::vector<uint64_t> info(row, 0), ALL((size_t)W * row), ri(4, 0);
    int rc = mums_shard_restart_counts(ctx, info.data());
    if (rc == MUMS_OK) rc = mums_shard_restart_info(ctx, ri.data());
    info[3 * Gu + 1] = ri[1];
    AGREE(rc);
    RC(comm->allgather_u64(info.data(), row, ALL.data(), st));
    std::vector<uint64_t> flat((size_t)W * (row - 1));   // rows of 3G + 1 for _prepare
    for (int r = 0; r < W; ++r) {
        if (ALL[(size_t)r * row + 3 * Gu]) return MUMS_OK;   // a rank asks for the gathered plan
        std::copy(ALL.begin() + (size_t)r * row, ALL.begin() + (size_t)r * row + row - 1,
                  flat.begin() + (size_t)r * (row - 1));
    }
    if (dbg)
        fprintf(stderr, "rank %d: restart counts ok, candidates %lu\n", R, (unsigned long)info[3 * Gu + 1]);
    std::vector<uint64_t> S(Gu, 0);
    AGREE(mums_shard_restart_prepare(ctx, (uint32_t)W, (uint32_t)R, flat.data(), S.data()));
    // the plan, rank after rank: [status, restarts, undecidable, S]
    std::vector<uint64_t> msg(3 + Gu), M((size_t)W * (3 + Gu)), Rn(W, 0);
    for (int r = 0; r < W; ++r) {
        if (ALL[(size_t)r * row + 3 * Gu + 1] == 0) continue;   // no candidates: S passes through
        std::fill(msg.begin(), msg.end(), 0);
        if (r == R) {
            std::copy(S.begin(), S.end(), msg.begin() + 3);
            uint64_t nr = 0, und = 0;
            const int src = mums_shard_restart_step(ctx, msg.data() + 3, &nr, &und);
            msg[0] = (uint64_t)(uint32_t)src;
            msg[1] = nr;
            msg[2] = und;
        }
        RC(comm->allgather_u64(msg.data(), msg.size(), M.data(), st));
        const uint64_t* m = M.data() + (size_t)r * (3 + Gu);
        const int code = (int)(int32_t)(uint32_t)m[0];
        if (code != MUMS_OK) {
            if (r != R) comm->err = "rank " + std::to_string(r) + " failed (status " + std::to_string(code) + ")";
            return code;
        }
        if (dbg) fprintf(stderr, "rank %d: plan step of rank %d: %lu restarts, undecidable %lu\n", R, r,
                         (unsigned long)m[1], (unsigned long)m[2]);
        if (m[2]) {   // undecidable on rank r: the gathered plan (nothing changed yet)
            if (mums::ctx_tie_all(ctx)) {   // (which does not order every run of equal keys)
                comm->err = "sharded repeat tolerance: a restart plan needs keys beyond a rank's neighbours";
                return MUMS_E_UNSUPPORTED;
            }
            return MUMS_OK;
        }
        Rn[r] = m[1];
        std::copy(m + 3, m + 3 + Gu, S.begin());
    }
    // every rank's restarts in rank order (= key order)
    uint64_t Rt = 0, Rmax = 0;
    for (int r = 0; r < W; ++r) {
        Rt += Rn[r];
        Rmax = std::max(Rmax, Rn[r]);
    }
    std::vector<uint64_t> rkey(Rt), rS(Rt * Gu);
    if (Rt) {
        const uint64_t blk = Rmax * (1 + Gu);
        std::vector<uint64_t> mine(blk, 0), L((size_t)W * blk);
        rc = Rn[R] ? mums_shard_restart_log(ctx, mine.data(), mine.data() + Rmax) : MUMS_OK;
        AGREE(rc);
        RC(comm->allgather_u64(mine.data(), blk, L.data(), st));
        uint64_t o = 0;
        for (int r = 0; r < W; ++r) {
            const uint64_t* b = L.data() + (size_t)r * blk;
            for (uint64_t k = 0; k < Rn[r]; ++k, ++o) {
                rkey[o] = b[k];
                std::copy(b + Rmax + k * Gu, b + Rmax + (k + 1) * Gu, rS.begin() + o * Gu);
            }
        }
    }
    // repeat tolerance: every run of equal keys in std::sort order.  Pair flags go to rank
    // g % W (blocks in rank order = SML order), which replays genome g's sort and returns each
    // rank the ids of its slots in the same layout.
    const bool rtol = mums::ctx_tie_all(ctx);   // repeat tolerance or enumeration tolerance > 1
    if (rtol) {
        auto part = [&](int r, uint32_t g) { return ALL[(size_t)r * row + g]; };
        std::vector<uint64_t> gofs(Gu, 0), sb(W, 0), rb(W, 0);
        uint64_t o = 0;
        for (int p = 0; p < W; ++p)   // send: destination-major, genomes ascending
            for (uint32_t g = (uint32_t)p; g < G; g += (uint32_t)W) {
                gofs[g] = o;
                o += part(R, g);
                sb[p] += 4 * part(R, g);
            }
        const uint64_t nloc = o;
        std::vector<std::vector<uint64_t>> foff(G, std::vector<uint64_t>(W, 0)), lens(G, std::vector<uint64_t>(W, 0));
        uint64_t ro = 0;
        for (int r = 0; r < W; ++r)   // receive: source-major, this rank's genomes ascending
            for (uint32_t g = (uint32_t)R; g < G; g += (uint32_t)W) {
                foff[g][r] = ro;
                lens[g][r] = part(r, g);
                ro += part(r, g);
                rb[r] += 4 * part(r, g);
            }
        AGREE(comm->rows.ensure(nloc * 4 + 8) || comm->rrows.ensure(ro * 4 + 8) || comm->recv.ensure(ro * 4 + 8)
                  ? MUMS_E_NOMEM : MUMS_OK);
        AGREE(mums_shard_tie_flags(ctx, gofs.data(), (uint32_t*)comm->rows.p));
        RC(comm->alltoallv(comm->rows.p, sb.data(), comm->rrows.p, rb.data(), st));
        RC(gather_packed(ctx, comm, st));
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        for (uint32_t g = (uint32_t)R; g < G && rc == MUMS_OK; g += (uint32_t)W)
            rc = mums_shard_tie_replay(ctx, (const uint32_t*)comm->packed_all.p, g, (uint32_t)W,
                                       (const uint32_t*)comm->rrows.p, foff[g].data(), lens[g].data(),
                                       (uint32_t*)comm->recv.p, foff[g].data());
        AGREE(rc);
        RC(comm->alltoallv(comm->recv.p, rb.data(), comm->rows.p, sb.data(), st));
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        if (rc == MUMS_OK) rc = mums_shard_tie_apply(ctx, (const uint32_t*)comm->rows.p, gofs.data());
        AGREE(rc);
        if (dbg) fprintf(stderr, "rank %d: every run of equal keys in std::sort order\n", R);
    }
    // the runs of equal keys the start points of every phase fall into, on their owner ranks
    // (all of them are in order already under repeat tolerance)
    const uint64_t cap = 3 * (Rt + 1) * Gu;
    std::vector<uint64_t> runs(cap + 3, 0);
    uint64_t nr = 0;
    if (!rtol) AGREE(mums_shard_restart_runs(ctx, Rt, rkey.data(), rS.data(), runs.data(), cap, &nr));
    std::vector<uint64_t> NR(W);
    RC(comm->allgather_u64(&nr, 1, NR.data(), st));
    if (dbg) {
        fprintf(stderr, "rank %d: %lu restarts in all, %lu straddled runs here:", R, (unsigned long)Rt, (unsigned long)nr);
        for (uint64_t q = 0; q < nr && q < 8; ++q)
            fprintf(stderr, " {%lu %lu %lu}", (unsigned long)runs[3 * q], (unsigned long)runs[3 * q + 1],
                    (unsigned long)runs[3 * q + 2]);
        fprintf(stderr, "\n");
    }
    uint64_t NRmax = 0, NRt = 0;
    for (int r = 0; r < W; ++r) {
        NRmax = std::max(NRmax, NR[r]);
        NRt += NR[r];
    }
    std::vector<uint64_t> vofs(nr, 0);
    if (NRt) {
        std::vector<uint64_t> AR((size_t)W * 3 * NRmax);
        runs.resize(std::max<uint64_t>(3 * NRmax, 3));
        RC(comm->allgather_u64(runs.data(), 3 * NRmax, AR.data(), st));
        RC(gather_packed(ctx, comm, st));
        // rank g % W replays genome g; its send block for rank p: p's runs of those genomes
        std::vector<uint64_t> sb(W, 0), rb(W, 0), des, dofs;
        uint64_t so = 0;
        for (int p = 0; p < W; ++p)
            for (uint64_t q = 0; q < NR[p]; ++q) {
                const uint64_t* x = AR.data() + (size_t)p * 3 * NRmax + 3 * q;
                if ((int)(x[0] % (uint64_t)W) != R) continue;
                des.insert(des.end(), x, x + 3);
                dofs.push_back(so);
                so += x[2] - x[1];
                sb[p] += 4 * (x[2] - x[1]);
            }
        uint64_t ro = 0;
        for (int d = 0; d < W; ++d)
            for (uint64_t q = 0; q < nr; ++q) {
                const uint64_t* x = runs.data() + 3 * q;
                if ((int)(x[0] % (uint64_t)W) != d) continue;
                vofs[q] = ro;
                ro += x[2] - x[1];
                rb[d] += 4 * (x[2] - x[1]);
            }
        AGREE(comm->rows.ensure(so * 4 + 8) || comm->rrows.ensure(ro * 4 + 8) ? MUMS_E_NOMEM : MUMS_OK);
        AGREE(mums_shard_restart_ties(ctx, (const uint32_t*)comm->packed_all.p, des.data(), dofs.size(), dofs.data(),
                                      (uint32_t*)comm->rows.p));
        RC(comm->alltoallv(comm->rows.p, sb.data(), comm->rrows.p, rb.data(), st));
    }
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK)
        rc = mums_shard_restart_finish(ctx, Rt, rkey.data(), rS.data(), runs.data(), nr,
                                       nr ? (const uint32_t*)comm->rrows.p : nullptr, vofs.data());
    *done = true;
    if (dbg) fprintf(stderr, "rank %d: restart finish rc %d (%s)\n", R, rc, rc ? mums_last_error(ctx) : "");
    return agree(comm, rc, st);
}

// 4b. MER_REPEAT_LIMIT restarts / start points (MatchFinder.cpp:253-277, MemHash.cpp:117-127):
// a restart moves the start points of every later key (records of other ranks) and its plan
// reads whole SortedMerLists, so the merged streams are gathered in rank order (= key order)
// onto rank 0, which plans, fixes the std::sort tie order of the runs the start points fall
// into and compacts every rank's live records; the blocks go back in one all-to-allv and
// every rank runs its groups stage again.  C: the keys stage's per-rank bucket counts.
int shard_restart(mums_ctx* ctx, mums_comm* comm, const std::vector<uint64_t>& C, const std::vector<uint32_t>& kf,
                  const std::vector<uint32_t>& kn, uint32_t nb, hipStream_t st) {
    const int W = comm->world, R = comm->rank;
    const void* d_stream = nullptr;
    uint64_t n = 0;
    AGREE(mums_shard_stream(ctx, &d_stream, &n));
    std::vector<uint64_t> NN(W);
    RC(comm->allgather_u64(&n, 1, NN.data(), st));
    uint64_t N = 0;
    for (int r = 0; r < W; ++r) N += NN[r];
    std::vector<uint64_t> sb(W, 0), rb(W, 0);
    sb[0] = n * 8;
    if (R == 0)
        for (int r = 0; r < W; ++r) rb[r] = NN[r] * 8;
    const uint64_t out_cap = 8 * (N + (uint64_t)W * (nb + 4));
    AGREE(R == 0 && (comm->recv.ensure(N * 8 + 8) || comm->rows.ensure(out_cap)) ? MUMS_E_NOMEM : MUMS_OK);
    RC(comm->alltoallv(d_stream, sb.data(), comm->recv.p, rb.data(), st));
    std::vector<uint64_t> bb(W, 0);
    int rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK && R == 0)
        rc = mums_shard_restart_plan(ctx, (uint64_t*)comm->recv.p, (uint32_t)W, C.data(), kf.data(), kn.data(),
                                     comm->rows.p, out_cap, bb.data());
    uint64_t rows = 0;
    uint32_t G = 0;
    if (rc == MUMS_OK) rc = mums_get_offset_log(ctx, nullptr, 0, &rows, &G);
    AGREE(rc);
    // rank 0's restart count and block sizes, then its offset log
    std::vector<uint64_t> meta(1 + W, 0), M((size_t)W * (1 + W));
    if (R == 0) {
        meta[0] = rows;
        for (int r = 0; r < W; ++r) meta[1 + r] = bb[r];
    }
    RC(comm->allgather_u64(meta.data(), meta.size(), M.data(), st));
    const uint64_t nres = M[0];
    std::vector<uint64_t> log(nres * G, 0);
    if (nres * G) {
        std::vector<uint64_t> mine(nres * G, 0), L((size_t)W * nres * G);
        if (R == 0) rc = mums_get_offset_log(ctx, mine.data(), nres, &rows, &G);
        AGREE(rc);
        RC(comm->allgather_u64(mine.data(), mine.size(), L.data(), st));
        std::copy(L.begin(), L.begin() + nres * G, log.begin());
    }
    std::fill(sb.begin(), sb.end(), 0);
    std::fill(rb.begin(), rb.end(), 0);
    if (R == 0)
        for (int r = 0; r < W; ++r) sb[r] = M[1 + r];
    rb[0] = M[1 + R];
    AGREE(comm->rrows.ensure(rb[0] + 8) ? MUMS_E_NOMEM : MUMS_OK);
    RC(comm->alltoallv(comm->rows.p, sb.data(), comm->rrows.p, rb.data(), st));
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK) rc = mums_shard_restart_apply(ctx, comm->rrows.p, nres, log.data());
    return agree(comm, rc, st);
}

}  // namespace

extern "C" {

int mums_comm_unique_id(void* id, uint64_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return MUMS_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return MUMS_E_HIP;
    std::memcpy(id, &u, sizeof(u));
    return MUMS_OK;
}

int mums_comm_init_rank(mums_comm** out, int device, int world, int rank, const void* id) {
    if (!out || !id || world < 1 || rank < 0 || rank >= world) return MUMS_E_INVALID;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return MUMS_E_NODEVICE;
    auto* c = new RcclComm();
    c->world = world;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->nc, world, u, rank) != ncclSuccess) {
        delete c;
        return MUMS_E_HIP;
    }
    *out = c;
    return MUMS_OK;
}

int mums_comm_init_all(mums_comm** out, int ndev, const int* devices) {
    if (!out || ndev < 1 || !devices) return MUMS_E_INVALID;
    std::vector<ncclComm_t> nc(ndev);
    if (ncclCommInitAll(nc.data(), ndev, devices) != ncclSuccess) return MUMS_E_HIP;
    for (int r = 0; r < ndev; ++r) {
        auto* c = new RcclComm();
        c->world = ndev;
        c->rank = r;
        c->device = devices[r];
        c->nc = nc[r];
        out[r] = c;
    }
    return MUMS_OK;
}

int mums_comm_init_local(mums_comm** out, int nranks, const int* devices) {
    if (!out || nranks < 1 || !devices) return MUMS_E_INVALID;
    auto sh = std::make_shared<LocalShared>(nranks);
    for (int r = 0; r < nranks; ++r) {
        auto* c = new LocalComm();
        c->world = nranks;
        c->rank = r;
        c->device = devices[r];
        c->sh = sh;
        out[r] = c;
    }
    return MUMS_OK;
}

int mums_comm_init_host(mums_comm** out, int device, int world, int rank, const mums_comm_ops* ops, void* user) {
    if (!out || !ops || !ops->allgather_u64 || !ops->alltoallv || world < 1 || rank < 0 || rank >= world)
        return MUMS_E_INVALID;
    auto* c = new HostComm();
    c->world = world;
    c->rank = rank;
    c->device = device;
    c->ops = *ops;
    c->user = user;
    *out = c;
    return MUMS_OK;
}

void mums_comm_destroy(mums_comm* c) { delete c; }

const char* mums_comm_last_error(mums_comm* c) { return c ? c->err.c_str() : "null communicator"; }

int mums_comm_exchange_info(mums_comm* c, uint64_t* info) {
    if (!c || !info) return MUMS_E_INVALID;
    info[0] = c->sent_rows;
    info[1] = c->sent_bytes;
    info[2] = c->recv_rows;
    info[3] = c->recv_bytes;
    return MUMS_OK;
}

int mums_shard_key_ranges(const uint64_t* totals, uint32_t nbuckets, uint32_t world, uint32_t* first,
                          uint32_t* count) {
    if (!totals || !first || !count || world < 1) return MUMS_E_INVALID;
    std::vector<uint32_t> f, n;
    key_ranges(std::vector<uint64_t>(totals, totals + nbuckets), (int)world, f, n);
    std::copy(f.begin(), f.end(), first);
    std::copy(n.begin(), n.end(), count);
    return MUMS_OK;
}

int mums_shard_run(mums_ctx* ctx, mums_comm* comm, int stage) {
    if (!ctx || !comm) return MUMS_E_INVALID;
    const int W = comm->world, R = comm->rank;
    hipStream_t st = mums::ctx_stream(ctx);
    int rc = hipSetDevice(mums::ctx_device(ctx)) != hipSuccess ? MUMS_E_NODEVICE : MUMS_OK;
    comm->packed_done = false;
    if (mums::ctx_pcompat(ctx)) {
        AGREE(rc);
        return compat_shard_run(ctx, comm, stage, st);
    }
    // 1-4: sharded seed stage.  Every local step's status is agreed on before the next
    // collective (agree), so one rank's failure never leaves the others waiting in it.
    uint32_t B = 0;
    uint64_t n_local = 0;
    if (rc == MUMS_OK) rc = mums_shard_msd_bits(ctx, &B, &n_local);
    const uint32_t nb = 1u << B;
    std::vector<uint64_t> counts(nb, 0), C;
    if (rc == MUMS_OK && comm->rec.ensure((n_local + 1) * 8)) rc = MUMS_E_NOMEM;
    if (rc == MUMS_OK) rc = mums_shard_keys(ctx, (uint64_t*)comm->rec.p, n_local + 1, counts.data());
    AGREE(rc);
    C.assign((size_t)W * nb, 0);
    RC(comm->allgather_u64(counts.data(), nb, C.data(), st));
    std::vector<uint64_t> tot(nb, 0);
    for (int r = 0; r < W; ++r)
        for (uint32_t b = 0; b < nb; ++b) tot[b] += C[(size_t)r * nb + b];
    std::vector<uint32_t> kf, kn;
    key_ranges(tot, W, kf, kn);
    const uint32_t first = kf[R], cnt = kn[R];
    std::vector<uint64_t> sub((size_t)W * cnt);
    for (int r = 0; r < W; ++r)
        for (uint32_t b = 0; b < cnt; ++b) sub[(size_t)r * cnt + b] = C[(size_t)r * nb + first + b];
    const uint64_t* merged = (const uint64_t*)comm->rec.p;
    if (W > 1) {
        std::vector<uint64_t> sb(W, 0), rb(W, 0);
        for (int p = 0; p < W; ++p)
            for (uint32_t b = kf[p]; b < kf[p] + kn[p]; ++b) sb[p] += 8 * C[(size_t)R * nb + b];
        for (int s = 0; s < W; ++s)
            for (uint32_t b = 0; b < cnt; ++b) rb[s] += 8 * sub[(size_t)s * cnt + b];
        uint64_t rtot = 0;
        for (int s = 0; s < W; ++s) rtot += rb[s];
        AGREE(comm->recv.ensure(rtot + 8) ? MUMS_E_NOMEM : MUMS_OK);
        RC(comm->alltoallv(comm->rec.p, sb.data(), comm->recv.p, rb.data(), st));
        merged = (const uint64_t*)comm->recv.p;
    }
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK) rc = mums_shard_merge(ctx, merged, (uint32_t)W, first, cnt, sub.data());
    AGREE(rc);
    {   // 4b: restarts, when any rank's key range holds a group above MER_REPEAT_LIMIT
        uint64_t pend = 0;
        AGREE(mums_shard_restart_pending(ctx, &pend));
        std::vector<uint64_t> PEND(W);
        RC(comm->allgather_u64(&pend, 1, PEND.data(), st));
        bool any = false;
        for (int r = 0; r < W; ++r) any = any || PEND[r] != 0;
        if (any) {
            bool done = false;
            RC(shard_restart_local(ctx, comm, st, &done));
            if (!done) {   // the gathered plan reads one merged stream per rank
                int rcg = MUMS_OK;
                if (mums::ctx_merge_chunked(ctx)) {
                    comm->err = "sharded restart after a key-chunked merge: a restart plan needs keys beyond a "
                                "rank's neighbours (the gathered plan needs one-pass merges)";
                    rcg = MUMS_E_UNSUPPORTED;
                }
                AGREE(rcg);
                RC(shard_restart(ctx, comm, C, kf, kn, nb, st));
            }
        }
    }
    if (stage != MUMS_STAGE_ALL) return MUMS_OK;
    // 5-8: sharded FindMatches
    uint32_t T = 0, G = 0;
    RC(mums::ctx_table_genomes(ctx, &T, &G));
    std::vector<uint64_t> bc(T, 0), BC((size_t)W * T);
    AGREE(mums_shard_bucket_counts(ctx, bc.data()));
    RC(comm->allgather_u64(bc.data(), T, BC.data(), st));
    std::vector<uint64_t> btot(T, 0);
    for (int r = 0; r < W; ++r)
        for (uint32_t b = 0; b < T; ++b) btot[b] += BC[(size_t)r * T + b];
    std::vector<uint32_t> bf, bn;
    key_ranges(btot, W, bf, bn);
    std::vector<uint32_t> bounds(bf.begin(), bf.end());
    bounds.push_back(T);
    uint64_t P = 0;
    const uint64_t rowb = 8ull * (G + 1);
    // default: chains labelled on the probes' own rank (key ranges balance the line sort and
    // the walks); MUMS_DEV_SHARD_BUCKET_CHAINS: labelled by the bucket owner (rows only)
    const bool labelled = getenv("MUMS_DEV_SHARD_BUCKET_CHAINS") == nullptr;
    // default: only the probes the owners' replay needs travel;
    // MUMS_DEV_SHARD_ALL_ROWS: every probe row (the round-5 layout)
    const bool kept = labelled && getenv("MUMS_DEV_SHARD_ALL_ROWS") == nullptr;
    comm->sent_rows = comm->sent_bytes = comm->recv_rows = comm->recv_bytes = 0;
    if (kept) {
        if (!comm->packed_done) RC(gather_packed(ctx, comm, st));
        uint64_t nch = 0;
        rc = mums_shard_chain_label(ctx, (const uint32_t*)comm->packed_all.p, &nch);
        if (rc == MUMS_OK) rc = mums_probe_count(ctx, &P);
        const uint64_t entb = 8ull * (G + 2);
        if (rc == MUMS_OK && (comm->ents.ensure((nch + 1) * entb) || comm->efk.ensure((nch + 1) * 4) ||
                              comm->thr.ensure((nch + 1) * 8)))
            rc = MUMS_E_NOMEM;
        // 7a. every chain entry to the owner of its bucket
        std::vector<uint64_t> ce(W, 0), CE((size_t)W * W);
        if (rc == MUMS_OK) rc = mums_shard_chain_entries(ctx, (uint32_t)W, bounds.data(), (int64_t*)comm->ents.p, nch + 1,
                                                         ce.data());
        AGREE(rc);
        RC(comm->allgather_u64(ce.data(), W, CE.data(), st));
        std::vector<uint64_t> src_ents(W);
        uint64_t nents = 0;
        for (int s2 = 0; s2 < W; ++s2) {
            src_ents[s2] = CE[(size_t)s2 * W + R];
            nents += src_ents[s2];
        }
        std::vector<uint64_t> sb(W), rb(W);
        const void* rents = comm->ents.p;
        void* rthr = comm->thr.p;
        if (W > 1) {
            AGREE(comm->rents.ensure((nents + 1) * entb) || comm->rthr.ensure((nents + 1) * 8) ? MUMS_E_NOMEM : MUMS_OK);
            for (int q = 0; q < W; ++q) {
                sb[q] = ce[q] * entb;
                rb[q] = src_ents[q] * entb;
            }
            RC(comm->alltoallv(comm->ents.p, sb.data(), comm->rents.p, rb.data(), st));
            rents = comm->rents.p;
            rthr = comm->rthr.p;
        }
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        // 7b. the owners' answers {next_s, first} back to the entries' sources
        if (rc == MUMS_OK) rc = mums_shard_entry_thresholds(ctx, (const int64_t*)rents, nents, (uint32_t*)rthr);
        AGREE(rc);
        if (W > 1) {
            for (int q = 0; q < W; ++q) {
                sb[q] = src_ents[q] * 8;
                rb[q] = ce[q] * 8;
            }
            RC(comm->alltoallv(comm->rthr.p, sb.data(), comm->thr.p, rb.data(), st));
        }
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        // 7c. the kept rows, their tags and each entry's first sent row
        if (rc == MUMS_OK && (comm->rows.ensure((P + 1) * rowb) || comm->tags.ensure((P + 1) * 4))) rc = MUMS_E_NOMEM;
        std::vector<uint64_t> cnt(2 * (size_t)W, 0), CNT((size_t)W * 2 * W);
        if (rc == MUMS_OK)
            rc = mums_shard_kept_export(ctx, (uint32_t)W, (const uint32_t*)comm->thr.p, (int64_t*)comm->rows.p,
                                        (uint32_t*)comm->tags.p, P + 1, (uint32_t*)comm->efk.p, cnt.data(),
                                        cnt.data() + W);
        AGREE(rc);
        RC(comm->allgather_u64(cnt.data(), 2 * (size_t)W, CNT.data(), st));
        std::vector<uint64_t> src_rows(W);
        uint64_t nrows = 0, dropped = 0;
        for (int s2 = 0; s2 < W; ++s2) {
            src_rows[s2] = CNT[(size_t)s2 * 2 * W + R];
            dropped += CNT[(size_t)s2 * 2 * W + W + R];
            nrows += src_rows[s2];
        }
        for (int q = 0; q < W; ++q) comm->sent_rows += cnt[q];
        comm->recv_rows = nrows;
        comm->sent_bytes = comm->sent_rows * (rowb + 4);
        comm->recv_bytes = nrows * (rowb + 4);
        for (int q = 0; q < W; ++q) comm->sent_bytes += ce[q] * (entb + 8 + 4);
        comm->recv_bytes += nents * (entb + 8 + 4);
        const void *rrows = comm->rows.p, *rtags = comm->tags.p, *refk = comm->efk.p;
        if (W > 1) {
            AGREE(comm->rrows.ensure((nrows + 1) * rowb) || comm->rtags.ensure((nrows + 1) * 4) ||
                          comm->refk.ensure((nents + 1) * 4)
                      ? MUMS_E_NOMEM
                      : MUMS_OK);
            auto xchg = [&](const uint64_t* sendn, const uint64_t* recvn, uint64_t unit, const void* sendp,
                            void* recvp) -> int {
                for (int q = 0; q < W; ++q) {
                    sb[q] = sendn[q] * unit;
                    rb[q] = recvn[q] * unit;
                }
                return comm->alltoallv(sendp, sb.data(), recvp, rb.data(), st);
            };
            RC(xchg(cnt.data(), src_rows.data(), rowb, comm->rows.p, comm->rrows.p));
            RC(xchg(cnt.data(), src_rows.data(), 4, comm->tags.p, comm->rtags.p));
            RC(xchg(ce.data(), src_ents.data(), 4, comm->efk.p, comm->refk.p));
            rrows = comm->rrows.p;
            rtags = comm->rtags.p;
            refk = comm->refk.p;
        }
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        if (rc == MUMS_OK)
            rc = mums_shard_find_kept(ctx, (const int64_t*)rrows, (const uint32_t*)rtags, nrows, (const int64_t*)rents,
                                      (const uint32_t*)refk, nents, (uint32_t)W, src_rows.data(), src_ents.data(),
                                      dropped, (const uint32_t*)comm->packed_all.p);
        return agree(comm, rc, st);
    }
    if (labelled) {
        if (!comm->packed_done) RC(gather_packed(ctx, comm, st));
        uint64_t nch = 0;
        rc = mums_shard_chain_label(ctx, (const uint32_t*)comm->packed_all.p, &nch);
        if (rc == MUMS_OK) rc = mums_probe_count(ctx, &P);
        const uint64_t entb = 8ull * (G + 2);
        if (rc == MUMS_OK && (comm->rows.ensure((P + 1) * rowb) || comm->tags.ensure((P + 1) * 4) ||
                              comm->ents.ensure((nch + 1) * entb) || comm->efk.ensure((nch + 1) * 4)))
            rc = MUMS_E_NOMEM;
        std::vector<uint64_t> cnt(2 * (size_t)W, 0), CNT((size_t)W * 2 * W);
        if (rc == MUMS_OK)
            rc = mums_shard_chain_export(ctx, (uint32_t)W, bounds.data(), (int64_t*)comm->rows.p, (uint32_t*)comm->tags.p,
                                         P + 1, (int64_t*)comm->ents.p, (uint32_t*)comm->efk.p, nch + 1, cnt.data(),
                                         cnt.data() + W);
        AGREE(rc);
        RC(comm->allgather_u64(cnt.data(), 2 * (size_t)W, CNT.data(), st));
        // rank s sends CNT[s][R] rows and CNT[s][W + R] entries here
        std::vector<uint64_t> src_rows(W), src_ents(W);
        uint64_t nrows = 0, nents = 0;
        for (int s2 = 0; s2 < W; ++s2) {
            src_rows[s2] = CNT[(size_t)s2 * 2 * W + R];
            src_ents[s2] = CNT[(size_t)s2 * 2 * W + W + R];
            nrows += src_rows[s2];
            nents += src_ents[s2];
        }
        for (int q = 0; q < W; ++q) comm->sent_rows += cnt[q];
        comm->recv_rows = nrows;
        comm->sent_bytes = comm->sent_rows * (rowb + 4);
        comm->recv_bytes = nrows * (rowb + 4) + nents * (entb + 4);
        for (int q = 0; q < W; ++q) comm->sent_bytes += cnt[(size_t)W + q] * (entb + 4);
        const void *rrows = comm->rows.p, *rtags = comm->tags.p, *rents = comm->ents.p, *refk = comm->efk.p;
        if (W > 1) {
            AGREE(comm->rrows.ensure((nrows + 1) * rowb) || comm->rtags.ensure((nrows + 1) * 4) ||
                          comm->rents.ensure((nents + 1) * entb) || comm->refk.ensure((nents + 1) * 4)
                      ? MUMS_E_NOMEM
                      : MUMS_OK);
            std::vector<uint64_t> sb(W), rb(W);
            auto xchg = [&](uint64_t unit, int which, const void* sendp, void* recvp) -> int {
                for (int p = 0; p < W; ++p) {
                    sb[p] = cnt[(size_t)which * W + p] * unit;
                    rb[p] = (which ? src_ents[p] : src_rows[p]) * unit;
                }
                return comm->alltoallv(sendp, sb.data(), recvp, rb.data(), st);
            };
            RC(xchg(rowb, 0, comm->rows.p, comm->rrows.p));
            RC(xchg(4, 0, comm->tags.p, comm->rtags.p));
            RC(xchg(entb, 1, comm->ents.p, comm->rents.p));
            RC(xchg(4, 1, comm->efk.p, comm->refk.p));
            rrows = comm->rrows.p;
            rtags = comm->rtags.p;
            rents = comm->rents.p;
            refk = comm->refk.p;
        }
        rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
        if (rc == MUMS_OK)
            rc = mums_shard_find_labelled(ctx, (const int64_t*)rrows, (const uint32_t*)rtags, nrows,
                                          (const int64_t*)rents, (const uint32_t*)refk, nents, (uint32_t)W,
                                          src_rows.data(), src_ents.data(), (const uint32_t*)comm->packed_all.p);
        return agree(comm, rc, st);
    }
    std::vector<uint64_t> send(W, 0), S((size_t)W * W);
    rc = mums_probe_count(ctx, &P);
    if (rc == MUMS_OK && comm->rows.ensure((P + 1) * rowb)) rc = MUMS_E_NOMEM;
    if (rc == MUMS_OK)
        rc = mums_shard_probe_rows(ctx, (uint32_t)W, bounds.data(), (int64_t*)comm->rows.p, P + 1, send.data());
    AGREE(rc);
    RC(comm->allgather_u64(send.data(), W, S.data(), st));
    const int64_t* rows = (const int64_t*)comm->rows.p;
    uint64_t nrows = P;
    if (W > 1) {
        std::vector<uint64_t> sb(W), rb(W);
        nrows = 0;
        for (int p = 0; p < W; ++p) {
            sb[p] = send[p] * rowb;
            rb[p] = S[(size_t)p * W + R] * rowb;
            nrows += S[(size_t)p * W + R];
        }
        AGREE(comm->rrows.ensure((nrows + 1) * rowb) ? MUMS_E_NOMEM : MUMS_OK);
        RC(comm->alltoallv(comm->rows.p, sb.data(), comm->rrows.p, rb.data(), st));
        rows = (const int64_t*)comm->rrows.p;
    }
    if (!comm->packed_done) RC(gather_packed(ctx, comm, st));
    rc = hipStreamSynchronize(st) != hipSuccess ? MUMS_E_HIP : MUMS_OK;
    if (rc == MUMS_OK) rc = mums_shard_find(ctx, rows, nrows, (const uint32_t*)comm->packed_all.p);
    return agree(comm, rc, st);
}

}  // extern "C"
