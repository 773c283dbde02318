// restart.hip -- MatchFinder::SearchRange's MER_REPEAT_LIMIT restart (MatchFinder.cpp:253-277)
// and FindMatchesFromPosition start points (MemHash.cpp:117-127) on the merged stream.
//
// The seed stage merges all genomes with one sort, so the reference's restart (drop a
// masked-key group once more than 1000 of its records are collected and another head
// still carries the key; restart from GetBreakpoint positions, MatchFinder.cpp:89-126)
// becomes a fix-up of the sorted stream, run only when the groups stage saw a group
// above MER_REPEAT_LIMIT (or start points were set):
//   1. per-genome SortedMerLists from the stream: full ckey + genome of every record,
//      a stable counting sort by genome (the stream's order inside a genome is its SML
//      order), ck[] genome-major and every record's SML index inv[];
//   2. candidate keys: masked keys with more than 1000 records (sorted on the host);
//   3. restart_plan.h (shared with the CPU model test): cand_precompute per candidate in
//      parallel, then the sequential plan in one lane -> restart keys + start points of
//      every phase;
//   4. a record lives iff its SML index >= the start point of its key's phase; the live
//      records are compacted (order kept) and the groups stage runs again on them.
#include <algorithm>
#include <vector>

#include "mums_internal.h"
#include "seed_device.h"

namespace mums {

namespace {

using restart::PlanData;
using restart::PlanOut;

__device__ __forceinline__ void rs_record(const RsStream& s, uint64_t j, uint64_t* ck, uint64_t* gi) {
    if (s.kind == 0) {
        const uint64_t r = s.rec[j];
        uint32_t b = 0;
        if (s.B > 0) {   // bucket of j: last start <= j
            uint32_t lo = 0, hi = 1u << s.B;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((uint64_t)s.bstart[mid] <= j) lo = mid;
                else hi = mid;
            }
            b = lo;
        }
        const int kb = s.kbits - s.B;
        const uint64_t low = (r >> 32) & ((kb >= 64) ? ~0ull : ((1ull << kb) - 1));
        *ck = ((uint64_t)b << kb) | low;
        *gi = r & 0xFFFFFFFFull;
    } else if (s.kind == 1) {
        *ck = ((const uint32_t*)s.key)[j];
        *gi = s.idx[j];
    } else {
        *ck = ((const uint64_t*)s.key)[j];
        *gi = s.idx[j];
    }
}

__global__ void rs_extract_kernel(RsStream s, uint64_t n, GenomeTable gt, uint64_t* __restrict__ ckf,
                                  uint32_t* __restrict__ gen) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint64_t ck, gi;
    rs_record(s, j, &ck, &gi);
    ckf[j] = ck;
    gen[j] = (uint32_t)genome_of(gt, gi);
}

// perm = stream indices in genome-major order -> ck (genome-major keys), inv (SML slot)
__global__ void rs_gather_kernel(const uint32_t* __restrict__ perm, uint64_t n, const uint64_t* __restrict__ ckf,
                                 uint64_t* __restrict__ ck, uint32_t* __restrict__ inv) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t j = perm[k];
    ck[k] = ckf[j];
    inv[j] = (uint32_t)k;
}

// masked keys with more than MER_REPEAT_LIMIT records (group heads whose run reaches +1000)
__global__ void rs_cand_kernel(const uint64_t* __restrict__ ckf, uint64_t n, uint64_t* __restrict__ list,
                               unsigned long long* __restrict__ cnt, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t v = ckf[j] >> 1;
    if (j > 0 && (ckf[j - 1] >> 1) == v) return;
    const uint64_t e = j + restart::kRepeatLimit;
    if (e >= n || (ckf[e] >> 1) != v) return;
    const unsigned long long k = atomicAdd(cnt, 1ull);
    if (k < cap) list[k] = v;
}

__global__ void rs_pre_kernel(PlanData d, const uint64_t* __restrict__ cand, uint64_t C, uint64_t* __restrict__ clo,
                              uint64_t* __restrict__ chi, uint64_t* __restrict__ cbp, int* __restrict__ cseq,
                              unsigned* __restrict__ cbad) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t G = (uint64_t)d.G;
    if (cbad) {   // distributed: flags per candidate (restart_plan reads them when one fires)
        cbad[c] = 0u;
        d.bad = cbad + c;
    }
    restart::cand_precompute(d, cand[c], clo + c * G, chi + c * G, cbp + c * G, cseq + c);
}

// the plan is sequential over the candidates (each restart moves the start points the
// next one sees): one lane
__global__ void rs_plan_kernel(PlanData d, const uint64_t* __restrict__ cand, uint64_t C,
                               const uint64_t* __restrict__ clo, const uint64_t* __restrict__ chi,
                               const uint64_t* __restrict__ cbp, const int* __restrict__ cseq, uint64_t* S,
                               PlanOut* out, const unsigned* __restrict__ cbad) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    PlanOut o = *out;
    restart::restart_plan(d, cand, C, clo, chi, cbp, cseq, S, &o, cbad);
    *out = o;
}

// live[j] = SML index of record j >= start point of its key's phase (phase p holds the
// keys from restart key p-1 on; phase 0 = the FindMatchSeeds start offsets S0)
__global__ void rs_live_kernel(const uint64_t* __restrict__ ckf, const uint32_t* __restrict__ gen,
                               const uint32_t* __restrict__ inv, uint64_t n, const uint64_t* __restrict__ dbase,
                               const uint64_t* __restrict__ rkey, uint64_t R, const uint64_t* __restrict__ rS,
                               const uint64_t* __restrict__ S0, int G, uint32_t* __restrict__ live) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    if (j == n) { live[n] = 0; return; }
    const uint64_t v = ckf[j] >> 1;
    uint64_t lo = 0, hi = R;   // phase = number of restart keys <= v
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (rkey[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t g = gen[j];
    const uint64_t idx = (uint64_t)inv[j] - dbase[g];
    const uint64_t s = lo == 0 ? S0[g] : rS[(lo - 1) * (uint64_t)G + g];
    live[j] = idx >= s ? 1u : 0u;
}

template <typename T>
__global__ void rs_compact_kernel(const T* __restrict__ src, const uint32_t* __restrict__ live,
                                  const uint32_t* __restrict__ pos, uint64_t n, T* __restrict__ dst) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || !live[j]) return;
    dst[pos[j]] = src[j];
}

__global__ void rs_bstart_kernel(const uint32_t* __restrict__ bstart, uint32_t nb, const uint32_t* __restrict__ pos,
                                 uint32_t* __restrict__ out) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    out[b] = pos[bstart[b]];
}

inline dim3 grid_of(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

inline char* align_up(char* p) { return (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255); }

}  // namespace

RestartWs restart_ws_layout(void* base, uint64_t n, int G) {
    RestartWs w{};
    char* p = align_up((char*)base);
    auto take = [&](size_t bytes) {
        char* r = p;
        p = align_up(p + bytes);
        return (void*)r;
    };
    const uint64_t n1 = n + 64;
    w.ckf = (uint64_t*)take(n1 * 8);
    w.ck = (uint64_t*)take(n1 * 8);
    w.gen = (uint32_t*)take(n1 * 4);
    w.inv = (uint32_t*)take(n1 * 4);
    w.kA = (uint32_t*)take(n1 * 4);
    w.kB = (uint32_t*)take(n1 * 4);
    w.vA = (uint32_t*)take(n1 * 4);
    w.vB = (uint32_t*)take(n1 * 4);
    w.dm = (uint64_t*)take((size_t)(G + 1) * 8);
    w.dbase = (uint64_t*)take((size_t)(G + 1) * 8);
    w.tmp = take(std::max(radix_tmp_bytes(n + 1), scan_tmp_bytes(n + 1)));
    w.bytes = (size_t)(p - (char*)base);
    return w;
}

size_t restart_ws_bytes(uint64_t n, int G) { return restart_ws_layout(nullptr, n, G).bytes + 256; }

hipError_t launch_restart_smls(const RsStream& s, uint64_t n, const GenomeTable& gt, const RestartWs& w,
                               hipStream_t st) {
    if (n == 0) return hipSuccess;
    std::vector<uint64_t> hm(gt.G + 1, 0), hb(gt.G + 1, 0);
    for (int g = 0; g < gt.G; ++g) {
        hm[g] = gt.m[g];
        hb[g] = gt.base[g];
    }
    hipError_t e = hipMemcpyAsync(w.dm, hm.data(), hm.size() * 8, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(w.dbase, hb.data(), hb.size() * 8, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs_extract_kernel, grid_of(n), dim3(kBlock), 0, st, s, n, gt, w.ckf, w.gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    int gbits = 1;
    while ((1 << gbits) < gt.G) ++gbits;
    int buf = 0;
    e = radix_sort<uint32_t>(w.gen, nullptr, n, gbits, w.kA, w.vA, w.kB, w.vB, w.tmp, &buf, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs_gather_kernel, grid_of(n), dim3(kBlock), 0, st, buf ? w.vB : w.vA, n, w.ckf, w.ck, w.inv);
    return hipGetLastError();
}

hipError_t launch_restart_cands(const RestartWs& w, uint64_t n, uint64_t* d_list, unsigned long long* d_cnt,
                                uint64_t cap, hipStream_t st) {
    hipError_t e = hipMemsetAsync(d_cnt, 0, 8, st);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(rs_cand_kernel, grid_of(n), dim3(kBlock), 0, st, w.ckf, n, d_list, d_cnt, cap);
    return hipGetLastError();
}

hipError_t launch_restart_plan(const RestartWs& w, int G, const uint64_t* d_cand, uint64_t C, uint64_t* d_pre,
                               uint64_t* d_S, PlanOut* d_out, hipStream_t st) {
    if (C == 0) return hipSuccess;
    const PlanData d{G, w.dm, w.dbase, w.ck};
    uint64_t* clo = d_pre;
    uint64_t* chi = clo + C * (uint64_t)G;
    uint64_t* cbp = chi + C * (uint64_t)G;
    int* cseq = (int*)(cbp + C * (uint64_t)G);
    hipLaunchKernelGGL(rs_pre_kernel, grid_of(C), dim3(kBlock), 0, st, d, d_cand, C, clo, chi, cbp, cseq, nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs_plan_kernel, dim3(1), dim3(64), 0, st, d, d_cand, C, clo, chi, cbp, cseq, d_S, d_out,
                       nullptr);
    return hipGetLastError();
}

// the sharded mode's plan (restart_plan.h PlanData with off / n / prv / nxt): candidate
// precompute on every rank at once, then the plan one rank after the other (running S)
hipError_t launch_restart_dpre(const PlanData& d, const uint64_t* d_cand, uint64_t C, uint64_t* d_pre, unsigned* cbad,
                               hipStream_t st) {
    if (C == 0) return hipSuccess;
    uint64_t* clo = d_pre;
    uint64_t* chi = clo + C * (uint64_t)d.G;
    uint64_t* cbp = chi + C * (uint64_t)d.G;
    int* cseq = (int*)(cbp + C * (uint64_t)d.G);
    hipLaunchKernelGGL(rs_pre_kernel, grid_of(C), dim3(kBlock), 0, st, d, d_cand, C, clo, chi, cbp, cseq, cbad);
    return hipGetLastError();
}

hipError_t launch_restart_dplan(const PlanData& d, const uint64_t* d_cand, uint64_t C, const uint64_t* d_pre,
                                const unsigned* cbad, uint64_t* d_S, PlanOut* d_out, hipStream_t st) {
    if (C == 0) return hipSuccess;
    const uint64_t* clo = d_pre;
    const uint64_t* chi = clo + C * (uint64_t)d.G;
    const uint64_t* cbp = chi + C * (uint64_t)d.G;
    const int* cseq = (const int*)(cbp + C * (uint64_t)d.G);
    hipLaunchKernelGGL(rs_plan_kernel, dim3(1), dim3(64), 0, st, d, d_cand, C, clo, chi, cbp, cseq, d_S, d_out, cbad);
    return hipGetLastError();
}

// LogProgress tie groups: the head order (restart_plan.h head_order) of the genomes U of a
// group at masked key K in the SearchRange call whose start points are S (phase p)
__global__ void tie_heads_kernel(PlanData d, const uint64_t* __restrict__ gk, const uint64_t* __restrict__ gu,
                                 const uint32_t* __restrict__ gp, const uint64_t* __restrict__ Sall, uint64_t ng,
                                 int* __restrict__ ord) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ng) return;
    const int G = d.G;
    const uint64_t* S = Sall + (uint64_t)gp[i] * G;
    uint64_t a[restart::kMaxGenomes];
    for (int g = 0; g < G; ++g) {
        a[g] = 0;
        if ((gu[i] >> g) & 1) {
            const uint64_t lb = restart::lower_bound_g(d, g, 0, d.m[g], gk[i] << 1);
            a[g] = lb > S[g] ? lb : S[g];
        }
    }
    uint64_t steps = 0;
    int* o = ord + i * (uint64_t)G;
    const int n = restart::head_order(d, gu[i], a, S, o, &steps);
    for (int k = n; k < G; ++k) o[k] = -1;
}

hipError_t launch_tie_heads(const RestartWs& w, int G, const uint64_t* gk, const uint64_t* gu, const uint32_t* gp,
                            const uint64_t* Sall, uint64_t ng, int* ord, hipStream_t st) {
    if (ng == 0) return hipSuccess;
    const PlanData d{G, w.dm, w.dbase, w.ck};
    hipLaunchKernelGGL(tie_heads_kernel, grid_of(ng), dim3(kBlock), 0, st, d, gk, gu, gp, Sall, ng, ord);
    return hipGetLastError();
}

hipError_t launch_restart_compact(const RsStream& s, uint64_t n, int G, const RestartWs& w, const uint64_t* d_rkey,
                                  uint64_t R, const uint64_t* d_rS, const uint64_t* d_S0, void* dst_a, uint32_t* dst_idx,
                                  uint32_t* dst_bstart, uint32_t* d_total, hipStream_t st) {
    uint32_t* live = w.kA;
    uint32_t* pos = w.kB;
    hipLaunchKernelGGL(rs_live_kernel, grid_of(n + 1), dim3(kBlock), 0, st, w.ckf, w.gen, w.inv, n, w.dbase, d_rkey, R,
                       d_rS, d_S0, G, live);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(pos, live, (n + 1) * 4, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    e = exclusive_scan_u32(pos, n + 1, w.tmp, d_total, st);
    if (e != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    if (s.kind == 0) {
        hipLaunchKernelGGL(rs_compact_kernel<uint64_t>, grid_of(n), dim3(kBlock), 0, st, s.rec, live, pos, n,
                           (uint64_t*)dst_a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        const uint32_t nb = 1u << s.B;
        hipLaunchKernelGGL(rs_bstart_kernel, grid_of(nb + 1), dim3(kBlock), 0, st, s.bstart, nb, pos, dst_bstart);
        return hipGetLastError();
    }
    if (s.kind == 1)
        hipLaunchKernelGGL(rs_compact_kernel<uint32_t>, grid_of(n), dim3(kBlock), 0, st, (const uint32_t*)s.key, live,
                           pos, n, (uint32_t*)dst_a);
    else
        hipLaunchKernelGGL(rs_compact_kernel<uint64_t>, grid_of(n), dim3(kBlock), 0, st, (const uint64_t*)s.key, live,
                           pos, n, (uint64_t*)dst_a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(rs_compact_kernel<uint32_t>, grid_of(n), dim3(kBlock), 0, st, s.idx, live, pos, n, dst_idx);
    return hipGetLastError();
}

hipError_t launch_map_starts(const uint32_t* bstart, uint32_t nb, const uint32_t* pos, uint32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(rs_bstart_kernel, grid_of(nb + 1), dim3(kBlock), 0, st, bstart, nb, pos, out);
    return hipGetLastError();
}

}  // namespace mums
