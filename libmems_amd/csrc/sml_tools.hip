// sml_tools.hip -- the data formats on either side of the seed finder:
//   * one genome's SortedMerList (MemorySML::Create, MemorySML.cpp:45-60) on its own;
//   * SeedOccurrenceList::construct (SeedOccurrenceList.h:22-61) + smoothFrequencies
//     (:71-87): per-position seed frequency from the masked-key runs of that SML;
//   * MatchList::MultiplicityFilter / LengthFilter (MatchList.h:636-664) on the result;
//   * 2-bit words -> ASCII for sequences read from DNAFileSML files (FileSML::LoadFile).
#include <hip/hip_runtime.h>

#include "mums_internal.h"

namespace mums {
namespace {

__device__ __forceinline__ bool run_head(const uint64_t* __restrict__ sk, uint64_t i) {
    return i == 0 || (sk[i] >> 1) != (sk[i - 1] >> 1);   // masked key = ckey without parity
}

__global__ void occ_heads_kernel(const uint64_t* __restrict__ sk, uint64_t m, uint32_t* __restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) flag[i] = run_head(sk, i) ? 1u : 0u;
}

// ex = exclusive scan of the head flags: a head's run id is ex[i]
__global__ void occ_runstart_kernel(const uint64_t* __restrict__ sk, uint64_t m, const uint32_t* __restrict__ ex,
                                    uint32_t* __restrict__ rstart) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && run_head(sk, i)) rstart[ex[i]] = (uint32_t)i;
}

// count[position] = length of the masked-key run holding it (SeedOccurrenceList.h:37-50)
__global__ void occ_count_kernel(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint64_t m,
                                 const uint32_t* __restrict__ ex, const uint32_t* __restrict__ rstart,
                                 const uint32_t* __restrict__ nruns, uint32_t* __restrict__ cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t r = run_head(sk, i) ? ex[i] : ex[i] - 1;
    const uint32_t R = *nruns;
    const uint64_t end = (r + 1 < R) ? rstart[r + 1] : m;
    cnt[sv[i]] = (uint32_t)(end - rstart[r]);
}

// raw frequency of position j: the run length for j < m, 1 for the last L-1 positions
// ("fudge", :52-54; with an empty SML the loop starts at 1, so position 0 keeps 0),
// 1 before the sequence (smoothFrequencies' initial buffer, :75-79)
__device__ __forceinline__ uint64_t raw_freq(const uint32_t* __restrict__ cnt, int64_t j, uint64_t m) {
    if (j < 0) return 1;
    if ((uint64_t)j < m) return cnt[j];
    return (j == 0 && m == 0) ? 0 : 1;
}

// smoothFrequencies (:71-87): position p < n-1 gets the mean raw frequency of the L seeds
// ending at p, as (float)(double window sum / L) -- the reference's running double sum
// holds integers only, so the window sum is exact; p = n-1 keeps its raw value; then
// zeros become 1 (:57-59).
__global__ void occ_smooth_kernel(const uint32_t* __restrict__ cnt, uint64_t m, uint64_t n, int L,
                                  float* __restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    float v;
    if (p + 1 == n) {
        v = (float)raw_freq(cnt, (int64_t)p, m);
    } else {
        uint64_t w = 0;
        for (int k = 0; k < L; ++k) w += raw_freq(cnt, (int64_t)p - k, m);
        v = (float)((double)w / (double)L);
    }
    out[p] = (v == 0.0f) ? 1.0f : v;
}

// MatchList filters: keep[k] = 1 when match k survives
__global__ void match_keep_kernel(const uint64_t* __restrict__ len, const int64_t* __restrict__ s, uint64_t M, int G,
                                  uint32_t mult, uint64_t min_len, uint32_t* __restrict__ keep) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    bool ok = true;
    if (mult) {   // Multiplicity() = genomes with a start (NO_MATCH = 0)
        uint32_t c = 0;
        for (int g = 0; g < G; ++g) c += s[k * (uint64_t)G + g] != 0 ? 1u : 0u;
        ok = c == mult;
    }
    if (min_len && len[k] < min_len) ok = false;
    keep[k] = ok ? 1u : 0u;
}

__global__ void match_compact_kernel(const uint64_t* __restrict__ len, const int64_t* __restrict__ s, uint64_t M,
                                     int G, const uint32_t* __restrict__ keep_ex, const uint32_t* __restrict__ total,
                                     uint64_t* __restrict__ len2, int64_t* __restrict__ s2) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const uint32_t o = keep_ex[k];
    const uint32_t nxt = (k + 1 < M) ? keep_ex[k + 1] : *total;
    if (nxt == o) return;   // dropped
    len2[o] = len[k];
    for (int g = 0; g < G; ++g) s2[(uint64_t)o * G + g] = s[k * (uint64_t)G + g];
}

// 2-bit words (translate32 layout, MSB-first) -> ASCII A/C/G/T
__global__ void unpack_kernel(const uint32_t* __restrict__ W, uint64_t n, char* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = (W[i >> 4] >> (30 - 2 * (uint32_t)(i & 15))) & 3u;
    out[i] = "ACGT"[c];
}

inline dim3 grid_of(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

size_t occ_tmp_bytes(uint64_t m) { return (3 * m + 64) * 4 + scan_tmp_bytes(m); }

hipError_t launch_seed_occurrence(const uint64_t* sk, const uint32_t* sv, uint64_t m, uint64_t n, int L, void* d_tmp,
                                  float* out, hipStream_t st) {
    uint32_t* a = (uint32_t*)d_tmp;         // head flags -> exclusive scan
    uint32_t* rstart = a + m + 16;
    uint32_t* cnt = rstart + m + 16;
    uint32_t* nruns = cnt + m + 16;
    void* stmp = (void*)(nruns + 16);
    if (m) {
        hipLaunchKernelGGL(occ_heads_kernel, grid_of(m), dim3(256), 0, st, sk, m, a);
        hipError_t e = exclusive_scan_u32(a, m, stmp, nruns, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(occ_runstart_kernel, grid_of(m), dim3(256), 0, st, sk, m, a, rstart);
        hipLaunchKernelGGL(occ_count_kernel, grid_of(m), dim3(256), 0, st, sk, sv, m, a, rstart, nruns, cnt);
    }
    if (n) hipLaunchKernelGGL(occ_smooth_kernel, grid_of(n), dim3(256), 0, st, cnt, m, n, L, out);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t* words, uint64_t n, char* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_kernel, grid_of(n), dim3(256), 0, st, words, n, out);
    return hipGetLastError();
}

size_t filter_tmp_bytes(uint64_t M) { return (M + 64) * 4 + scan_tmp_bytes(M + 1); }

hipError_t launch_match_filter(const uint64_t* len, const int64_t* s, uint64_t M, int G, uint32_t mult,
                               uint64_t min_len, void* d_tmp, uint32_t* d_kept, uint64_t* len2, int64_t* s2,
                               hipStream_t st) {
    if (M == 0) return hipMemsetAsync(d_kept, 0, 4, st);
    uint32_t* keep = (uint32_t*)d_tmp;
    void* stmp = (void*)(keep + M + 64);
    hipLaunchKernelGGL(match_keep_kernel, grid_of(M), dim3(256), 0, st, len, s, M, G, mult, min_len, keep);
    hipError_t e = exclusive_scan_u32(keep, M, stmp, d_kept, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(match_compact_kernel, grid_of(M), dim3(256), 0, st, len, s, M, G, keep, d_kept, len2, s2);
    return hipGetLastError();
}

}  // namespace mums
