// Micro-benchmark / ablation harness for the segmented onesweep sort (development tool).
// Built from the library sources with -DMUMS_ABL_* switches; times seg_onesweep_sort on
// n random 8-B records (one bucket, 32 key bits = 4 passes).
#include "../libmems_amd/csrc/scan.hip"
#include "../libmems_amd/csrc/radix_seg.hip"
#include <cstdio>
#include <vector>
#include <random>
using namespace mums;
int main(int argc, char** argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 800000000ull;
    const int msd = argc > 2 ? atoi(argv[2]) : 0;   // records pre-split into 2^msd equal buckets
    const uint64_t nb = 1ull << msd;
    const bool rts = argc > 3 && argv[3][0] == 'r';  // reduce-then-scan sort; events bracket the downsweeps only
    std::vector<uint64_t> h(n);
    std::mt19937_64 r(7);
    for (uint64_t i = 0; i < n; ++i) h[i] = (r() & 0xFFFFFFFF00000000ull) | i;
    uint64_t *a, *b; SegTile* tiles; void* tmp; uint32_t *err, *nt, *bst;
    const uint64_t ub = seg_tiles_upper(n, msd);
    std::vector<uint32_t> hs(nb);
    for (uint64_t b = 0; b < nb; ++b) hs[b] = (uint32_t)(b * (n / nb));
    uint32_t* dhs; (void)hipMalloc(&dhs, nb * 4); (void)hipMemcpy(dhs, hs.data(), nb * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&a, n * 8); (void)hipMalloc(&b, n * 8);
    (void)hipMalloc(&tiles, ub * sizeof(SegTile));
    size_t tb = std::max(onesweep_tmp_bytes(n, msd, 32), seg_tmp_bytes(n, msd));
    (void)hipMalloc(&tmp, tb); (void)hipMalloc(&err, 64); (void)hipMalloc(&nt, 64); (void)hipMalloc(&bst, (nb + 1) * 4 + 64);
    (void)hipMemset(err, 0, 64);
    hipStream_t st; (void)hipStreamCreate(&st);
    (void)build_seg_tiles(msd ? dhs : nullptr, 1, msd, n, tiles, nt, bst, tmp, st);
    hipEvent_t ev[10]; for (auto& e : ev) (void)hipEventCreate(&e);
    int buf;
    float tot[4] = {0, 0, 0, 0}, whole = 0;
    const int K = 5;
    for (int it = 0; it < K + 1; ++it) {
        (void)hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(ev[8], st);
        if (rts) (void)seg_radix_sort(a, b, n, 32, tiles, ub, tmp, &buf, st, ev);
        else (void)seg_onesweep_sort(a, b, n, 32, msd, tiles, ub, bst, tmp, err, &buf, st, ev);
        (void)hipEventRecord(ev[9], st);
        (void)hipStreamSynchronize(st);
        if (it == 0) continue;
        { float ms; (void)hipEventElapsedTime(&ms, ev[8], ev[9]); whole += ms; }
        for (int p = 0; p < 4; ++p) { float ms; (void)hipEventElapsedTime(&ms, ev[2 * p], ev[2 * p + 1]); tot[p] += ms; }
    }
    uint32_t e; (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    // check sortedness of the final output (not meaningful under ablation)
    std::vector<uint64_t> o(n); (void)hipMemcpy(o.data(), buf ? b : a, n * 8, hipMemcpyDeviceToHost);
    uint64_t bad = 0, lost = 0;
    const uint64_t bs = n / nb;
    for (uint64_t i = 1; i < n; ++i) bad += (i % bs != 0 || i >= nb * bs) && (o[i] >> 32) < (o[i - 1] >> 32);
    std::vector<uint8_t> seen(n, 0);
    for (uint64_t i = 0; i < n; ++i) { const uint32_t j = (uint32_t)o[i]; lost += seen[j]; seen[j] = 1; }
    printf("%s%s whole=%.3f ms n=%lu msd=%d per-pass ms: %.3f %.3f %.3f %.3f  (avg %.3f, %.0f GB/s) err=%u unsorted=%lu dup=%lu\n", TAG, rts ? "-rts" : "", whole / K, (unsigned long)n, msd,
           tot[0] / K, tot[1] / K, tot[2] / K, tot[3] / K, (tot[0] + tot[1] + tot[2] + tot[3]) / 4 / K,
           n * 16.0 / ((tot[0] + tot[1] + tot[2] + tot[3]) / 4 / K) / 1e6, e, (unsigned long)bad, (unsigned long)lost);
    return 0;
}
