// Development harness: MSD pass (kBits-wide digit) + LDS local sort of the resulting
// sub-buckets on n random records pre-split into 2^msd equal buckets (the seed
// scatter's output shape).  Checks final order (key, then index) inside every bucket.
#include "../libmems_amd/csrc/scan.hip"
#include "../libmems_amd/csrc/radix_seg.hip"
#include "proto/msd_pass.hip"
#include "proto/local_sort.hip"
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
using namespace mums;
int main(int argc, char** argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 800000000ull;
    const int msd = argc > 2 ? atoi(argv[2]) : 8;
    const int kb = argc > 3 ? atoi(argv[3]) : 9;
    const int skew = argc > 4 ? atoi(argv[4]) : 1;   // 1: canonical-key skew (density 2(1-x))
    const uint64_t nb = 1ull << msd;
    std::mt19937_64 r(7);
    // bucket sizes: equal, or proportional to 2(1-x) (min of two uniforms) as canonical keys
    std::vector<uint64_t> bs(nb);
    uint64_t tot = 0;
    for (uint64_t b = 0; b < nb; ++b) {
        double w = skew ? 2.0 * (1.0 - (b + 0.5) / nb) : 1.0;
        bs[b] = (uint64_t)(w * n / nb);
        tot += bs[b];
    }
    n = tot;
    std::vector<uint64_t> h(n);
    std::vector<uint32_t> hs(nb + 1);
    uint64_t o = 0;
    for (uint64_t b = 0; b < nb; ++b) {
        hs[b] = (uint32_t)o;
        for (uint64_t i = 0; i < bs[b]; ++i, ++o) h[o] = (r() & 0xFFFFFFFF00000000ull) | o;
    }
    hs[nb] = (uint32_t)n;
    uint64_t *a, *b2; SegTile* tiles; void* tmp; uint32_t *err, *nt, *bst, *dbase;
    const uint64_t ub = seg_tiles_upper(n, msd);
    (void)hipMalloc(&a, n * 8); (void)hipMalloc(&b2, n * 8);
    (void)hipMalloc(&tiles, ub * sizeof(SegTile));
    size_t tb = std::max(msd_pass_tmp_bytes(n, msd, kb), seg_tmp_bytes(n, msd));
    (void)hipMalloc(&tmp, tb); (void)hipMalloc(&err, 64); (void)hipMalloc(&nt, 64);
    (void)hipMalloc(&bst, (nb + 1) * 4 + 64); (void)hipMalloc(&dbase, (nb << kb) * 4 + 64);
    (void)hipMemset(err, 0, 64);
    (void)hipMemcpy(bst, hs.data(), (nb + 1) * 4, hipMemcpyHostToDevice);
    hipStream_t st; (void)hipStreamCreate(&st);
    (void)build_seg_tiles_from_starts(bst, msd, n, tiles, nt, tmp, st);
    hipEvent_t e0, e1, e2; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&e2);
    const int shift = 64 - kb;
    const uint64_t nsub = nb << kb;
    std::vector<uint32_t> db(nsub);
    std::vector<uint64_t> rg;
    uint64_t* drg = nullptr;
    float tm = 0, tl = 0; const int K = 5;
    uint32_t mx = 0;
    for (int it = 0; it <= K; ++it) {
        (void)hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, st);
        (void)msd_pass(a, b2, n, shift, msd, kb, tiles, ub, bst, tmp, err, dbase, st);
        (void)hipEventRecord(e1, st);
        if (it == 0) {
            (void)hipStreamSynchronize(st);
            (void)hipMemcpy(db.data(), dbase, nsub * 4, hipMemcpyDeviceToHost);
            for (uint64_t s = 0; s < nsub; ++s) {
                const uint64_t s0 = db[s], s1 = (s + 1 < nsub) ? db[s + 1] : n;
                if (s1 > s0) { rg.push_back(s0 | ((s1 - s0) << 40)); mx = std::max<uint32_t>(mx, (uint32_t)(s1 - s0)); }
            }
            (void)hipMalloc(&drg, rg.size() * 8);
            (void)hipMemcpy(drg, rg.data(), rg.size() * 8, hipMemcpyHostToDevice);
        }
        const int kbits = 32 - kb;
        if (mx <= 4096) hipLaunchKernelGGL(local_sort_kernel<256>, dim3((unsigned)rg.size()), dim3(256), 0, st, b2, a, drg, (uint32_t)rg.size(), kbits);
        else if (mx <= 8192) hipLaunchKernelGGL(local_sort_kernel<512>, dim3((unsigned)rg.size()), dim3(512), 0, st, b2, a, drg, (uint32_t)rg.size(), kbits);
        else hipLaunchKernelGGL(local_sort_kernel<1024>, dim3((unsigned)rg.size()), dim3(1024), 0, st, b2, a, drg, (uint32_t)rg.size(), kbits);
        (void)hipEventRecord(e2, st);
        (void)hipStreamSynchronize(st);
        if (it) { float x; (void)hipEventElapsedTime(&x, e0, e1); tm += x; (void)hipEventElapsedTime(&x, e1, e2); tl += x; }
    }
    uint32_t ev; (void)hipMemcpy(&ev, err, 4, hipMemcpyDeviceToHost);
    std::vector<uint64_t> out(n); (void)hipMemcpy(out.data(), a, n * 8, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t b = 0; b < nb; ++b)
        for (uint64_t i = (uint64_t)hs[b] + 1; i < hs[b + 1]; ++i) {
            const uint64_t k1 = out[i - 1] >> 32, k2 = out[i] >> 32;
            bad += (k2 < k1) || (k2 == k1 && (uint32_t)out[i] < (uint32_t)out[i - 1]);
        }
    printf("msd=%d kb=%d skew=%d n=%lu: msd pass %.3f ms, local sort %.3f ms (ranges %zu, max %u), total %.3f ms, err=%u bad=%lu\n",
           msd, kb, skew, (unsigned long)n, tm / K, tl / K, rg.size(), mx, (tm + tl) / K, ev, (unsigned long)bad);
    return 0;
}
