// chunked.hip -- helpers of the chunked mode for more than 2^32 seed-mers per context
// (BASELINE config 5, 2 x 3 Gbp; SURVEY.md 8(e) "chunked SML over 288 GB HBM").
//
// The packed records carry 33-bit global indices (RecViewT<33>): with 2w+1 = 39 key bits
// the top 8 are the MSD digit (implicit in the record's bucket), 31 sit in the record.
// The MSD digits are cut into power-of-two chunks of < 2^30 records; every chunk is
// scattered (seed_scatter_kernel<.., 33, true>), sorted (onesweep, key bits from 33),
// grouped and probed on its own, in key order, so 32-bit stream offsets suffice inside a
// chunk and the probes come out in the reference's AddHashEntry order.
#include <hip/hip_runtime.h>

#include "mums_internal.h"

namespace mums {
namespace {

// out[r] = sum of hist[r * T .. r * T + T) (records of MSD digit r)
__global__ __launch_bounds__(256) void digit_totals_kernel(const uint32_t* __restrict__ hist, uint32_t T,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s[256];
    const uint32_t r = blockIdx.x;
    unsigned long long acc = 0;
    for (uint32_t t = threadIdx.x; t < T; t += 256) acc += hist[(uint64_t)r * T + t];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[r] = s[0];
}

}  // namespace

hipError_t launch_digit_totals(const uint32_t* hist, uint32_t ndigits, uint32_t T, unsigned long long* out,
                               hipStream_t st) {
    if (ndigits == 0) return hipSuccess;
    hipLaunchKernelGGL(digit_totals_kernel, dim3(ndigits), dim3(256), 0, st, hist, T, out);
    return hipGetLastError();
}

}  // namespace mums
