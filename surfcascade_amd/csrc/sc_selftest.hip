// sc_selftest.hip -- exhaustive device check of the shortened IEEE sequences
// the item loop uses in Normalize (DenseSURFFeatureExtractor.cpp:427-457):
// sqrt_rn (for sqrt(SS), sqrt(SS2)) and rcp_rn (for 1/sqrt(SS2)),
// sc_device.hpp.  Every f32 bit pattern of a range is run through the short
// sequence, the compiler's full IEEE sequence (sqrtf, 1.0f / d) and the f64
// route ((float)sqrt((double)x), (float)(1.0 / (double)d): correctly rounded
// f32 results, since 53 >= 2*24 + 2 makes the double rounding innocuous), and
// the bit differences are counted.  sc_selftest_rn (C ABI) launches it.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sc_device.hpp"

namespace sc {

namespace {

// out[0]: patterns where the short sequence differs from the full one,
// out[1]: ... from the f64 route, out[2]: patterns checked, out[3]: the
// smallest differing pattern (UINT64_MAX: none)
__global__ __launch_bounds__(256) void rn_check_kernel(int op, uint32_t lo, uint32_t hi,
                                                      unsigned long long *out) {
    const unsigned long long n = (unsigned long long)hi - lo + 1ull;
    const unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
    unsigned long long bad_full = 0, bad_f64 = 0, first = ~0ull, done = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += nthreads) {
        const uint32_t u = lo + (uint32_t)i;
        const float x = __uint_as_float(u);
        float s, full, ref;
        if (op == 0) {
            s = sqrt_rn(x);
            full = sqrtf(x);
            ref = (float)sqrt((double)x);
        } else {
            s = rcp_rn(x);
            full = 1.0f / x;
            ref = (float)(1.0 / (double)x);
        }
        const bool b1 = __float_as_uint(s) != __float_as_uint(full);
        const bool b2 = __float_as_uint(s) != __float_as_uint(ref);
        bad_full += b1;
        bad_f64 += b2;
        if ((b1 || b2) && u < first) first = u;
        done++;
    }
    // wave sums, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        bad_full += __shfl_xor(bad_full, o, 64);
        bad_f64 += __shfl_xor(bad_f64, o, 64);
        done += __shfl_xor(done, o, 64);
        const unsigned long long f2 = __shfl_xor(first, o, 64);
        first = f2 < first ? f2 : first;
    }
    if ((threadIdx.x & 63) == 0) {
        if (bad_full) atomicAdd(&out[0], bad_full);
        if (bad_f64) atomicAdd(&out[1], bad_f64);
        atomicAdd(&out[2], done);
        if (first != ~0ull) atomicMin(&out[3], first);
    }
}

}  // namespace

void launch_rn_check(int op, uint32_t lo, uint32_t hi, unsigned long long *out, int cus, hipStream_t s) {
    const int grid = (cus > 0 ? cus : 256) * 32;
    hipLaunchKernelGGL(rn_check_kernel, dim3(grid), dim3(256), 0, s, op, lo, hi, out);
}

}  // namespace sc
